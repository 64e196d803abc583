# held long-lattice DP (task.submit gates its step ranges at the next encoder's attention launches): parity tests, then
# config 5 (300 s, one utterance) held vs --no-held-dp, interleaved, 10 steps; config 2 once each (not held: T < 8192)
set -o pipefail
O=gpurun_out/held_dp; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_viterbi_gpu.py tests/test_pipeline_gpu.py tests/test_longform_gpu.py tests/test_split_gpu.py tests/test_configs_gpu.py > $O/tests.txt 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); b=d.get('step_breakdown',{}); h=d.get('host_cpu',{}); print('$tag', round(d['value'],1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in b.items() if isinstance(v,float)}, 'enqueue', round(h.get('enqueue_wall_ms_per_step',0),2), 'wait+asm', round(h.get('wait_assemble_wall_ms_per_step',0),2))"
}
C5="--batch 1 --seconds 300 --words 600 --steps 10 --warmup 2"
run c5_held1 $C5 && run c5_whole1 $C5 --no-held-dp && run c5_held2 $C5 && run c5_whole2 $C5 --no-held-dp && \
run c5c_held --batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --chunk-seconds 20 && \
run c5c_whole --batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --chunk-seconds 20 --no-held-dp && \
run c2_a --steps 20 --warmup 3 && run c2_b --steps 20 --warmup 3 --no-held-dp && echo ALLOK
