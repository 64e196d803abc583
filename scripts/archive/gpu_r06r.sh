# Round 6: the features' gather writing the head's split planes (no conversion pass on the side stream): its test,
# the GPU suite, and an interleaved A/B against the head converting them (bench --no-gather-planes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -k "gather_planes" -x -q --timeout 200 --timeout-method thread > $O/planes_tests.log 2>&1 || { echo "PLANES TESTS FAIL"; tail -40 $O/planes_tests.log; exit 1; }
tail -2 $O/planes_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
for r in 1 2 3; do
  for arm in planes conv; do
    F=""; [ $arm = conv ] && F="--no-gather-planes"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 $F > $O/bench_${arm}_$r.json 2> $O/bench_${arm}_$r.err || { echo "BENCH $arm FAIL"; tail -20 $O/bench_${arm}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm', $r, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3), d['step_breakdown']['side_stream_cost_ms'] if 'step_breakdown' in d else '')"
  done
done
echo ALLOK
