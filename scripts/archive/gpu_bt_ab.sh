# Backtrack rework: DP/backtrack parity, then the DP microbenchmark and config 5 on old vs new libhfa.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_viterbi_gpu.py tests/test_longform_gpu.py tests/test_reference10s_gpu.py tests/test_pipeline_gpu.py > gpurun_out/dp_tests.log 2>&1 || { echo "DP TESTS FAIL"; tail -40 gpurun_out/dp_tests.log; exit 1; }
tail -n 2 gpurun_out/dp_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), [(s['kernel'], round(s.get('avg_launch_ms') or 0, 3)) for s in d.get('secondary', [])])" $1 $2; }
for n in old new; do
  if [ $n = old ]; then export HFA_LIB=$PWD/hubertfa_amd/_build_ab/dpold/libhfa.so; else unset HFA_LIB; fi
  echo "== $n"; timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep -v amdgpu.ids || { echo "BENCH FAIL"; exit 1; }
  timeout -k 10 300 python bench.py --batch 1 --seconds 300 --words 600 --steps 4 --warmup 1 --no-cpu-baseline --chunk-seconds 20 > gpurun_out/c5c_$n.json 2> gpurun_out/c5c_$n.err || { echo "C5C FAIL"; tail gpurun_out/c5c_$n.err; exit 1; }
  show gpurun_out/c5c_$n.json "c5-chunked $n"
  timeout -k 10 300 python bench.py --batch 1 --seconds 300 --words 600 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$n.json 2> gpurun_out/c5_$n.err || { echo "C5 FAIL"; tail gpurun_out/c5_$n.err; exit 1; }
  show gpurun_out/c5_$n.json "c5 $n"
done
