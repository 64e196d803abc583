# New large-grid tile rule + DP LDS reservation: parity (split GEMM, varlen bit-identity, pipeline, DP), then
# config 2 / config 5 (20 s windows) on the old build (dpold) and the new one with HFA_DP_RESERVE_KB 0 / 112.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gpu.py tests/test_varlen_gpu.py tests/test_pipeline_gpu.py tests/test_viterbi_gpu.py > gpurun_out/ab_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -n 2 gpurun_out/ab_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" $1 "$2"; }
for rep in 1 2; do
for v in old new0 new112; do
  case $v in old) export HFA_LIB=$PWD/hubertfa_amd/_build_ab/dpold/libhfa.so; unset HFA_DP_RESERVE_KB;;
             new0) unset HFA_LIB; export HFA_DP_RESERVE_KB=0;; new112) unset HFA_LIB; export HFA_DP_RESERVE_KB=112;; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c2.json 2> gpurun_out/ab_c2.err || { echo "C2 FAIL"; tail gpurun_out/ab_c2.err; exit 1; }
  show gpurun_out/ab_c2.json "c2 $v"
  timeout -k 10 300 python bench.py --batch 1 --seconds 300 --words 600 --steps 6 --warmup 2 --no-cpu-baseline --chunk-seconds 20 > gpurun_out/ab_c5.json 2> gpurun_out/ab_c5.err || { echo "C5 FAIL"; tail gpurun_out/ab_c5.err; exit 1; }
  show gpurun_out/ab_c5.json "c5c $v"
done; done
