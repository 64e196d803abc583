# Round 4: the one-round 192x256 tile rule (tests + interleaved library A/B against the 256x256 rule).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_split_gpu.py tests/test_pipeline_gpu.py tests/test_cli_gpu.py tests/test_api_gpu.py tests/test_varlen_gpu.py tests/test_reference10s_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/libs REPS=3 bash scripts/gpu_ab_libs.sh
