# Round 4: 512-row window positional conv (tests + interleaved library A/B against the 256-row tiles).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_split_gpu.py tests/test_encoder_gpu.py tests/test_reference10s_gpu.py tests/test_varlen_gpu.py tests/test_longform_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/libs REPS=3 MICRO="python scripts/posconv_bench.py" bash scripts/gpu_ab_libs.sh
