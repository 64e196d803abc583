# Round 4: the UNet's 192/384-channel convs on the 128x192 tile (candidate library in hubertfa_amd/_build_ab)
# against the shipped 128x128 choice: parity of the candidate (UNet head golden, split GEMM tiles, varlen), then
# the UNet microbenchmark and the pipelined bench step interleaved.  OUT=gpurun_out/r04j.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
HFA_LIB=$ALT timeout -k 10 600 python -u -m pytest tests/test_encoder_gpu.py tests/test_varlen_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -k "unet or varlen or single_acc or linear" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/libs REPS=3 MICRO="python scripts/unet_bench.py --tiles 0,18,25" bash scripts/gpu_ab_libs.sh
