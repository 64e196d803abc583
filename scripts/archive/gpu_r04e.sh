# Round 4: side work interleaved with the next encoder's FFN2 (tests + A/B), then the residual-prefetch library A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_cli_gpu.py tests/test_api_gpu.py tests/test_canary_gpu.py tests/test_varlen_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python scripts/pipe_ab.py --variants base,serialside,gatestart,fill1,serialsidefill1 --rounds 3 --steps 20 --encoder-only > $O/ab.txt 2>&1 || { echo "AB FAIL"; tail -20 $O/ab.txt; exit 1; }
tail -5 $O/ab.txt
timeout -k 10 300 python scripts/layer_gemm_bench.py --cfgs 0,25,26,23,24,17,0 > $O/tiles.txt 2>&1 || { echo "TILES FAIL"; tail -5 $O/tiles.txt; exit 1; }
grep cfg $O/tiles.txt
OUT=$O/libs REPS=2 bash scripts/gpu_ab_libs.sh
