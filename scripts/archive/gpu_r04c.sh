# Round 4: residual prefetch in the split GEMM's f32 epilogue (tests + per-shape trace) and the side-stream
# scheduling A/B (LDS-filling one-round GEMM grids, CU-masked side stream).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_encoder_gpu.py tests/test_reference10s_gpu.py tests/test_canary_gpu.py tests/test_varlen_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
rm -rf $O/tr_pipe
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_pipe -o run -- python3 scripts/shape_trace.py --mode pipe --steps 8 --warmup 3 --log $O/tr_pipe/launch_log.json > $O/tr_pipe.log 2>&1 || { echo "TRACE FAIL"; tail -20 $O/tr_pipe.log; exit 1; }
python scripts/shape_table.py --trace $O/tr_pipe --log $O/tr_pipe/launch_log.json --csv $O/shape_pipe.csv > $O/shape_pipe.txt 2>&1 || { echo "TABLE FAIL"; cat $O/shape_pipe.txt; }
head -9 $O/shape_pipe.txt
timeout -k 10 600 python scripts/pipe_ab.py --variants base,fill1,fill2,mask64,mask64fill1,mask32 --rounds 3 --steps 20 --encoder-only > $O/ab.txt 2>&1 || { echo "AB FAIL"; tail -20 $O/ab.txt; exit 1; }
tail -7 $O/ab.txt
echo ALLOK
