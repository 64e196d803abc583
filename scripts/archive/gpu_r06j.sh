# Round 6: the 16x16x32 attention's 8-wave schedules (stagger / priority): bit identity, then the microbenchmark.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention" > $O/attn_tests.log 2>&1 || { echo "ATTN TESTS FAIL"; tail -40 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
timeout -k 10 300 python scripts/attn_bench.py --reps 20 --rounds 3 > $O/attn_bench.txt 2>&1 || { echo "ATTN BENCH FAIL"; tail -20 $O/attn_bench.txt; exit 1; }
grep -v amdgpu.ids $O/attn_bench.txt
echo ALLOK
