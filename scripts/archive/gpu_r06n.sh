# Round 6: the persistent UNet GEMM tiles under the side pass's tile cap (GEMM body refactored into a tile function):
# the split GEMM / attention / cap tests, then an interleaved A/B of the working library (cur) against the previous
# commit's (alt: row caps only) -- layer GEMM microbenchmark + bench step -- and the side-cost arms.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_split_gpu.py tests/test_pipeline_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OUT=$O REPS=3 bash scripts/gpu_ab_libs.sh > $O/ab.txt 2>&1 || { echo "AB FAIL"; tail -30 $O/ab.txt; exit 1; }
grep -E "^(cur|alt) " $O/ab.txt
timeout -k 10 500 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt
echo ALLOK
