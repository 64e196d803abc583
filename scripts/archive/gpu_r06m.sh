# Round 6: side-stream A/B with replay arms capping only the GEMM / GroupNorm grids (what a persistent UNet GEMM
# would hold beside the encoder).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
true

timeout -k 10 500 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt


echo ALLOK
