# Round 6: side-stream decomposition with grid-capped occupancy replays (does the side pass's workgroup count --
# 74 000 per pass, 60 000 of them in small elementwise / norm kernels -- cost the encoder?).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 500 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt
echo ALLOK
