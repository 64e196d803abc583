# Round 6: which HIP operation keeps the HSA async-events thread spinning (micro patterns), and the side-stream
# decomposition with the occupancy replay fixed (one deadline per grid).  Outputs under gpurun_out/r06c.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 200 python scripts/host_thread_micro.py > $O/micro.txt 2> $O/micro.err || { echo "MICRO FAIL"; tail -20 $O/micro.err; exit 1; }
cat $O/micro.txt | head -8
timeout -k 10 400 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
cat $O/side_ab.txt
echo ALLOK
