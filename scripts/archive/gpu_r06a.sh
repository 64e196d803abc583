# Round 6, first box: the bench line with the new sustained block and the per-stage CPU baseline; the host-thread
# probe under the four HIP device schedules; the 8-rank rehearsal (gloo, all ranks on GPU 0, config-3 block at 64 per
# rank).  Outputs under gpurun_out/r06a.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
for f in default blocking yield spin; do
  timeout -k 10 200 python scripts/host_thread_probe.py --device-flags $f --steps 40 > $O/threads_$f.json 2> $O/threads_$f.err || { echo "PROBE $f FAIL"; tail -20 $O/threads_$f.err; exit 1; }
  head -c 400 $O/threads_$f.json; echo
done
S=$(date +%s)
timeout -k 10 600 python bench.py --gpus 8 --device 0 --dist-backend gloo --batch 4 --seconds 10 --steps 3 --warmup 1 --no-cpu-baseline > $O/rehearsal8.json 2> $O/rehearsal8.err || { echo "REHEARSAL FAIL"; tail -30 $O/rehearsal8.err; exit 1; }
echo "rehearsal wall $(( $(date +%s) - S )) s"
head -c 800 $O/rehearsal8.json
echo ALLOK
