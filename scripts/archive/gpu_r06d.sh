# Round 6: sleeper calibration; the async-events thread under stream memory operations (wait/write value) with and
# without GPU_STREAMOPS_CP_WAIT.  Outputs under gpurun_out/r06d.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 120 python scripts/side_cost.py --mode calib > $O/calib.txt 2>&1 || { echo "CALIB FAIL"; tail -20 $O/calib.txt; exit 1; }
cat $O/calib.txt
timeout -k 10 120 python scripts/host_thread_micro.py --only idle,side_wait_event,wait_value32 > $O/micro_a.txt 2> $O/micro_a.err || { echo "MICRO A FAIL"; tail -20 $O/micro_a.err; exit 1; }
head -3 $O/micro_a.txt
timeout -k 10 120 python scripts/host_thread_micro.py --only idle,side_wait_event,wait_value32 --env GPU_STREAMOPS_CP_WAIT=1 > $O/micro_b.txt 2> $O/micro_b.err || { echo "MICRO B FAIL"; tail -20 $O/micro_b.err; exit 1; }
head -3 $O/micro_b.txt
echo ALLOK
