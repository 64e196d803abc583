# Round 6: (1) the host-thread probe with stack scans under HIP/HSA runtime knobs; (2) the side-stream cost
# decomposition (scripts/side_cost.py: kernel trace of the side pass alone -> occupancy replay; zero-operand and
# replay arms beside the encoder).  Outputs under gpurun_out/r06b.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
i=0
for e in "" "ROC_ACTIVE_WAIT_TIMEOUT=0" "ROC_CPU_WAIT_FOR_SIGNAL=0" "AMD_DIRECT_DISPATCH=0"; do
  i=$((i+1))
  timeout -k 10 200 python scripts/host_thread_probe.py --steps 40 ${e:+--env $e} > $O/threads_$i.json 2> $O/threads_$i.err || { echo "PROBE $e FAIL"; tail -20 $O/threads_$i.err; exit 1; }
  head -c 300 $O/threads_$i.json; echo
done
rm -rf $O/sidetrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sidetrace -o run -- python3 scripts/side_cost.py --mode trace > $O/sidetrace.log 2>&1 || { echo "SIDE TRACE FAIL"; tail -20 $O/sidetrace.log; exit 1; }
python scripts/side_cost.py --mode build --trace $O/sidetrace --out $O/side_replay.json > $O/side_replay.txt 2>&1 || { echo "BUILD FAIL"; cat $O/side_replay.txt; exit 1; }
cat $O/side_replay.txt
rm -rf $O/sidetrace
timeout -k 10 400 python scripts/side_cost.py --mode ab --replay $O/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
cat $O/side_ab.txt
echo ALLOK
