# Round 5: paired side passes (task.pair_batches) -- the parity test, then an interleaved A/B of the bench step
# (--pair off / on) on one box, with the side stream's cost from step_breakdown.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_pair
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 240 --timeout-method thread -k "paired or smoke" > $O/tests.log 2>&1 || { echo "PAIR TEST FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for mode in off on on-dp1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-extra-configs --pair $mode > $O/b_$mode$rep.json 2> $O/b_$mode$rep.err || { echo "BENCH FAIL $mode"; tail -5 $O/b_$mode$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$mode$rep.json').read().strip().splitlines()[-1]); s=d['step_breakdown']; print('$mode', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'enc', round(s['encoder_only_ms'],3), 'side', round(s['side_stream_cost_ms'],3))"
  done
done
echo ALLOK
