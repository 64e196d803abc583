set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_ln_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "FUSED LN TEST FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/ln_fuse_bench.py > $O/micro.txt 2>&1 || { echo "MICRO FAIL"; tail -5 $O/micro.txt; exit 1; }
grep -v amdgpu.ids $O/micro.txt
for rep in 1 2; do
  for mode in two one; do
    f=""; [ $mode = two ] && f="--no-fuse-ln"
    timeout -k 10 300 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-extra-configs $f > $O/b_$mode$rep.json 2> $O/b_$mode$rep.err || { echo "BENCH FAIL $mode"; tail -5 $O/b_$mode$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$mode$rep.json').read().strip().splitlines()[-1]); s=d['step_breakdown']; print('$mode', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'enc', round(s['encoder_only_ms'],3), 'side', round(s['side_stream_cost_ms'],3))"
  done
done
echo ALLOK
