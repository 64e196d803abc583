# Round 6: the one-pass 16 k -> 44.1 k -> 16 k chain (resample.ChainResampler): its tests, the GPU suite, an
# interleaved A/B against the two stages (bench --two-stage-resample), and the kernel stats of the chain build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "chain or resample" -x -q --timeout 200 --timeout-method thread > $O/chain_tests.log 2>&1 || { echo "CHAIN TESTS FAIL"; tail -40 $O/chain_tests.log; exit 1; }
tail -2 $O/chain_tests.log
if [ -z "$QUICK" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
fi
tail -2 $O/gputests.log
for r in 1 2 3; do
  for arm in chain two; do
    F=""; [ $arm = two ] && F="--two-stage-resample"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 $F > $O/bench_${arm}_$r.json 2> $O/bench_${arm}_$r.err || { echo "BENCH $arm FAIL"; tail -20 $O/bench_${arm}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm', $r, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3))"
  done
done
timeout -k 10 300 python scripts/resample_tiles.py > $O/resample_tiles.txt 2>&1 || { echo "TILES FAIL"; tail -20 $O/resample_tiles.txt; exit 1; }
cat $O/resample_tiles.txt
rm -rf $O/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --sustained-s 0 > $O/stats.log 2>&1 || { echo "STATS FAIL"; tail -5 $O/stats.log; exit 1; }
find $O/stats -name "*kernel_stats.csv" -exec head -40 {} \; > $O/kernel_stats_top.csv
grep -i "pad_split\|chain_edges\|128, 192\|128, 128\|64, 192\|192, 128" $O/kernel_stats_top.csv | cut -c1-200
echo ALLOK
