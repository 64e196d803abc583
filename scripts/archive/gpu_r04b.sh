# Round 4, second box: tests of the DP-init fold / flag snapshot / kernel-name query, then per-shape traces of the
# pipelined step and of the encoder alone (the side stream's per-kernel cost).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_viterbi_gpu.py tests/test_pipeline_gpu.py tests/test_api_gpu.py tests/test_cli_gpu.py tests/test_reference10s_gpu.py tests/test_longform_gpu.py -x -q -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in pipe encoder; do
  rm -rf $O/tr_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$m -o run -- python3 scripts/shape_trace.py --mode $m --steps 8 --warmup 3 --log $O/tr_$m/launch_log.json > $O/tr_$m.log 2>&1 || { echo "TRACE $m FAIL"; tail -20 $O/tr_$m.log; exit 1; }
  python scripts/shape_table.py --trace $O/tr_$m --log $O/tr_$m/launch_log.json --csv $O/shape_$m.csv > $O/shape_$m.txt 2>&1 || { echo "TABLE $m FAIL"; cat $O/shape_$m.txt; }
done
head -14 $O/shape_pipe.txt
head -14 $O/shape_encoder.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 300 python bench.py --batch 1 --seconds 300 --words 600 --chunk-seconds 20 --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_c5c.json 2> $O/bench_c5c.err || { echo "BENCH C5C FAIL"; tail -20 $O/bench_c5c.err; exit 1; }
tail -c 900 $O/bench_c5c.json
echo ALLOK
