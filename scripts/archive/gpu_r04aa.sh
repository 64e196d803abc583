# CLI loop with held long-file DPs (test) + a kernel trace of config 5 with the held DP (where the DP ranges run)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cli_gpu.py tests/test_pipeline_gpu.py -k "held or repeatable" > $O/tests.txt 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
rm -rf $O/c5trace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c5trace -o run -- python3 bench.py --batch 1 --seconds 300 --words 600 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5trace.log 2>&1 || { echo "TRACE FAIL"; tail -20 $O/c5trace.log; exit 1; }
echo ALLOK
