# Round 4: host CPU of the step with the poll-and-sleep wait in AlignmentDecoder.assemble (was a spinning HIP event
# wait), plus the tests that run the pipelined assemble path.  OUT=gpurun_out/r04i.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_pipeline_gpu.py tests/test_api_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_cpu'], d['step_breakdown']['side_stream_cost_ms'])"
echo ALLOK
