# Round 6: does the stream-order word order and publish? (the new tests alone, then the held-DP test under each sync)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -q --timeout 200 --timeout-method thread -k "stream_order or matches_align_batch" > $O/tests.log 2>&1; echo "rc $?"; grep -E "passed|failed|Error|assert" $O/tests.log | head -20
echo ALLOK
