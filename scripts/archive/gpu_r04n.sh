# Round 4: the side-work interleave again, now with the host assembling two batches behind (depth 2), against the
# shipped schedule (serial side stream, depth 1).  Tests of the pipelined path first (interleave off = shipped).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_cli_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python scripts/pipe_ab.py --variants serial1,inter1,inter2,serial2,interstart2 --rounds 3 --steps 20 > $O/ab.txt 2>&1 || { echo "AB FAIL"; tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
echo ALLOK
