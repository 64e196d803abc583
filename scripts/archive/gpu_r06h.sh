# Round 6: side-stream decomposition (fixed occupancy replay), the 8-rank rehearsal test, the pipelined-submit
# bit-identity test, and the CLI over a 1 024-file synthetic corpus (infer.py --metrics).  Outputs: gpurun_out/r06h.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 120 python scripts/side_cost.py --mode calib > $O/calib.txt 2>&1 || { echo "CALIB FAIL"; tail -20 $O/calib.txt; exit 1; }
grep -v amdgpu.ids $O/calib.txt
timeout -k 10 400 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt
timeout -k 10 700 python -u -m pytest tests/test_cli_gpu.py tests/test_pipeline_gpu.py -q --timeout 600 --timeout-method thread -k "eight_ranks or submit_matches" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python scripts/cli_bench.py --n 1024 --batch 32 --reps 2 --seconds 10 10 --metrics $O/cli_metrics_10s.jsonl > $O/cli_10s.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli_10s.txt; exit 1; }
grep "^run" $O/cli_10s.txt
timeout -k 10 600 python scripts/cli_bench.py --n 1024 --batch 32 --reps 2 --metrics $O/cli_metrics_8_12s.jsonl > $O/cli_8_12s.txt 2>&1 || { echo "CLI2 FAIL"; tail -20 $O/cli_8_12s.txt; exit 1; }
grep "^run" $O/cli_8_12s.txt
echo ALLOK
