# Round 6: the CLI with its batches assembled by batch_results and a leaner export: the CLI tests, then 1 024 synthetic 10 s files and
# 1 024 files of 8-12 s (infer.py --metrics), three runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_config1_gpu.py -x -q --timeout 300 --timeout-method thread > $O/cli_tests.log 2>&1 || { echo "CLI TESTS FAIL"; tail -40 $O/cli_tests.log; exit 1; }
tail -1 $O/cli_tests.log
rm -f $O/cli_metrics_10s.jsonl $O/cli_metrics_8_12s.jsonl
timeout -k 10 400 python scripts/cli_bench.py --n 1024 --seconds 10 10 --reps 3 --metrics $O/cli_metrics_10s.jsonl > $O/cli_10s.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli_10s.txt; exit 1; }
grep -v amdgpu.ids $O/cli_10s.txt | tail -3
timeout -k 10 400 python scripts/cli_bench.py --n 1024 --reps 3 --metrics $O/cli_metrics_8_12s.jsonl > $O/cli_8_12s.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli_8_12s.txt; exit 1; }
grep -v amdgpu.ids $O/cli_8_12s.txt | tail -3
python -c "import json; [print(f, round(json.loads(l)['rtf_inv_align'])) for f in ('$O/cli_metrics_10s.jsonl','$O/cli_metrics_8_12s.jsonl') for l in open(f)]"
echo ALLOK
