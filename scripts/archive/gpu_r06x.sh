# Round 6: the CLI's per-batch timeline (HFA_CLI_TRACE: submit / loaded / submitted / settle / assembled / exported
# times of the launching thread) with the loaded program frozen out of the cyclic collector (gc.freeze), 1 024
# synthetic 10 s files, three runs (and 8-12 s files); the CLI tests; the bench's collector pauses in its timed region.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
rm -f $O/cli_trace.jsonl $O/cli_metrics_10s.jsonl $O/cli_metrics_8_12s.jsonl
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_config1_gpu.py -x -q --timeout 300 --timeout-method thread > $O/cli_tests.log 2>&1 || { echo "CLI TESTS FAIL"; tail -40 $O/cli_tests.log; exit 1; }
tail -1 $O/cli_tests.log
HFA_CLI_TRACE=$PWD/$O/cli_trace.jsonl timeout -k 10 400 python scripts/cli_bench.py --n 1024 --seconds 10 10 --reps 3 --metrics $O/cli_metrics_10s.jsonl > $O/cli.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli.txt; exit 1; }
grep -v amdgpu.ids $O/cli.txt | tail -3
timeout -k 10 400 python scripts/cli_bench.py --n 1024 --reps 3 --metrics $O/cli_metrics_8_12s.jsonl > $O/cli_8_12s.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli_8_12s.txt; exit 1; }
python -c "import json; [print(f, round(json.loads(l)['rtf_inv_align'])) for f in ('$O/cli_metrics_10s.jsonl','$O/cli_metrics_8_12s.jsonl') for l in open(f)]"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 > $O/bench_$r.json 2> $O/bench_$r.err || { echo "BENCH FAIL"; tail -5 $O/bench_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print('bench', $r, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3), d['host_cpu']['gc_pauses'])"
done
echo ALLOK
