# Round 4, final tree (held DP, attention wave rule): the whole GPU test suite and smoke, the default bench line, and config 5
# unchunked / in 20 s windows at 10 steps (the drain of the last batch's side pass amortised).  OUT=gpurun_out/r04z2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 400 python bench.py --batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH C5 FAIL"; tail $O/bench_c5.err; exit 1; }
timeout -k 10 400 python bench.py --batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --no-cpu-baseline --chunk-seconds 20 > $O/bench_c5c.json 2> $O/bench_c5c.err || { echo "BENCH C5C FAIL"; tail $O/bench_c5c.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_c5', 'bench_c5c'):
    d = json.loads(open('$O/%s.json' % f).read().strip().splitlines()[-1]); print(f, round(d['value'], 1), round(d['ms_per_step'], 3))"
echo ALLOK
