# Round 6: is the 20-step timed region slower than the sustained run because of warm-up length?  --warmup 5 / 40,
# interleaved, 3 rounds; per-step event times of the timed region via --sustained-s (the block after it).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
for r in 1 2; do
  for w in 5 40; do
    timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-extra-configs --sustained-s 3 > $O/b_w${w}_$r.json 2> $O/b_w${w}_$r.err || { echo "BENCH FAIL $w"; tail -20 $O/b_w${w}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_w${w}_$r.json').read().strip().splitlines()[-1]); print("w$w", round(d["ms_per_step"],3), "sustained", round(d["sustained"]["ms_per_step"],3), {k: round(v,3) for k, v in d["timed_step_profile"].items() if k != "note"})"
  done
done
echo ALLOK
