# Round 6: what the live HIP-event probe costs the timed region -- old form (dominant + secondary kernels in every
# timed step) vs the dominant kernel alone in every step vs every 4th step; interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
for r in 1 2 3; do
  for m in "--probe-secondary" "--probe-every 1" "--probe-every 4"; do
    t=$(echo $m | tr -d ' -')
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 3 $m > $O/b_${t}_$r.json 2> $O/b_${t}_$r.err || { echo "BENCH FAIL $m"; tail -20 $O/b_${t}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${t}_$r.json').read().strip().splitlines()[-1]); print('$t', round(d['ms_per_step'],3), 'sustained', round(d['sustained']['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'probed', d['roofline']['timed_steps_probed'], d['roofline']['launches'])"
  done
done
echo ALLOK
