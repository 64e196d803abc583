# Round 5: config 5 (one 300 s utterance) with the held DP's backtrack gated at the last attention launch, A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
for rep in 1 2 3; do
  for mode in plain gate; do
    f=""; [ $mode = gate ] && f="--gate-backtrack"
    timeout -k 10 300 python bench.py --batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs $f > $O/c5_$mode$rep.json 2> $O/c5_$mode$rep.err || { echo "BENCH FAIL $mode"; tail -5 $O/c5_$mode$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c5_$mode$rep.json').read().strip().splitlines()[-1]); print('$mode', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3))"
  done
done
echo ALLOK
