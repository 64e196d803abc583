# Round 6: config 2 with its forward DP held for the next encoder's attention launches (bench --defer-dp-frames 512:
# 12 step ranges of ~72 frames, the backtrack after the last) against one DP launch behind the head (default), one
# box, interleaved; the held path's own tests first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
for rep in 1 2 3; do
  for n in held whole; do
    F=""; [ $n = held ] && F="--defer-dp-frames 512"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 $F > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3), round(d['step_breakdown']['side_stream_cost_ms'],3))"
  done
done
echo ALLOK
