# Round 6: the side pass's row-kernel workgroup cap re-tuned on the final tree (bench --side-grid-cap 128 / 256 / 512;
# first pass 256 / 512 / 1024), one box, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
for rep in 1 2 3; do
  for c in 128 256 512; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 --side-grid-cap $c > $O/bench_${c}_$rep.json 2> $O/bench_${c}_$rep.err || { echo "BENCH FAIL $c"; tail -5 $O/bench_${c}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${c}_$rep.json').read().strip().splitlines()[-1]); print('$c', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3), round(d['step_breakdown']['side_stream_cost_ms'],3))"
  done
done
echo ALLOK
