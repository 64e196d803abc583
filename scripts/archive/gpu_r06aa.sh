# Round 6: the PCIe-inclusive path (bench --host-input: each step's waves uploaded from pinned host memory, as the CLI
# does) with task.upload's H2D on a stream of its own (an --upload-stream knob built for this A/B, since removed)
# against the encoder's stream, with the HBM-resident rate beside them; one box, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
for rep in 1 2 3; do
  for n in hbm host hoststream; do
    F=""; [ $n = host ] && F="--host-input"; [ $n = hoststream ] && F="--host-input --upload-stream"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 $F > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3))"
  done
done
echo ALLOK
