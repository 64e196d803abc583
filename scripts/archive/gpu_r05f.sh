# Round 5: Hubert-large's LayerNorm-conv extractor writing the next conv's planes from the LayerNorm (no f32 write,
# no conversion pass): the large-encoder parity tests, then the config-4 bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "large or reference10s or varlen or loaders or configs or groupnorm or unet" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --encoder large --steps 10 --warmup 3 --no-cpu-baseline --no-extra-configs > $O/c4_$rep.json 2> $O/c4_$rep.err || { echo "BENCH FAIL"; tail -5 $O/c4_$rep.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_$rep.json').read().strip().splitlines()[-1]); print('config 4', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3))"
done
echo ALLOK
