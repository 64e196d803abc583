# A/B of whole-pipeline bench.py between the current build and hubertfa_amd/_build_abl/<name> builds, interleaved
# on one box (device-to-device clock differences make cross-box comparisons unreliable).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for n in cur $(ls hubertfa_amd/_build_abl); do
    lib=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = cur ] && lib=$PWD/hubertfa_amd/_build/libhfa.so
    HFA_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "BENCH FAIL $n"; tail -5 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['ms_per_step'],3), [(s['kernel'][:14], round(s['avg_launch_ms'],4)) for s in d['secondary']])"
  done
done
echo ALLOK
