# Round 5, secondary bench lines (one box): hubertsoft at config-2 geometry, config 5 in 20 s windows (the chunked
# throughput mode), the PCIe-inclusive host-input rate, the serial (one-stream) step and the f16 fast mode.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_side
mkdir -p $O
run() {  # name, args...
  n=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-extra-configs "$@" > $O/$n.json 2> $O/$n.err || { echo "BENCH FAIL $n"; tail -20 $O/$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3), 'ms/step', round(d['value'],1), d['unit'])"
}
run base --steps 20 --warmup 5
run soft --encoder soft --steps 20 --warmup 5
run c5chunk20 --batch 1 --seconds 300 --words 600 --chunk-seconds 20 --steps 10 --warmup 2
run hostin --host-input --steps 20 --warmup 5
run serial --serial --steps 20 --warmup 5
run f16 --precision f16 --steps 20 --warmup 5
echo ALLOK
