# Measurement (TAG=r02 ...): bench line, rocprof kernel stats, PMC traffic of the dominant kernel.
# The dominant kernel name is taken from a first bench run's roofline.kernel, so the PMC pass always
# measures the instantiation bench.py probes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > $OUT/ktest.log 2>&1 || { echo "KTEST FAIL"; tail -30 $OUT/ktest.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_pre.json 2> $OUT/bench_pre.err || { echo "BENCH0 FAIL"; tail -20 $OUT/bench_pre.err; exit 1; }
K=$(python -c "import json,sys; print(json.loads(open('$OUT/bench_pre.json').read().strip().splitlines()[-1])['roofline']['kernel'])")
echo "dominant kernel: $K"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/stats.log 2>&1 || { echo "PROF FAIL"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc1.log 2>&1 || { echo "PMC1 FAIL"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc2.log 2>&1 || { echo "PMC2 FAIL"; exit 1; }
python scripts/pmc_traffic.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --kernel "$K" --out $OUT/traffic_${TAG:-r02}.json > $OUT/traffic.log 2>&1 || { echo "TRAFFIC PARSE FAIL"; cat $OUT/traffic.log; }
rm -rf $OUT/pmc_fetch $OUT/pmc_write
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --traffic-file $OUT/traffic_${TAG:-r02}.json > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAIL"; exit 1; }
cat $OUT/bench.json
echo ALLOK
