# rocprof kernel stats of a short bench run (per-kernel time per batch): gpurun_out/stats/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/stats.log 2>&1 || { echo "PROF FAIL"; tail -20 gpurun_out/stats.log; exit 1; }
python scripts/kstats.py gpurun_out/stats/run_kernel_stats.csv ${NBATCH:-9}
