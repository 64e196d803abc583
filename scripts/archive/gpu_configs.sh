# Bench lines for the other BASELINE configs on one GPU: config 4 geometry (Hubert-large, 32 per GPU) and
# config 5 (one 300 s utterance, unchunked).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --encoder large --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo C4FAIL; tail -5 gpurun_out/bench_c4.err; exit 1; }
cut -c1-400 gpurun_out/bench_c4.json
timeout -k 10 400 python bench.py --batch 1 --seconds 300 --words 600 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo C5FAIL; tail -5 gpurun_out/bench_c5.err; exit 1; }
cut -c1-400 gpurun_out/bench_c5.json
echo ALLOK
