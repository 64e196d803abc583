# bench variants of the round-4 build into gpurun_out/multi_r04: config 2, config 4 (large), the 2-rank rehearsal of the N>1 path on one GPU (gloo), config 5 unchunked and in 20 s windows.
set -o pipefail
O=gpurun_out/multi_r04; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "BENCH C2 FAIL"; tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --encoder large --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo "BENCH C4 FAIL"; tail $O/bench_c4.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 --dist-backend gloo --device 0 > $O/bench_n2.json 2> $O/bench_n2.err || { echo "BENCH N2 FAIL"; tail $O/bench_n2.err; exit 1; }
timeout -k 10 400 python bench.py --batch 1 --seconds 300 --words 600 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH C5 FAIL"; tail $O/bench_c5.err; exit 1; }
timeout -k 10 400 python bench.py --batch 1 --seconds 300 --words 600 --steps 6 --warmup 2 --no-cpu-baseline --chunk-seconds 20 > $O/bench_c5c.json 2> $O/bench_c5c.err || { echo "BENCH C5 CHUNKED FAIL"; tail $O/bench_c5c.err; exit 1; }
echo ALLOK
