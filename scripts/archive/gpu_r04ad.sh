# 2-rank rehearsal (gloo, both ranks on GPU 0) of the bench with a held long-lattice DP: each rank one 200 s utterance
# (17 226 DP frames >= defer_dp_frames), the boundary gather (on_device) running in the held batch's completion
set -o pipefail
mkdir -p gpurun_out/r04ad
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --batch 1 --seconds 200 --words 400 --steps 4 --warmup 1 --dist-backend gloo --device 0 --no-cpu-baseline > gpurun_out/r04ad/bench_n2_held.json 2> gpurun_out/r04ad/bench_n2_held.err || { echo "N2 FAIL"; tail -30 gpurun_out/r04ad/bench_n2_held.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04ad/bench_n2_held.json').read().strip().splitlines()[-1]); print(d['n_gpus'], round(d['value'],1), round(d['ms_per_step'],2), d['config']['workload'][:80])"
echo ALLOK
