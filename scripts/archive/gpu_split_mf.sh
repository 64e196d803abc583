# Split GEMM tile / MFMA-shape comparison on the workload's shapes (accuracy vs f64 and TF/s per cfg).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python scripts/split_gemm_bench.py --reps ${REPS:-20} --cfgs ${CFGS:-7,17,9,18,10,19} ${SHAPES:+--shapes $SHAPES} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/split_mf.txt
