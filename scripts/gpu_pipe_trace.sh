# Kernel traces of the pipelined step, chip-wide UNet (A) vs fused UNet (B).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HFA_UNET_FUSED=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptA -o run -- python3 scripts/pipe_trace.py > gpurun_out/ptA.log 2>&1 &&
HFA_UNET_FUSED=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptB -o run -- python3 scripts/pipe_trace.py > gpurun_out/ptB.log 2>&1 &&
python3 scripts/pipe_cmp.py $(ls gpurun_out/ptA/*/run_kernel_trace.csv gpurun_out/ptA/run_kernel_trace.csv 2>/dev/null | head -1) $(ls gpurun_out/ptB/*/run_kernel_trace.csv gpurun_out/ptB/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/pipe_cmp.txt
