# UNet + head alone (B=32 x 864 frames): per-launch kernel trace, to see where the side stream's CU time goes
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/unet_trace
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/unet_trace -o run --output-format csv -- python3 scripts/unet_bench.py --reps 5 > gpurun_out/unet_trace/out.txt 2>&1
