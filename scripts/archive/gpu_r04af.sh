# UNet + head alone with every backbone GEMM forced onto one split tile: automatic, 128x128, 128x64, 256x64 (MF16)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 200 python scripts/unet_bench.py --tiles 0,18,19,20 2>&1 | grep -v amdgpu.ids || exit 1; done
echo ALLOK
