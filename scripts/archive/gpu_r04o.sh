# Round 4: UNet + head alone at B = 32, 64, 96 (does a larger UNet batch amortise its per-launch cost?).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
for B in 32 64 96 32; do
  timeout -k 10 200 python scripts/unet_bench.py --B $B --tiles 0 > $O/unet_$B.txt 2>&1 || { echo "UNET FAIL $B"; tail -5 $O/unet_$B.txt; exit 1; }
  grep "head split" $O/unet_$B.txt
done
echo ALLOK
