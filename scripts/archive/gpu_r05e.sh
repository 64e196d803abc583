# Round 5: rocprof kernel tables of configs 4 and 5 (bench.py geometry), to see where their steps go.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --encoder large --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/c4.log 2>&1 || { echo "C4 FAIL"; tail -5 $O/c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 bench.py --batch 1 --seconds 300 --words 600 --steps 6 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/c5.log 2>&1 || { echo "C5 FAIL"; tail -5 $O/c5.log; exit 1; }
for c in c4 c5; do S=$(find $O/$c -name '*kernel_stats.csv' | head -1); cp "$S" $O/${c}_kernel_stats.csv; find $O/$c -name '*kernel_trace.csv' -delete; done
head -14 $O/c4_kernel_stats.csv | cut -c1-200
head -14 $O/c5_kernel_stats.csv | cut -c1-200
echo ALLOK
