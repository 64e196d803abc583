# Round 6: the CLI's GPU timeline (rocprofv3 kernel trace over scripts/cli_bench.py, 512 synthetic 10 s files, two
# runs): how much of the alignment phase the device is busy.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
rm -rf $O/trace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 scripts/cli_bench.py --n 512 --seconds 10 10 --reps 2 > $O/cli.txt 2>&1 || { echo "TRACE FAIL"; tail -20 $O/cli.txt; exit 1; }
grep -v amdgpu.ids $O/cli.txt | tail -2
find $O/trace -name "*kernel_trace.csv" | head -2
echo ALLOK
