# Round 6: the CLI's per-batch timeline (HFA_CLI_TRACE: submit / loaded / submitted / settle / assembled / exported
# times of the launching thread), 1 024 synthetic 10 s files, three runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
rm -f $O/cli_trace.jsonl
HFA_CLI_TRACE=$PWD/$O/cli_trace.jsonl timeout -k 10 400 python scripts/cli_bench.py --n 1024 --seconds 10 10 --reps 3 > $O/cli.txt 2>&1 || { echo "CLI FAIL"; tail -20 $O/cli.txt; exit 1; }
grep -v amdgpu.ids $O/cli.txt | tail -3
echo ALLOK
