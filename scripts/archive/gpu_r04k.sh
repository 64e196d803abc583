# Round 4: which host threads burn CPU around the pipelined step (scripts/host_threads.py).  OUT=gpurun_out/r04k.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python scripts/host_threads.py > $O/threads.txt 2>&1 || { echo "THREADS FAIL"; tail -20 $O/threads.txt; exit 1; }
grep -v amdgpu.ids $O/threads.txt
echo ALLOK
