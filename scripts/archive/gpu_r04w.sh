# config 5: the DP gated at the next encoder's attention launches (scripts/dp_gate_ab.py) + the step-range parity test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
true
true
timeout -k 10 400 python -u scripts/dp_gate_ab.py --batch 32 --seconds 10 --words 30 --segments 1,2,3 --reps 10 > gpurun_out/dp_gate_ab.txt 2>&1 || { echo "AB FAIL"; tail -30 gpurun_out/dp_gate_ab.txt; exit 1; }
cat gpurun_out/dp_gate_ab.txt
