# A/B: the one-wave DP with 1 / 2 / 4 utterances per workgroup beside the encoder (config-2 geometry)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/dp_upw_ab.py > gpurun_out/dp_upw_ab.txt 2>&1 || { echo "AB FAIL"; tail -30 gpurun_out/dp_upw_ab.txt; exit 1; }
cat gpurun_out/dp_upw_ab.txt
