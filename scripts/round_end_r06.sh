# Round-end check (verdict r05 item 1): the CPU suite in the build container first -- a tile-rule or ABI change must
# not ship with it red -- then the full GPU validation + measurement on one box (scripts/gpu_final_r06.sh).
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 1200 python -m pytest tests -x -q -m "not gpu" || { echo "CPU SUITE RED: not running the GPU validation"; exit 1; }
/usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_final_r06.sh'
