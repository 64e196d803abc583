# Round-3: the new tests first (reported, not fatal), then the full validation + profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${NEWTESTS:-tests/test_config1_gpu.py tests/test_api_gpu.py} -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/newtests.log 2>&1
echo "new tests rc=$?"; grep -E "PASSED|FAILED|ERROR|error vs|error:|300 s" gpurun_out/newtests.log | tail -40
bash scripts/gpu_full.sh
