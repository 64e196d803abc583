set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "attention" > gpurun_out/atest.log 2>&1 || { echo "ATEST FAIL"; tail -30 gpurun_out/atest.log; exit 1; }
tail -1 gpurun_out/atest.log
timeout -k 10 200 python scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids || { echo "ABENCH FAIL"; exit 1; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/ktest.log 2>&1 || { echo "KTEST FAIL"; tail -30 gpurun_out/ktest.log; exit 1; }
tail -1 gpurun_out/ktest.log
for n in $(ls hubertfa_amd/_build_abl 2>/dev/null); do
  echo "== $n"; HFA_LIB=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so timeout -k 10 200 python scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
echo ALLOK
