# Round 4: the 64-queries-per-wave split attention (attention64.hip, hfa_attention_split_tuning(64)): parity (bit
# identity with the 4/8-wave kernel and the f64 tests), then the equal-work length sweep and the layer microbenchmark.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -k attention > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python scripts/attn_len_sweep.py --modes 0,64 > $O/attn_len.txt 2>&1 || { echo "SWEEP FAIL"; tail -5 $O/attn_len.txt; exit 1; }
grep -v amdgpu.ids $O/attn_len.txt
timeout -k 10 200 python scripts/layer_gemm_bench.py --cfgs 0 > $O/layer.txt 2>&1 || { echo "LAYER FAIL"; tail -5 $O/layer.txt; exit 1; }
grep attention $O/layer.txt
echo ALLOK
