set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/split_gemm_bench.py --reps 20 --cfgs 0,17,18,23,24,21,22 --shapes qkv_c2,ffn1_c2,qkv_c5,ffn1_c5,ffn2_c5,outproj_c5 > gpurun_out/tiles_c5.txt 2>&1 || { tail gpurun_out/tiles_c5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tiles_c5.txt
bash scripts/gpu_c5_trace.sh
