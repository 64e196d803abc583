set -o pipefail
V=102:1 SH=conv1,qkv,ffn1,ffn2 bash scripts/gpu_pmc_gemm.sh > /dev/null 2>&1 || { echo PMCFAIL; exit 1; }
awk 'NR==1 || NR%6==2' gpurun_out/pmc_gemm_summary.txt
for e in 0 1; do timeout -k 10 120 python scripts/gemm_bench.py --variants 102:1 --shapes conv1,conv3,ffn1,ffn2,qkv --epi $e --reps 10 2>&1 | grep -v amdgpu.ids; done
echo ALLOK
