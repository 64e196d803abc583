set -o pipefail
bash scripts/gpu_r05f.sh && MICRO=scripts/gemm_abl.py ALTS="_abl_novm _abl_nobar _abl_nodma" bash scripts/gpu_ab_micro.sh && bash scripts/gpu_r05h.sh
