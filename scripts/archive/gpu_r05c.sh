set -o pipefail
bash scripts/gpu_ab_pair.sh && ALTS="_abl_nobar _abl_nowait" bash scripts/gpu_ab_micro.sh
