# split attention waves per workgroup: the CU-share rule (automatic, mode 0) against forced 4 / 8 waves
set -o pipefail
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
: > $O/attn_waves_rule.txt
for bl in "1 1000,2000,3000,4000,5000,6000,7000,8000,9000,10000,11000,12000,13000,14000,14999,16000,18000" "32 499" "15 1200" "4 3000" "2 7000" "8 1000"; do
  set -- $bl
  timeout -k 10 300 python scripts/attn_len_sweep.py --reps 10 --modes 0,4,8 --batch $1 --lengths $2 2>&1 | grep "^mode" >> $O/attn_waves_rule.txt || exit 1
done
cat $O/attn_waves_rule.txt
