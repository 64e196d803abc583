# Interleaved microbenchmark A/B of library builds: cur (hubertfa_amd/_build) against every alt build listed in
# ALTS (directories under hubertfa_amd/, each holding a libhfa.so), MICRO = the script to run (default attention).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_micro
mkdir -p $O
M=${MICRO:-scripts/attn_abl.py}
for rep in 1 2 3; do
  for n in cur $ALTS; do
    if [ $n = cur ]; then unset HFA_LIB; else export HFA_LIB=$PWD/hubertfa_amd/$n/libhfa.so; fi
    timeout -k 10 200 python $M > $O/$n.$rep.txt 2>&1 || { echo "MICRO FAIL $n"; tail -5 $O/$n.$rep.txt; exit 1; }
    grep -v amdgpu.ids $O/$n.$rep.txt
  done
done
unset HFA_LIB
echo ALLOK
