# A/B: split GEMM 8-wave tiles with the younger half (waves 4-7) at static issue priority 1 (HFA_GEMM_YPRIO build in
# _build_ab) against the shipped build; config 2, three interleaved pairs
set -o pipefail
O=gpurun_out/yprio; mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1 lib=$2
  HFA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('$tag', round(d['value'],1), round(d['ms_per_step'],3), 'dominant', round(r['avg_launch_ms']*1e3,1), 'us', round(r['frac'],3))"
}
A=hubertfa_amd/_build/libhfa.so; B=hubertfa_amd/_build_ab/libhfa.so
run base1 $A && run yprio1 $B && run base2 $A && run yprio2 $B && run base3 $A && run yprio3 $B && echo ALLOK
