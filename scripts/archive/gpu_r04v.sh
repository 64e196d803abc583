# A/B: the encoder's MFMA kernels (split GEMM, split attention, positional conv) at issue priority 1 over the
# co-resident side-stream waves (DP, norms), HFA_LIB=_build_prio, against the shipped priority 0.  Config 2 and config 5.
set -o pipefail
O=gpurun_out/prio_ab; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  HFA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$tag.json')); b=d.get('step_breakdown',{}); print('$tag', round(d['value'],1), round(d['ms_per_step'],3), {k:(round(v,3) if isinstance(v,float) else v) for k,v in b.items() if 'ms' in k})"
}
A=hubertfa_amd/_build/libhfa.so; B=hubertfa_amd/_build_prio/libhfa.so
run c5_base $A --batch 1 --seconds 300 --words 600 --steps 3 --warmup 1 && \
run c5_prio $B --batch 1 --seconds 300 --words 600 --steps 3 --warmup 1 && \
run c2_base1 $A --steps 20 --warmup 3 && \
run c2_prio1 $B --steps 20 --warmup 3 && \
run c2_base2 $A --steps 20 --warmup 3 && \
run c2_prio2 $B --steps 20 --warmup 3 && echo ALLOK
