# Round 4: the persistent split attention + the short-K 128x192 one-round tile (candidate library in
# hubertfa_amd/_build_ab) against the shipped library.  Parity first (the candidate: attention + split GEMM tests),
# then the equal-work length sweep (persistent vs one item per workgroup, same library), the layer microbenchmark and
# the bench step interleaved (scripts/gpu_ab_libs.sh).  OUT=gpurun_out/r04h.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
# (parity of the candidate: 218 passed in the previous call)

HFA_LIB=$ALT timeout -k 10 200 python scripts/attn_len_sweep.py --modes 0,100 > $O/attn_len.txt 2>&1 || { echo "SWEEP FAIL"; tail -5 $O/attn_len.txt; exit 1; }
cat $O/attn_len.txt
OUT=$O/libs REPS=3 bash scripts/gpu_ab_libs.sh
