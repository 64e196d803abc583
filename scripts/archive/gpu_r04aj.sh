# DP with f32 curr (CF) and one select fewer per state: parity tests, then the DP alone (scripts/dp_bench.py) and the
# benches against the previous build (_build_ab, HEAD sources before the change)
set -o pipefail
O=gpurun_out/dpcf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_viterbi_gpu.py tests/test_longform_gpu.py tests/test_reference10s_gpu.py tests/test_pipeline_gpu.py > $O/tests.txt 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
A=hubertfa_amd/_build_ab/libhfa.so; B=hubertfa_amd/_build/libhfa.so
echo "== dp old"; HFA_LIB=$A timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep "K=auto" || exit 1
echo "== dp new"; HFA_LIB=$B timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep "K=auto" || exit 1
run() {
  local tag=$1 lib=$2; shift 2
  HFA_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value'],1), round(d['ms_per_step'],3))"
}
C5C="--batch 1 --seconds 300 --words 600 --steps 10 --warmup 2 --chunk-seconds 20"
run c2_old1 $A --steps 20 --warmup 5 && run c2_new1 $B --steps 20 --warmup 5 && run c2_old2 $A --steps 20 --warmup 5 && run c2_new2 $B --steps 20 --warmup 5 && \
run c5c_old $A $C5C && run c5c_new $B $C5C && echo ALLOK
