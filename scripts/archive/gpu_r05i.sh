# Round 5: conv K-steps in channel-block-major / tap-minor order.  GPU tests on the GEMM / conv / encoder paths,
# then the split-GEMM micro (conv1 is the one conv shape in it) against the tap-major build and the L2-hot
# ablation, then the config-2 bench twice.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "split or kernels or configs or reference10s or unet or canary or large or posconv or varlen or pipeline or smoke" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MICRO=scripts/gemm_abl.py ALTS="_abl_tapmajor _abl_l2hot" bash scripts/gpu_ab_micro.sh || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs > $O/b$r.json 2> $O/b$r.err || { echo "BENCH FAIL"; tail -20 $O/b$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b$r.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'])"
  HFA_LIB=$PWD/hubertfa_amd/_abl_tapmajor/libhfa.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs > $O/t$r.json 2> $O/t$r.err || { echo "BENCH FAIL"; tail -20 $O/t$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/t$r.json').read().strip().splitlines()[-1]); print('tapmajor', d['ms_per_step'], d['value'])"
done
echo ALLOK
