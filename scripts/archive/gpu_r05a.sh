# Round 5, first box: every GPU test (incl. bench.py --gpus 2 without an outer torchrun), smoke, and the default
# bench line (now with the config4 / config5 blocks).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
echo ALLOK
