# Round 6: the chain resampler's edge pass as two kernels (per-sample window kernel over many small workgroups, then
# per-phase-slice frame kernel) against the one-kernel form (alt = hubertfa_amd/_build_ab, the previous commit):
# chain tests, isolated timings, interleaved bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -k "chain or resample or full_path" -x -q --timeout 200 --timeout-method thread > $O/chain_tests.log 2>&1 || { echo "CHAIN TESTS FAIL"; tail -40 $O/chain_tests.log; exit 1; }
tail -1 $O/chain_tests.log
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
for n in cur alt; do
  if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
  timeout -k 10 300 python scripts/resample_tiles.py > $O/tiles_$n.txt 2>&1 || { echo "TILES FAIL $n"; tail -5 $O/tiles_$n.txt; exit 1; }
  echo "== $n"; grep -E "chain edges|chain body|two stages" $O/tiles_$n.txt
done
for rep in 1 2 3; do
  for n in cur alt; do
    if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3))"
  done
done
unset HFA_LIB
echo ALLOK
