# Round-6 full validation + measurement of the shipped build (the CPU suite, `pytest -m "not gpu"`, runs in the build
# container before this script: scripts/round_end_r06.sh): every GPU test, smoke, the dominant kernel's PMC
# traffic (FETCH_SIZE / WRITE_SIZE passes), the per-shape in-pipeline table and per-kernel MFMA busy / clock (kernel
# trace + two PMC passes over scripts/shape_trace.py), the rocprof kernel stats of a bench run, then the bench line
# reading those files.  Outputs under gpurun_out/final6 (copied into profiles/r06/ by hand).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final6
mkdir -p $O
(nproc; lscpu) > $O/host_cpu.txt 2>&1 || true
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
  tail -2 $O/gputests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --sustained-s 0 > $O/bench_pre.json 2> $O/bench_pre.err || { echo "BENCH0 FAIL"; tail -20 $O/bench_pre.err; exit 1; }
K=$(python -c "import json; print(json.loads(open('$O/bench_pre.json').read().strip().splitlines()[-1])['roofline']['kernel'])")
echo "dominant kernel: $K"
rm -rf $O/pmc_fetch $O/pmc_write $O/stats $O/trace $O/pmc_mfma $O/pmc_wait
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --sustained-s 0 > $O/pmc1.log 2>&1 || { echo "PMC FETCH FAIL"; tail -5 $O/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --sustained-s 0 > $O/pmc2.log 2>&1 || { echo "PMC WRITE FAIL"; tail -5 $O/pmc2.log; exit 1; }
python scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --kernel "$K" --out $O/traffic_r06.json > $O/traffic.log 2>&1 || { echo "TRAFFIC PARSE FAIL"; cat $O/traffic.log; }
rm -rf $O/pmc_fetch $O/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --sustained-s 0 > $O/stats.log 2>&1 || { echo "STATS FAIL"; tail -5 $O/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 scripts/shape_trace.py --steps 8 --warmup 3 --log $O/trace/launch_log.json > $O/trace.log 2>&1 || { echo "TRACE FAIL"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_mfma -o run -- python3 scripts/shape_trace.py --steps 2 --warmup 1 --log $O/pmc_mfma/launch_log.json > $O/pmc_mfma.log 2>&1 || { echo "PMC MFMA FAIL"; tail -20 $O/pmc_mfma.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_wait -o run -- python3 scripts/shape_trace.py --steps 2 --warmup 1 --log $O/pmc_wait/launch_log.json > $O/pmc_wait.log 2>&1 || { echo "PMC WAIT FAIL"; tail -20 $O/pmc_wait.log; exit 1; }
python scripts/shape_table.py --trace $O/trace --log $O/trace/launch_log.json --pmc $O/pmc_mfma --pmc-log $O/pmc_mfma/launch_log.json --pmc $O/pmc_wait --pmc-log $O/pmc_wait/launch_log.json --csv $O/shape_roofline.csv --json $O/shape_roofline.json > $O/shape_table.txt 2>&1 || { echo "TABLE FAIL"; cat $O/shape_table.txt; }
python scripts/pmc_kernels.py --mfma $O/pmc_mfma --wait $O/pmc_wait --out $O/pmc_r06.json > $O/pmc_kernels.txt 2>&1 || { echo "PMC KERNELS FAIL"; cat $O/pmc_kernels.txt; }
rm -rf $O/pmc_mfma/*.csv.bak
head -12 $O/shape_table.txt
rm -rf $O/serial
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/serial -o run -- python3 scripts/shape_trace.py --mode serial --steps 6 --warmup 3 --log $O/serial/launch_log.json > $O/serial.log 2>&1 || { echo "SERIAL TRACE FAIL"; tail -20 $O/serial.log; exit 1; }
python scripts/shape_table.py --trace $O/serial --log $O/serial/launch_log.json --csv $O/shape_serial.csv > $O/shape_serial.txt 2>&1 || { echo "SERIAL TABLE FAIL"; cat $O/shape_serial.txt; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --traffic-file $O/traffic_r06.json --pmc-file $O/pmc_r06.json > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
echo ALLOK
