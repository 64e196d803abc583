# Per-shape in-pipeline roofline table (scripts/shape_trace.py + shape_table.py): one kernel-trace pass and two PMC
# passes (MFMA busy + clock; SQ wait split), each in its own rocprofv3 run.  OUT=gpurun_out/<tag>; ENC=base|large.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/shapes}
ENC=${ENC:-base}
mkdir -p $O
rm -rf $O/trace $O/pmc_mfma $O/pmc_wait
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --encoder $ENC > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/shape_trace.py --encoder $ENC --steps 6 --warmup 3 --log $O/trace/launch_log.json > $O/trace.log 2>&1 || { echo "TRACE FAIL"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_mfma -o run -- python3 scripts/shape_trace.py --encoder $ENC --steps 2 --warmup 1 --log $O/pmc_mfma/launch_log.json > $O/pmc_mfma.log 2>&1 || { echo "PMC MFMA FAIL"; tail -20 $O/pmc_mfma.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_wait -o run -- python3 scripts/shape_trace.py --encoder $ENC --steps 2 --warmup 1 --log $O/pmc_wait/launch_log.json > $O/pmc_wait.log 2>&1 || { echo "PMC WAIT FAIL"; tail -20 $O/pmc_wait.log; exit 1; }
python scripts/shape_table.py --trace $O/trace --log $O/trace/launch_log.json --pmc $O/pmc_mfma --pmc-log $O/pmc_mfma/launch_log.json --pmc $O/pmc_wait --pmc-log $O/pmc_wait/launch_log.json --csv $O/shape_roofline.csv --json $O/shape_roofline.json > $O/shape_table.txt 2>&1 || { echo "TABLE FAIL"; cat $O/shape_table.txt; }
cat $O/shape_table.txt
tail -c 600 $O/bench.json
echo ALLOK
