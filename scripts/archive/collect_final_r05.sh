# Copy the round-5 final run's outputs (gpurun_out/final, scripts/gpu_final_r05.sh) into profiles/r05/ under the
# names bench.py's defaults and DESIGN.md cite.  CPU only.
set -e
F=gpurun_out/final5
P=profiles/r05
mkdir -p $P
cp $F/traffic_r05.json $P/traffic_r05.json
cp $F/pmc_r05.json $P/pmc_r05.json
cp $F/pmc_kernels.txt $P/pmc_kernels_r05.txt
cp $F/shape_roofline.csv $P/shape_roofline.csv
cp $F/shape_roofline.json $P/shape_roofline.json
cp $F/shape_table.txt $P/shape_roofline.txt
[ -f $F/shape_serial.csv ] && cp $F/shape_serial.csv $P/shape_serial.csv
[ -f $F/attn_len.txt ] && cp $F/attn_len.txt $P/attn_len_sweep.txt
[ -f $F/host_cpu.txt ] && cp $F/host_cpu.txt $P/host_cpu.txt
tail -n 1 $F/bench.json > $P/bench_r05.json
cp $F/gputests.log $P/gputests_r05.txt
cp $F/smoke.log $P/smoke_r05.txt
# rocprof kernel table of the bench run
S=$(ls $F/stats/*kernel_stats.csv 2>/dev/null | head -1)
[ -z "$S" ] && S=$(find $F/stats -name '*kernel_stats.csv' | head -1)
cp "$S" $P/bench_kernel_stats_r05.csv
ls -la $P
