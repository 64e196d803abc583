set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5t -o run -- python3 bench.py --batch 1 --seconds 300 --words 600 --steps 4 --warmup 1 --no-cpu-baseline --chunk-seconds 20 > gpurun_out/c5t.log 2>&1 &&
python3 scripts/c5_trace_summary.py gpurun_out/c5t/run_kernel_trace.csv > gpurun_out/c5t_summary.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c2_bd.json 2> gpurun_out/c2_bd.err &&
python -c "import json; d=json.loads(open('gpurun_out/c2_bd.json').read().strip().splitlines()[-1]); print('c2', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
