# Side-stream UNet GEMM tile A/B: the lean 64 x 64 tile (SCFG 26: 32 KiB LDS, <= 96 VGPRs, co-resident with an
# encoder tile) against the automatic tiles, config-2 bench (20 steps), 3 interleaved rounds; UNet parity first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/side_lean
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "unet or split_single_acc" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/gemm_abl.py --cfg 26 > $O/micro26.txt 2>&1 || { echo MICRO FAIL; tail -5 $O/micro26.txt; exit 1; }
grep -v amdgpu.ids $O/micro26.txt
for r in 1 2 3; do
  for c in 0 26; do
    timeout -k 10 300 python scripts/side_lean_ab.py $c --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs > $O/b$c.$r.json 2> $O/b$c.$r.err || { echo "BENCH FAIL $c"; tail -20 $O/b$c.$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b$c.$r.json').read().strip().splitlines()[-1]); b=d['step_breakdown']; print('cfg $c', round(d['ms_per_step'],3), round(d['value'],1), 'enc', round(b['encoder_only_ms'],3), 'side', round(b['side_stream_cost_ms'],3), 'head_dp', round(b['head_dp_only_ms'],3))"
  done
done
echo ALLOK
