# Round 5: narrow-N tile rule (UNet N = 192 at K <= 1152 on 128 x 64, the resampler's N = 160 on 128 x 192).  Tests
# on the tiles / UNet / resampler / pipeline, the shape micros under the new automatic choice, then the config-2
# bench against the previous rule's build (hubertfa_amd/_abl_prevrule), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/side_tiles
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "split or unet or resample or pipeline or reference10s or configs" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/tile_sweep.py > $O/sweep.txt 2>&1 && grep "cfg  0" $O/sweep.txt
timeout -k 10 300 python scripts/resample_tiles.py > $O/resample.txt 2>&1 && grep "cfg  0" $O/resample.txt
for r in 1 2 3; do
  for n in cur prev; do
    if [ $n = cur ]; then unset HFA_LIB; else export HFA_LIB=$PWD/hubertfa_amd/_abl_prevrule/libhfa.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs > $O/$n.$r.json 2> $O/$n.$r.err || { echo "BENCH FAIL"; tail -20 $O/$n.$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/$n.$r.json').read().strip().splitlines()[-1]); b=d['step_breakdown']; print('$n', round(d['ms_per_step'],3), round(d['value'],1), 'enc', round(b['encoder_only_ms'],3), 'side', round(b['side_stream_cost_ms'],3), 'head_dp', round(b['head_dp_only_ms'],3))"
  done
done
unset HFA_LIB
echo ALLOK
