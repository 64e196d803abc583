# A/B: split GEMMs with N < 512 (the UNet's convs, the head, the resamplers) on the 128x64 tile (HFA_SMALLN_64 build in
# _build_ab) instead of 128x128: UNet alone (automatic tiles), then config 2 bench, three interleaved pairs
set -o pipefail
O=gpurun_out/smalln; mkdir -p $O
export TMPDIR=/tmp
A=hubertfa_amd/_build/libhfa.so; B=hubertfa_amd/_build_ab/libhfa.so
echo "== unet cur"; HFA_LIB=$A timeout -k 10 200 python scripts/unet_bench.py --tiles 0 2>&1 | grep "tile 0" || exit 1
echo "== unet alt"; HFA_LIB=$B timeout -k 10 200 python scripts/unet_bench.py --tiles 0 2>&1 | grep "tile 0" || exit 1
run() {
  local tag=$1 lib=$2
  HFA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); b=d['step_breakdown']; print('$tag', round(d['value'],1), round(d['ms_per_step'],3), 'enc', round(b['encoder_only_ms'],3), 'side', round(b['side_stream_cost_ms'],3), 'head_dp', round(b['head_dp_only_ms'],3))"
}
run cur1 $A && run alt1 $B && run cur2 $A && run alt2 $B && run cur3 $A && run alt3 $B && echo ALLOK
