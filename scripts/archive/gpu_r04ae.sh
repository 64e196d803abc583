# A/B: LayerNorm with 2 rows per wave (HFA_LN_RPW=2 build in _build_ab) vs 1; microbench twice each + bit-identity
set -o pipefail
O=gpurun_out/ln_ab; mkdir -p $O
export TMPDIR=/tmp
A=hubertfa_amd/_build/libhfa.so; B=hubertfa_amd/_build_ab/libhfa.so
for i in 1 2; do
  echo "== rpw1 $i"; HFA_LIB=$A timeout -k 10 120 python scripts/ln_bench.py --save $O/a.pt 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== rpw2 $i"; HFA_LIB=$B timeout -k 10 120 python scripts/ln_bench.py --save $O/b.pt 2>&1 | grep -v amdgpu.ids || exit 1
done
python3 -c "
import torch; a=torch.load('$O/a.pt'); b=torch.load('$O/b.pt'); print('bit-identical', all(torch.equal(a[k], b[k]) for k in a))"
rm -f $O/a.pt $O/b.pt
echo ALLOK
