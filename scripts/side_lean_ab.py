"""A/B of the side stream's UNet GEMM tile (run on the GPU box): bench.py's config-2 step with the UNet's split
GEMMs forced to split tile CFG (hfa_gemm_split_tuning, thread-local, set around each UNet GEMM call) against the
automatic tiles.  Usage: python scripts/side_lean_ab.py CFG [bench.py args]; CFG 0 = shipped choice."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hubertfa_amd import _lib, unet  # noqa: E402

CFG = int(sys.argv[1])


def forced(fn):
    def run(*a, **kw):
        if not CFG:
            return fn(*a, **kw)
        _lib.lib().hfa_gemm_split_tuning(CFG)
        try:
            return fn(*a, **kw)
        finally:
            _lib.lib().hfa_gemm_split_tuning(0)
    return run


unet._Ctx.conv = forced(unet._Ctx.conv)
unet._Ctx.linear = forced(unet._Ctx.linear)
bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
sys.argv = [bench] + sys.argv[2:]
runpy.run_path(bench, run_name="__main__")
