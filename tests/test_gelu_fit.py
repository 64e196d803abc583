"""The epilogue GELU's constants (hfa::gelu_fast in hubertfa_amd/csrc/hfa_common.h) under an f32 emulation of the
kernel's arithmetic (scripts/fit_gelu_erf.py): within 1.25 |x| 2^-24 of the f64 GELU everywhere and 5 ulp where
x > -1.5 -- the bars tests/test_kernels_gpu.py::test_epilogue_gelu_accuracy checks on the device (4 |x| 2^-24, 12 ulp)
with margin.  CPU only."""
import os
import re
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_coefficients():
    src = open(os.path.join(REPO, "hubertfa_amd", "csrc", "hfa_common.h")).read()
    body = src[src.index("float gelu_fast(float x)"):]
    body = body[:body.index("\n}\n")]
    hexes = re.findall(r"__uint_as_float\(0x([0-9a-f]{8})u\)", body)
    vals = [struct.unpack("<f", struct.pack("<I", int(h, 16)))[0] for h in hexes]
    return np.array(vals[::-1], dtype=np.float64)          # lowest degree first, as fit() returns


def test_gelu_fast_constants_accuracy():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import fit_gelu_erf as F
    from scipy.special import erf
    r = _device_coefficients()
    assert len(r) == 8                                       # R7: 7 fmas + the leading constant
    x = np.concatenate([np.linspace(-12, 12, 400_001), np.random.default_rng(5).normal(0, 3, 400_000)]).astype(np.float32)
    xd = x.astype(np.float64)
    truth = 0.5 * xd * (1 + erf(xd / np.sqrt(2.0)))
    y = F.gelu_emulated(x, r).astype(np.float64)
    err = np.abs(y - truth)
    assert (err / (np.abs(xd) * 2.0 ** -24 + 1e-38)).max() <= 1.25
    m = xd > -1.5
    ulp = np.spacing(np.abs(truth[m]).astype(np.float32)).astype(np.float64)
    assert (err[m] / ulp).max() <= 5.0


def test_gelu_fit_reproduces_device_constants():
    """The fit script, rerun, gives the constants the kernel holds (to f32 rounding)."""
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import fit_gelu_erf as F
    r = F.fit()
    dev = _device_coefficients()
    assert np.array_equal(np.float32(r), np.float32(dev))
