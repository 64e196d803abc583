"""Fit of the GELU epilogue's erf (hfa::gelu_fast in hubertfa_amd/csrc/hfa_common.h) and its f32 accuracy check.

erf(z) = sign(z) * (1 - exp(-q(|z|))), q(a) = a + a * P8(a) ~ -log(1 - erf(a)) on [0, 3.95], fitted by least squares
weighted by d erf / d q = exp(-q) (absolute error of erf), iteratively re-weighted toward minimax.  Prints the f32 hex
coefficients (highest degree first, Horner order of the kernel) and the f32-emulated GELU error against fp64.

python scripts/fit_gelu_erf.py
"""
import struct

import numpy as np
from scipy.special import erf as erf64

f32 = np.float32


def fit(deg=8, hi=3.95, n=400001, iters=30):
    zs = np.linspace(0, hi, n)[1:]
    target = -np.log1p(-erf64(zs))
    y = (target - zs) / zs
    A = np.vstack([zs ** k for k in range(deg + 1)]).T
    w = np.exp(-target)
    c, *_ = np.linalg.lstsq(A * (w * zs)[:, None], y * w * zs, rcond=None)
    for _ in range(iters):          # multiplicative re-weighting toward the minimax solution
        r = np.abs((A @ c - y) * zs * w)
        w = w * (1 + 20 * r / r.max())
        w = w / w.max()
        c, *_ = np.linalg.lstsq(A * (w * zs)[:, None], y * w * zs, rcond=None)
    return c


def gelu_emulated(x, c, hi=3.95):
    """The kernel's f32 arithmetic (fma exact via f64; v_exp_f32 ~ correctly rounded exp2)."""
    def fma(a, b, d):
        return (a.astype(np.float64) * b.astype(np.float64) + d.astype(np.float64)).astype(f32)
    x = x.astype(f32)
    z = (x * f32(0.7071067811865476)).astype(f32)
    a = np.minimum(np.abs(z), f32(hi))
    q = np.full_like(a, f32(c[-1]))
    for k in c[-2::-1]:
        q = fma(q, a, np.full_like(a, f32(k)))
    q = fma(a, q, a)
    ex = np.exp2((-q * f32(1.4426950408889634)).astype(f32).astype(np.float64)).astype(f32)
    e = np.copysign((f32(1) - ex).astype(f32), z)
    return (f32(0.5) * x * (f32(1) + e)).astype(f32)


def main():
    c = fit()
    print("coefficients, highest degree first:")
    for k in c[::-1]:
        print(f"  {float(f32(k)): .9e}  0x{struct.unpack('<I', struct.pack('<f', f32(k)))[0]:08x}")
    x = np.concatenate([np.linspace(-12, 12, 2_000_001),
                        np.random.default_rng(0).normal(0, 3, 2_000_000)]).astype(f32)
    xd = x.astype(np.float64)
    truth = 0.5 * xd * (1 + erf64(xd / np.sqrt(2)))
    new = gelu_emulated(x, c).astype(np.float64)
    formula = (f32(0.5) * x * (f32(1) + erf64(xd / np.sqrt(2)).astype(f32))).astype(np.float64)
    floor = np.abs(xd) * 2.0 ** -24 + 1e-38
    print("max |err| / (|x| 2^-24): new", (np.abs(new - truth) / floor).max(),
          " f32 formula with exact erf", (np.abs(formula - truth) / floor).max())
    print("bit-identical to the f32 formula with exact erf:", np.mean(new == formula))


if __name__ == "__main__":
    main()
