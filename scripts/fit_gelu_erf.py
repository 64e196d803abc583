"""Fit of the GELU epilogue's erfc (hfa::gelu_fast in hubertfa_amd/csrc/hfa_common.h) and its f32 accuracy check.

GELU(x) = max(x, 0) - |x / 2| E with E = erfc(|x| / sqrt 2) = exp2(q(a)), a = min(|x|, 3.95 sqrt 2),
q(a) = a R7(a) ~ log2 erfc(a / sqrt 2), fitted by least squares weighted by the absolute error of E (erfc-weighted),
iteratively re-weighted toward minimax.  Prints the f32 hex coefficients (highest degree first, Horner order of the
kernel) and the f32-emulated GELU error against fp64, next to the round-1/2 form 0.5 x (1 + sign(z)(1 - exp(-q(|z|)))).

python scripts/fit_gelu_erf.py
"""
import struct

import numpy as np
from scipy.special import erf as erf64, erfc as erfc64

f32 = np.float32
S2 = np.sqrt(2.0)
HI = 3.95                 # clamp in z = x / sqrt 2 units: f32 erf(3.95) is already 1


def fma(a, b, d):
    """f32 fma (the product exact in f64)."""
    return (a.astype(np.float64) * b.astype(np.float64) + d.astype(np.float64)).astype(f32)


def _irls(A, y, w, scale, iters):
    sw = w * scale
    c, *_ = np.linalg.lstsq(A * sw[:, None], y * sw, rcond=None)
    for _ in range(iters):          # multiplicative re-weighting toward the minimax solution
        r = np.abs((A @ c - y) * sw)
        w = w * (1 + 20 * r / r.max())
        w = w / w.max()
        sw = w * scale
        c, *_ = np.linalg.lstsq(A * sw[:, None], y * sw, rcond=None)
    return c


def fit(deg=7, n=400001, iters=30):
    """q(a) = a R7(a) ~ log2 erfc(a / sqrt 2) on (0, 3.95 sqrt 2]; coefficients lowest degree first."""
    a = np.linspace(0, HI * S2, n)[1:]
    target = np.log2(erfc64(a / S2))
    A = np.vstack([a ** k for k in range(deg + 1)]).T
    return _irls(A, target / a, erfc64(a / S2), a, iters)


def gelu_emulated(x, r):
    """The kernel's f32 arithmetic (fma exact via f64; v_exp_f32 ~ correctly rounded exp2)."""
    x = x.astype(f32)
    a = np.minimum(np.abs(x), f32(HI * S2))
    q = np.full_like(a, f32(r[-1]))
    for k in r[-2::-1]:
        q = fma(q, a, np.full_like(a, f32(k)))
    e = np.exp2((a * q).astype(f32).astype(np.float64)).astype(f32)
    return fma(-np.abs((f32(0.5) * x).astype(f32)), e, np.maximum(x, f32(0)))


def fit_round1(deg=8, n=400001, iters=30):
    """The round-1/2 form: q(z) = z + z P8(z) ~ -log(1 - erf(z)) on (0, 3.95]."""
    zs = np.linspace(0, HI, n)[1:]
    target = -np.log1p(-erf64(zs))
    A = np.vstack([zs ** k for k in range(deg + 1)]).T
    return _irls(A, (target - zs) / zs, np.exp(-target), zs, iters)


def gelu_round1(x, c):
    x = x.astype(f32)
    z = (x * f32(0.7071067811865476)).astype(f32)
    a = np.minimum(np.abs(z), f32(HI))
    q = np.full_like(a, f32(c[-1]))
    for k in c[-2::-1]:
        q = fma(q, a, np.full_like(a, f32(k)))
    q = fma(a, q, a)
    ex = np.exp2((-q * f32(1.4426950408889634)).astype(f32).astype(np.float64)).astype(f32)
    e = np.copysign((f32(1) - ex).astype(f32), z)
    return (f32(0.5) * x * (f32(1) + e)).astype(f32)


def main():
    r = fit()
    print("coefficients of R7, highest degree first:")
    for k in r[::-1]:
        print(f"  {float(f32(k)): .9e}  0x{struct.unpack('<I', struct.pack('<f', f32(k)))[0]:08x}")
    x = np.concatenate([np.linspace(-12, 12, 2_000_001),
                        np.random.default_rng(0).normal(0, 3, 2_000_000)]).astype(f32)
    xd = x.astype(np.float64)
    truth = 0.5 * xd * (1 + erf64(xd / S2))
    floor = np.abs(xd) * 2.0 ** -24 + 1e-38
    m = xd > -1.5
    ulp = np.spacing(np.abs(truth[m]).astype(f32)).astype(np.float64)
    formula = (f32(0.5) * x * (f32(1) + erf64(xd / S2).astype(f32))).astype(np.float64)
    for name, y in (("gelu_fast", gelu_emulated(x, r)), ("round-1 form", gelu_round1(x, fit_round1())),
                    ("f32 formula, exact erf", formula)):
        err = np.abs(y.astype(np.float64) - truth)
        print(f"{name}: max |err| / (|x| 2^-24) {(err / floor).max():.3f}, max ulp where x > -1.5 "
              f"{(err[m] / ulp).max():.2f}")


if __name__ == "__main__":
    main()
