"""Fused residual GEMM + LayerNorm (ops.linear_split_ln) against the two launches it replaces (linear_split, then
layernorm with plane output) on config 2's shapes: out-projection (K = 768) and FFN2 (K = 3072), M = 32 x 499.
Median of 5 x --reps launches per form (run on the GPU box).  Needs the library and ops of commit 9c5bf4c (the fused
form was measured slower and reverted: profiles/r05/fused_ln_ab.txt)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    d = torch.device("cuda")
    M, N = 32 * 499, 768
    for name, K in (("out-proj", 768), ("FFN2", 3072), ("large out-proj", 1024)):
        n = 1024 if name.startswith("large") else N
        xs = ops.split(torch.randn(M, K, device=d))
        ws = ops.split(torch.randn(n, K, device=d) * K ** -0.5)
        b, g, be = torch.randn(n, device=d), torch.ones(n, device=d), torch.zeros(n, device=d)
        rs = ops.split(torch.randn(M, n, device=d))
        gemm = lambda: ops.linear_split(xs, ws, b, residual=rs)  # noqa: E731
        y = gemm()
        ln = lambda: ops.layernorm(y, g, be, 1e-5, out=False, out_split=True)  # noqa: E731
        two = lambda: ops.layernorm(gemm(), g, be, 1e-5, out=False, out_split=True)  # noqa: E731
        one = lambda: ops.linear_split_ln(xs, ws, b, rs, g, be, 1e-5, out_f32=False, out_split=True)  # noqa: E731
        tg, tl, tt, to = (timeit(f, args.reps) for f in (gemm, ln, two, one))
        print(f"{name:15s} M={M} N={n} K={K}: gemm {tg:7.1f} us  layernorm {tl:6.1f}  two launches {tt:7.1f}  "
              f"fused {to:7.1f}  ({tt - to:+.1f} us)", flush=True)


if __name__ == "__main__":
    main()
