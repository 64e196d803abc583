"""conv0 + GroupNorm + GELU (split-plane output) at the bench geometry (GPU box): the shipped kernels (lag-product
statistics + the packed f16-MFMA apply pass, conv.hip); the round-3 alternatives are in git history.
python scripts/conv0_bench.py [--reps 20] [--B 32] [--seconds 10]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    args = ap.parse_args()
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    N = int(16000 * args.seconds)
    x = torch.randn(args.B, N, device=d, generator=g) * 0.1
    w0 = torch.randn(512, 10, device=d, generator=g) * 0.3
    gam, bet = 1 + 0.1 * torch.randn(512, device=d, generator=g), 0.1 * torch.randn(512, device=d, generator=g)
    T0 = (N - 10) // 5 + 1
    out = torch.empty(2, args.B, T0, 512, dtype=torch.float16, device=d)
    ws = torch.empty(_lib.lib().hfa_conv0_workspace_bytes(args.B, N), dtype=torch.uint8, device=d)
    nbytes = args.B * (4.0 * N + 4.0 * 512 * T0)
    for rep in range(3):
        fn = lambda: ops.conv0(x, w0, gamma=gam, beta=bet, out=out, workspace=ws, out_split=True)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(f"run {rep}: {ms:.3f} ms per batch (stats + apply), "
              f"{nbytes / ms / 1e6:.0f} GB/s of algorithmic bytes", flush=True)


if __name__ == "__main__":
    main()
