"""GEMM microbenchmark over the workload's shapes and tile variants (run on the GPU box).

python scripts/gemm_bench.py [--reps 20]  -> one line per (shape, variant): ms, TFLOP/s
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402

B = 32
SHAPES = [
    # name, Tin, Cin, Cout, k, stride, pad, G, epi, M(out rows)
    ("conv1", 31999, 512, 512, 3, 2, 0, 1, 1),
    ("conv3", 7999, 512, 512, 3, 2, 0, 1, 1),
    ("conv5", 1999, 512, 512, 2, 2, 0, 1, 1),
    ("qkv", 499, 768, 2304, 1, 1, 0, 1, 0),
    ("outproj", 499, 768, 768, 1, 1, 0, 1, 0),
    ("ffn1", 499, 768, 3072, 1, 1, 0, 1, 1),
    ("ffn2", 499, 3072, 768, 1, 1, 0, 1, 0),
    ("posconv", 499, 768, 768, 128, 1, 64, 16, 1),
    ("unet_k3", 864, 192, 192, 3, 1, 1, 1, 0),
]


def run(shape, bk, cfg, reps):
    name, Tin, Cin, Cout, k, s, pad, G, epi = shape
    dev = torch.device("cuda")
    Tout = (Tin + 2 * pad - k) // s + 1
    if name == "posconv":
        Tout = Tin
    Cg, Ng = Cin // G, Cout // G
    x = torch.randn(B, Tin, Cin, device=dev)
    w = torch.randn(Cout, k * Cg, device=dev) * (k * Cg) ** -0.5
    b = torch.randn(Cout, device=dev)
    y = torch.empty(B, Tout, Cout, device=dev)
    _lib.lib().hfa_gemm_tuning(bk, cfg)

    def go():
        ops.conv_gemm(x, w, y, M=Tout, N=Ng, K=k * Cg, Zb=B, G=G, sAb=Tin * Cin, sAg=Cg, ldx=Cin, stride=s, pad=pad,
                      Cg=Cg, Tin=Tin, sWg=Ng * k * Cg, bias=b, sBg=Ng, sCb=Tout * Cout, sCg=Ng, ldc=Cout,
                      epilogue=epi)
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * B * Tout * Cout * k * Cg
    return ms, flops / ms / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="16:1,16:2,16:4,103:1,103:2,103:4",
                    help="pipe:cfg pairs; pipe 16/32 register-staged BK, 102/103 LDS-DMA 2/3 stages")
    ap.add_argument("--shapes", default="", help="comma-separated subset of shape names")
    ap.add_argument("--epi", type=int, default=-1, help="force the epilogue (0 none, 1 GELU) on every shape")
    args = ap.parse_args()
    keep = set(args.shapes.split(",")) if args.shapes else None
    names = {0: "auto", 1: "128x128/2x2", 2: "128x64/2x2", 3: "256x128/4x2", 4: "128x256/2x4", 5: "256x128/2x2",
             6: "128x256/2x2", 7: "256x256/4x2", 8: "128x48/4x1", 9: "128x96/4x1"}
    variants = [tuple(int(v) for v in s.split(":")) for s in args.variants.split(",")]
    for shape in SHAPES:
        if keep is not None and shape[0] not in keep:
            continue
        for bk, cfg in variants:
            if bk == 32 and (shape[2] // shape[7]) % 32:
                continue
            if args.epi >= 0:
                shape = shape[:8] + (args.epi,)
            ms, tf = run(shape, bk, cfg, args.reps)
            pipe = {0: "auto", 16: "reg16", 32: "reg32", 102: "dma2", 103: "dma3"}.get(bk, str(bk))
            print(f"{shape[0]:10s} {pipe:6s} {names[cfg]:12s} {ms:8.3f} ms  {tf:7.1f} TFLOP/s", flush=True)
    _lib.lib().hfa_gemm_tuning(0, 0)


if __name__ == "__main__":
    main()
