"""Split attention at equal work, growing row length (GPU): B x L^2 held at config 2's 32 x 499^2, 12 heads of 64,
so a longer row means fewer, longer query blocks per (batch, head).  What the L = 499 point loses against the long
rows is the per-block cost (prologue loads, epilogue stores, the padded last tile).  ``--modes``:
hfa_attention_split_tuning values to compare (0 = automatic, 4 / 8 waves).
    python scripts/attn_len_sweep.py [--reps 200] [--modes 0,4,8] [--lengths 499,14999]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import _lib, ops  # noqa: E402

CEIL = 2516.6 / 3.0     # f32-equivalent ceiling of the 3-product split scheme (TFLOP/s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--modes", default="0")
    ap.add_argument("--lengths", default="499,704,998,1411,1996,3992,7984",
                    help="row lengths (B = 32 x 499^2 / L^2, at least 1); 14999 = config 5's 300 s utterance")
    ap.add_argument("--batch", type=int, default=0, help="fixed batch instead of equal work (0: equal work)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, dh = 12, 64
    work = 32 * 499 * 499
    g = torch.Generator(device=dev).manual_seed(0)
    for L in (int(v) for v in a.lengths.split(",")):
        B = a.batch if a.batch > 0 else max(1, round(work / (L * L)))
        x = torch.randn(B, L, 3 * H * dh, device=dev, generator=g) * 0.5
        qs = ops.split(x)
        o = torch.empty(2, B, L, H * dh, dtype=torch.float16, device=dev)
        run = lambda: ops.attention_split(qs, o, B=B, H=H, L=L, head_dim=dh, scale=0.125)  # noqa: E731
        for mode in (int(m) for m in a.modes.split(",")):
            _lib.call("hfa_attention_split_tuning", mode)
            try:
                for _ in range(20):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run()
                e1.record()
                torch.cuda.synchronize()
            finally:
                _lib.call("hfa_attention_split_tuning", 0)
            ms = e0.elapsed_time(e1) / a.reps
            fl = 4.0 * B * H * L * L * dh
            print(f"mode {mode:3d} L={L:5d} B={B:3d} tiles/block={math.ceil(L / 64):4d} blocks={B * H * math.ceil(L / 128):5d}:"
                  f" {ms * 1e3:8.1f} us {fl / ms / 1e9:6.1f} TF/s f32-eq  {fl / ms / 1e9 / CEIL:.3f} of the split ceiling",
                  flush=True)


if __name__ == "__main__":
    main()
