"""Flash-attention microbenchmark on the workload's shapes (run on the GPU box).

python scripts/attn_bench.py [--reps 20] [--rounds 3]  -> median ms and TFLOP/s (4*B*H*L*L*64 algorithmic FLOPs)
per shape, f32 kernel and the split kernel in both MFMA forms (hfa_attention_split_form 32 / 16) x waves (auto, 4, 8)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402

SHAPES = [("base B32 L499", 32, 12, 499), ("large B32 L499", 32, 16, 499), ("long B1 L14999", 1, 12, 14999)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    d = torch.device("cuda")
    for name, B, H, L in SHAPES:
        D = 64
        qkv = torch.randn(B, L, 3 * H * D, device=d)
        out = torch.empty(B, L, H * D, device=d)

        qs = ops.split(qkv)
        os_ = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)

        def go_split():
            ops.attention_split(qs, os_, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5)

        def go():
            ops.attention(qkv, qkv[..., H * D:], qkv[..., 2 * H * D:], out, B=B, H=H, L=L, head_dim=D,
                          scale=D ** -0.5, q_bs=L * 3 * H * D, q_ld=3 * H * D, k_bs=L * 3 * H * D, k_ld=3 * H * D,
                          v_bs=L * 3 * H * D, v_ld=3 * H * D, o_bs=L * H * D, o_ld=H * D)
        arms = [("f32", go, 0, 0)] + [(f"mf{form}-{'auto' if nw == 0 else f'{nw}w'}", go_split, nw, form)
                                       for form in (32, 16) for nw in (0, 4, 8)]
        res = {a[0]: [] for a in arms}
        for _ in range(args.rounds):                  # interleaved rounds: clock drift hits every arm alike
            for tag, fn, nw, form in arms:
                _lib.call("hfa_attention_split_tuning", nw)
                _lib.call("hfa_attention_split_form", form)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[tag].append(e0.elapsed_time(e1) / args.reps)
                _lib.call("hfa_attention_split_tuning", 0)
                _lib.call("hfa_attention_split_form", 0)
        for tag, v in res.items():
            ms = sorted(v)[len(v) // 2]
            tf = 4.0 * B * H * L * L * D / ms / 1e9
            frac = tf / (2516.6 / 3) if tag != "f32" else tf / 157.3
            print(f"{name:16s} {tag:9s} {ms:8.4f} ms  {tf:7.1f} TFLOP/s  {frac:.3f} of its ceiling", flush=True)

if __name__ == "__main__":
    main()
