"""Bit-identity check of hfa_attention_split between two libhfa builds (run once per build, then --compare).

HFA_LIB=<lib> python scripts/attn_ab_check.py --tag cur|alt     -> gpurun_out/attn_out_<tag>.pt
python scripts/attn_ab_check.py --compare cur alt               -> max |diff| and differing-element counts
Seeded inputs: the workload shapes (base, large), a variable-length batch, tiny and odd lengths, a long row.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

CASES = [(32, 12, 499, None), (32, 16, 499, None), (4, 12, 700, [700, 513, 64, 1]), (2, 12, 63, None),
         (2, 12, 65, None), (3, 12, 130, [130, 129, 128]), (1, 12, 4999, None)]


def run(tag):
    from hubertfa_amd import ops
    d = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1234)
    outs = {}
    for i, (B, H, L, lens) in enumerate(CASES):
        D = 64
        qkv = (torch.randn(B, L, 3 * H * D, generator=g) * 2.0).to(d)
        qs = ops.split(qkv)
        o = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)
        kl = torch.tensor(lens, dtype=torch.int32, device=d) if lens else None
        ops.attention_split(qs, o, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5, key_len=kl)
        torch.cuda.synchronize()
        outs[i] = o.cpu()
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(outs, f"gpurun_out/attn_out_{tag}.pt")
    print("saved", tag, len(outs))


def compare(a, b):
    A = torch.load(f"gpurun_out/attn_out_{a}.pt", weights_only=True)
    Bo = torch.load(f"gpurun_out/attn_out_{b}.pt", weights_only=True)
    bad = 0
    for i in A:
        x, y = A[i], Bo[i]
        ndiff = int((x.view(torch.int16) != y.view(torch.int16)).sum())
        md = float((x[0].float() + x[1].float() / 2048 - y[0].float() - y[1].float() / 2048).abs().max())
        print(f"case {i} {CASES[i][:3]} differing halves {ndiff} max|diff| {md:.3e}")
        bad += ndiff
    print("BIT-IDENTICAL" if bad == 0 else "DIFFERENT")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        compare(*a.compare)
    else:
        run(a.tag)
