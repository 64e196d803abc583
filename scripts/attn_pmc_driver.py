"""The config-2 split attention alone (B=32, L=499, 12 heads of 64), 20 launches: a short program for rocprofv3 PMC
passes (scripts/archive/gpu_r04p.sh).   python scripts/attn_pmc_driver.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402


def main():
    d = torch.device("cuda")
    B, L, H, dh = 32, 499, 12, 64
    g = torch.Generator(device=d).manual_seed(0)
    qs = ops.split(torch.randn(B, L, 3 * H * dh, device=d, generator=g) * 0.5)
    o = torch.empty(2, B, L, H * dh, dtype=torch.float16, device=d)
    for _ in range(20):
        ops.attention_split(qs, o, B=B, H=H, L=L, head_dim=dh, scale=0.125)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
