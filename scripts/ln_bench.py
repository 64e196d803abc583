"""LayerNorm microbenchmark at the encoder's shape (32 x 499 rows x 768, planes out, as the post-LN layers call it)
and a bit-identity check of the rows-per-wave kernel against the one-row kernel (GPU box):
HFA_LN_ROWS=0|1 python scripts/ln_bench.py  (prints ms, GB/s and an output checksum)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402


def main():
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    for rows, C in ((15968, 768), (15968, 1024)):
        x = torch.randn(rows, C, device=d, generator=g) * 3 + 1
        gm = torch.randn(C, device=d, generator=g)
        bt = torch.randn(C, device=d, generator=g)
        planes = torch.empty((2, rows, C), dtype=torch.float16, device=d)
        fn = lambda: ops.layernorm(x, gm, bt, 1e-5, out=False, out_split=planes)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 50
        gb = rows * C * (4 + 4) / 1e9
        ck = int(planes.view(torch.int16).to(torch.int64).sum().item())
        print(f"rows {rows} C {C}: {ms * 1e3:.1f} us, {gb / ms:.0f} GB/s, checksum {ck}", flush=True)


if __name__ == "__main__":
    main()
