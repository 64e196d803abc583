"""LayerNorm microbenchmark (GPU box): the encoder's post-LN shape [32 x 499, 768] f32 -> split planes only (the
pipelined step's layernorm_kernel<3>), and -> f32 + planes, against a plain f32 device copy of the same bytes;
HIP events over 200 launches.  Bit-identity of the outputs against HFA_LIB's reference build is checked by the
caller (scripts/archive/gpu_r04ae.sh saves them).    python scripts/ln_bench.py [--save out.pt]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", default=None)
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    d = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn((32 * 499, 768), generator=g) * 3).to(d)
    w = (1 + 0.1 * torch.randn(768, generator=g)).to(d)
    b = (0.1 * torch.randn(768, generator=g)).to(d)
    planes = torch.empty((2, 32 * 499, 768), dtype=torch.float16, device=d)
    y = torch.empty_like(x)
    flag = torch.zeros(1, dtype=torch.int32, device=d)

    def clock(fn, nbytes, label):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        print(f"{label}: {us:.2f} us, {nbytes / us / 1e6:.2f} TB/s", flush=True)
    nb = x.numel() * 4
    clock(lambda: ops.layernorm(x, w, b, 1e-5, out=False, out_split=planes, flag=flag), 2 * nb, "LN -> planes")
    clock(lambda: ops.layernorm(x, w, b, 1e-5, out=y, out_split=planes, flag=flag), 3 * nb, "LN -> f32 + planes")
    clock(lambda: ops.layernorm(x, w, b, 1e-5, out=y), 2 * nb, "LN -> f32")
    clock(lambda: y.copy_(x), 2 * nb, "copy f32")
    if args.save:
        ops.layernorm(x, w, b, 1e-5, out=y, out_split=planes, flag=flag)
        torch.save({"y": y.cpu(), "planes": planes.cpu()}, args.save)


if __name__ == "__main__":
    main()
