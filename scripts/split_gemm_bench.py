"""Split-f16 GEMM vs f32-MFMA GEMM on the workload's shapes (GPU box): accuracy against an f64 evaluation and
speed.  python scripts/split_gemm_bench.py [--reps 20] [--cfgs 0,1,2,3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402

B = 32
SHAPES = [  # name, Tin, Cin, Cout, k, stride, epi
    ("conv1", 31999, 512, 512, 3, 2, 1),
    ("conv5", 1999, 512, 512, 2, 2, 1),
    ("conv6", 999, 512, 512, 2, 2, 1),
    ("conv4", 3999, 512, 512, 3, 2, 1),
    ("qkv", 499, 768, 2304, 1, 1, 0),
    ("outproj", 499, 768, 768, 1, 1, 0),
    ("ffn1", 499, 768, 3072, 1, 1, 1),
    ("ffn2", 499, 3072, 768, 1, 1, 0),
    # UNet (T padded to 864 at 86.13 fps, pad 1 for the k3 convs: shapes only, the pad is ignored here)
    ("unet_k3_768", 866, 768, 192, 3, 1, 0),
    ("unet_k3_192", 866, 192, 192, 3, 1, 0),
    ("unet_sc", 864, 768, 192, 1, 1, 0),
    ("unet_down", 864, 192, 384, 2, 2, 0),
    ("unet_up", 216, 384, 384, 1, 1, 0),
    # flattened [B*T] rows as the encoder launches them (Z = 1): config 2 (32 x 499) and config 5 in 20 s windows
    # (15 windows x ~1195 frames)
    ("qkv_c2", 15968, 768, 2304, 1, 1, 0, 1),
    ("ffn1_c2", 15968, 768, 3072, 1, 1, 1, 1),
    ("qkv_c5", 17924, 768, 2304, 1, 1, 0, 1),
    ("ffn1_c5", 17924, 768, 3072, 1, 1, 1, 1),
    ("ffn2_c5", 17924, 3072, 768, 1, 1, 0, 1),
    ("outproj_c5", 17924, 768, 768, 1, 1, 0, 1),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cfgs", default="0,1,2,3")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--epi", action="store_true", help="epilogue ablation: GELU vs none, f32 vs planes out")
    args = ap.parse_args()
    keep = set(args.shapes.split(",")) if args.shapes else None
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for shape in SHAPES:
        name, Tin, Cin, Cout, k, s, epi = shape[:7]
        B = shape[7] if len(shape) > 7 else globals()["B"]
        if keep and name not in keep:
            continue
        Tout = (Tin - k) // s + 1
        K = k * Cin
        x = torch.randn(B, Tin, Cin, device=dev, generator=g)
        w = torch.randn(Cout, K, device=dev, generator=g) * K ** -0.5
        b = torch.randn(Cout, device=dev, generator=g) * 0.1
        y32 = torch.empty(B, Tout, Cout, device=dev)
        ys = torch.empty(B, Tout, Cout, device=dev)
        xs, ws = ops.split(x), ops.split(w)
        kw = dict(M=Tout, N=Cout, K=K, Zb=B, sAb=Tin * Cin, ldx=Cin, stride=s, Cg=Cin, Tin=Tin, bias=b,
                  sCb=Tout * Cout, ldc=Cout, epilogue=epi)
        f32 = lambda: ops.conv_gemm(x, w, y32, **kw)  # noqa: E731
        spl = lambda: ops.conv_gemm_split(xs, ws, C=ys, **kw)  # noqa: E731
        f32()
        spl()
        torch.cuda.synchronize()
        # f64 reference on a row sample
        rows = torch.arange(0, Tout, max(1, Tout // 64), device=dev)
        bsel = torch.tensor([0, B - 1], device=dev)
        xw = torch.stack([x[:, rows * s + j] for j in range(k)], dim=-2)[bsel].double()   # [2, R, k, Cin]
        ref = xw.reshape(2, len(rows), K) @ w.double().t() + b.double()
        if epi:
            ref = torch.nn.functional.gelu(ref)
        e32 = (y32[bsel][:, rows].double() - ref).abs().max().item()
        es = (ys[bsel][:, rows].double() - ref).abs().max().item()
        flops = 2.0 * B * Tout * Cout * K
        ms32 = timeit(f32, args.reps)
        line = f"{name:8s} f32 {flops / ms32 / 1e9:6.1f} TF ({ms32:.3f} ms) err {e32:.1e} | split err {es:.1e}"
        for cfg in (int(c) for c in args.cfgs.split(",")):
            _lib.lib().hfa_gemm_split_tuning(cfg)
            ys.zero_()
            spl()
            ec = (ys[bsel][:, rows].double() - ref).abs().max().item()
            ms = timeit(spl, args.reps)
            line += f" | cfg{cfg} {flops / ms / 1e9:6.1f} TF e{ec:.0e}"
        _lib.lib().hfa_gemm_split_tuning(0)
        if args.epi:
            ysp = torch.empty(2, B, Tout, Cout, dtype=torch.float16, device=dev)
            for e_ in (1, 0):
                kw2 = dict(kw, epilogue=e_)
                t_c = timeit(lambda: ops.conv_gemm_split(xs, ws, C=ys, **kw2), args.reps)
                t_p = timeit(lambda: ops.conv_gemm_split(xs, ws, Cs=ysp, **kw2), args.reps)
                line += f" | epi{e_}: f32-out {t_c:.3f} ms, planes-out {t_p:.3f} ms"
        print(line, flush=True)


if __name__ == "__main__":
    main()
