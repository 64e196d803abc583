"""The encoder layer's four split GEMMs exactly as hubert.py launches them at config 2 (B*L = 15968 rows, planes in;
QKV and FFN1 write planes, the out-projection and FFN2 add the LayerNorm's residual planes into f32), timed alone
with HIP events, plus the split attention: python scripts/layer_gemm_bench.py [--reps 50] [--rows 15968]."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402

SPLIT_PEAK = 2516.6 / 3


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
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rows", type=int, default=15968)
    ap.add_argument("--H", type=int, default=768)
    ap.add_argument("--F", type=int, default=3072)
    ap.add_argument("--cfgs", default="0", help="split GEMM tile overrides (hfa_gemm_split_tuning), 0 = automatic")
    ap.add_argument("--dump", default=None, help="write the GEMMs' output digests (sha256) here: A/B bit checks")
    args = ap.parse_args()
    d = torch.device("cuda")
    g = torch.Generator(device=d).manual_seed(0)
    M, H, F = args.rows, args.H, args.F
    r = lambda *s, sc=1.0: torch.randn(*s, device=d, generator=g) * sc  # noqa: E731
    xs = ops.split(r(M, H))                 # LayerNorm-like planes (the residual stream)
    fs = ops.split(r(M, F, sc=0.5))         # FFN1's GELU planes
    os_ = ops.split(r(M, H, sc=0.5))        # attention output planes
    w = {n: ops.split(r(*s, sc=s[1] ** -0.5)) for n, s in
         (("qkv", (3 * H, H)), ("o", (H, H)), ("f1", (F, H)), ("f2", (H, F)))}
    b = {n: r(s, sc=0.1) for n, s in (("qkv", 3 * H), ("o", H), ("f1", F), ("f2", H))}
    qkv_out = torch.empty((2, M, 3 * H), dtype=torch.float16, device=d)
    f1_out = torch.empty((2, M, F), dtype=torch.float16, device=d)
    y = torch.empty((M, H), device=d)
    cases = [
        ("QKV (planes out)", 2.0 * M * 3 * H * H,
         lambda: ops.linear_split(xs, w["qkv"], b["qkv"], out=qkv_out, out_split=True)),
        ("out-proj (+res planes)", 2.0 * M * H * H,
         lambda: ops.linear_split(os_, w["o"], b["o"], residual=xs, out=y)),
        ("FFN1 (GELU, planes out)", 2.0 * M * F * H,
         lambda: ops.linear_split(xs, w["f1"], b["f1"], out=f1_out, out_split=True, epilogue=ops.EPI_GELU)),
        ("FFN2 (+res planes)", 2.0 * M * H * F,
         lambda: ops.linear_split(fs, w["f2"], b["f2"], residual=xs, out=y)),
    ]
    B, L = 32, M // 32
    if B * L == M:
        qs = ops.split(r(B, L, 3 * H))
        o = torch.empty((2, B, L, H), dtype=torch.float16, device=d)
        cases.append(("attention (split)", 4.0 * B * H * L * L,
                      lambda: ops.attention_split(qs, o, B=B, H=H // 64, L=L, head_dim=64, scale=0.125)))

        def attn8():
            _lib.lib().hfa_attention_split_tuning(8)
            ops.attention_split(qs, o, B=B, H=H // 64, L=L, head_dim=64, scale=0.125)
            _lib.lib().hfa_attention_split_tuning(0)
        cases.append(("attention (split, 8 waves)", 4.0 * B * H * L * L, attn8))
    if args.dump:
        import hashlib
        import json
        dig = {}
        for (name, _, fn), out in zip(cases[:4], (qkv_out, y, f1_out, y)):
            fn()
            torch.cuda.synchronize()
            dig[name] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
        with open(args.dump, "w") as f:
            json.dump(dig, f, indent=1)
    for cfg in [int(c) for c in args.cfgs.split(",")]:
        _lib.lib().hfa_gemm_split_tuning(cfg)
        for name, flop, fn in cases:
            if cfg and name.startswith("attention"):
                continue
            ms = timeit(fn, args.reps)
            tf = flop / (ms * 1e-3) / 1e12
            print(f"cfg {cfg:2d} {name:26s} {ms * 1e3:8.1f} us  {tf:6.1f} TF/s f32-eq  {tf / SPLIT_PEAK:.3f} of the "
                  f"split ceiling", flush=True)
        _lib.lib().hfa_gemm_split_tuning(0)


if __name__ == "__main__":
    main()
