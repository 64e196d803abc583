"""Grouped positional conv (k128, pad 64, 16 groups, Cg = 48 at Hubert-base) on the f32 MFMA GEMM vs the split-f16
GEMM's general-tap path, B=32 x 499 frames: python scripts/posconv_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402


def timeit(fn, reps=20):
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


d = torch.device("cuda")
for H, G in ((768, 16), (1024, 16)):
    B, L, k = 32, 499, 128
    Cg = H // G
    x = torch.randn(B, L, H, device=d)
    w = torch.randn(H, k * Cg, device=d) * (k * Cg) ** -0.5
    b = torch.randn(H, device=d) * 0.1
    out = torch.empty_like(x)
    kw = dict(M=L, N=Cg, K=k * Cg, Zb=B, G=G, sAb=L * H, sAg=Cg, ldx=H, stride=1, pad=k // 2, Cg=Cg, Tin=L,
              sWg=Cg * k * Cg, bias=b, sBg=Cg, R=x, sRb=L * H, sRg=Cg, ldr=H, sCb=L * H, sCg=Cg, ldc=H,
              epilogue=ops.EPI_GELU)
    ws = ops.split(w)
    fl = 2.0 * B * L * H * Cg * k
    ms32 = timeit(lambda: ops.conv_gemm(x, w, out, **kw))
    line = f"H={H} Cg={Cg}: f32 {ms32:.3f} ms ({fl / ms32 / 1e9:.0f} TF)"
    xs = ops.split(x)
    for cfg in (0, 10, 14, 15, 16):
        _lib.lib().hfa_gemm_split_tuning(cfg)
        mss = timeit(lambda: ops.conv_gemm_split(xs, ws, C=out, **kw))
        line += f" | cfg{cfg} {mss:.3f} ms ({fl / mss / 1e9:.0f} TF)"
    _lib.lib().hfa_gemm_split_tuning(0)
    print(line, flush=True)
