"""Vendor f16 GEMM (torch.mm -> hipBLASLt) on the workload's Linear/conv-as-GEMM shapes, as a ceiling reference
for the split-f16 kernel (3 f16 products per f32 MAC): python scripts/f16_mm_ref.py"""
import torch

B = 32
SHAPES = [("conv1", 15999, 1536, 512), ("conv5", 999, 1024, 512), ("qkv", 499, 768, 2304),
          ("outproj", 499, 768, 768), ("ffn1", 499, 768, 3072), ("ffn2", 499, 3072, 768)]


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


dev = torch.device("cuda")
for name, T, K, N in SHAPES:
    a = torch.randn(B * T, K, device=dev, dtype=torch.half)
    w = torch.randn(N, K, device=dev, dtype=torch.half)
    o = torch.empty(B * T, N, device=dev, dtype=torch.half)
    ms = timeit(lambda: torch.mm(a, w.t(), out=o))
    fl = 2.0 * B * T * K * N
    print(f"{name:8s} f16 torch.mm {fl / ms / 1e9:7.1f} TF ({ms:.3f} ms); /3 = {fl / ms / 3e9:6.1f} f32-eq TF", flush=True)
