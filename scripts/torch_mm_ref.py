"""Reference point (GPU box): torch.mm fp32 (hipBLASLt/rocBLAS) on the workload's Linear shapes, next to ours."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
for name, M, N, K in (("qkv", 15968, 2304, 768), ("outproj", 15968, 768, 768), ("ffn1", 15968, 3072, 768),
                      ("ffn2", 15968, 768, 3072), ("square4k", 4096, 4096, 4096)):
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    res = {}
    for tag, fn in (("torch.mm", lambda: torch.mm(a, w.t())), ("hfa", lambda: ops.linear(a, w))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[tag] = 2.0 * M * N * K / ms / 1e9
    print(f"{name:9s} torch.mm {res['torch.mm']:6.1f} TFLOP/s   hfa {res['hfa']:6.1f} TFLOP/s", flush=True)
