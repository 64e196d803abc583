"""Split-attention microbenchmark for library A/Bs (HFA_LIB selects the build): ms per launch on the workload's
shapes, median of 5 repeats of --reps launches each (run on the GPU box)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops  # noqa: E402

SHAPES = [("base B32 L499", 32, 12, 499), ("large B32 L499", 32, 16, 499), ("long B1 L14999", 1, 12, 14999)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tag", default=os.environ.get("HFA_LIB", "cur"))
    args = ap.parse_args()
    d = torch.device("cuda")
    for name, B, H, L in SHAPES:
        D = 64
        qs = ops.split(torch.randn(B, L, 3 * H * D, device=d))
        os_ = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)

        def go():
            ops.attention_split(qs, os_, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5)
        reps = max(4, args.reps // (30 if L > 5000 else 1))
        for _ in range(3):
            go()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                go()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / reps)
        ms = sorted(ts)[2]
        print(f"{os.path.basename(os.path.dirname(args.tag)) or args.tag:10s} {name:16s} {ms:8.4f} ms "
              f"{4.0 * B * H * L * L * D / ms / 1e9:7.1f} TF/s  {4.0 * B * H * L * L * D / ms / 1e9 / 838.87:.3f}",
              flush=True)


if __name__ == "__main__":
    main()
