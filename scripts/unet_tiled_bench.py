"""The UNet head alone at the bench geometry (B = 32 x 864 padded frames): chip-wide launches vs the tiled op
engine, HIP events per batch.  python scripts/unet_tiled_bench.py [--reps 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    head = task.head
    for B, T in ((32, 864), (1, 25840)):
        x = torch.randn(B, T, 768, device=d) * 0.5
        flops = head.flops(T) * B
        for name, fn in (("chip-wide", lambda: head._chipwide(x)),
                         ("tiled", lambda: head.fused(x, [T] * B, head.ctx.flag, tiled=True)),
                         ("chip-wide", lambda: head._chipwide(x))):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(f"B={B} T={T} {name}: {ms:.3f} ms per batch, {flops / ms / 1e9:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
