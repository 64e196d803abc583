"""The UNet head in isolation at the bench geometry (GPU box): wall time per batch with HIP events, on the split
path (automatic tiles, and the backbone GEMMs forced onto one split-GEMM tile: the gemm.hip SCFG index) and on the
f32 MFMA path.   python scripts/unet_bench.py [--reps 20] [--B 32] [--tiles 0,18,25]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--tiles", default="0")
    args = ap.parse_args()
    from hubertfa_amd import _lib
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    T = task.head.padded_len(861)
    x = torch.randn(args.B, T, 768, device=d) * 0.5
    flops = task.head.flops(T) * args.B

    def clock(label):
        for _ in range(3):
            task.head.logits(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            task.head.logits(x)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(f"head {label}: {ms:.3f} ms per batch of {args.B} x {T} frames, {flops / ms / 1e9:.1f} TFLOP/s "
              f"({flops / 1e9:.1f} GFLOP)", flush=True)

    for tile in (int(t) for t in args.tiles.split(",")):
        _lib.lib().hfa_gemm_split_tuning(tile)
        try:
            clock(f"split, tile {tile}")
        finally:
            _lib.lib().hfa_gemm_split_tuning(0)
    task.head.precision = "f32"
    clock("f32")
    task.head.precision = "split"


if __name__ == "__main__":
    main()
