"""The UNet head + lattice decoder in isolation at the bench geometry (GPU box): wall time per batch with HIP
events, and the split / f32 GEMM FLOP rate.  python scripts/unet_bench.py [--reps 20] [--B 32]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=32)
    args = ap.parse_args()
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    T = task.head.padded_len(861)
    x = torch.randn(args.B, T, 768, device=d) * 0.5
    flops = task.head.flops(T) * args.B
    for prec, fused in (("split", True), ("split", False), ("f32", False), ("split", True)):
        task.head.precision = prec
        task.head.use_fused = fused
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
        print(f"head {prec}{' fused' if fused and prec == 'split' else ''}: {ms:.3f} ms per batch of {args.B} x {T} frames, {flops / ms / 1e9:.1f} TFLOP/s "
              f"({flops / 1e9:.1f} GFLOP)", flush=True)
    task.head.precision = "split"
    task.head.use_fused = False
    for tile in (0, 23, 19, 18, 17, 0):        # chip-wide backbone, forced split-GEMM tiles (gemm.hip SCFG index)
        task.head.unet_tile = tile
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
        print(f"head split chip-wide, backbone tile {tile}: {ms:.3f} ms per batch", flush=True)
    task.head.unet_tile = 0
    task.head.use_fused = True
    for B in (1, 8, 32, 64):          # fused: one workgroup per utterance
        xb = x[:1].expand(B, -1, -1).contiguous()
        for _ in range(2):
            task.head.logits(xb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            task.head.logits(xb)
        e1.record()
        torch.cuda.synchronize()
        print(f"fused B={B}: {e0.elapsed_time(e1) / args.reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
