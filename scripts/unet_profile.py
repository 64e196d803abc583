"""Per-op time of the fused UNet kernel (workgroup 0's s_memrealtime at each op boundary, hfa_unet_profile) at the
bench geometry: python scripts/unet_profile.py [--B 32]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    args = ap.parse_args()
    from hubertfa_amd import _lib, ops
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    T = task.head.padded_len(861)
    x = torch.randn(args.B, T, 768, device=d) * 0.5
    fp = task.head.fused
    for _ in range(3):
        task.head.logits(x)
    buf = torch.zeros(fp.nops + 1, dtype=torch.int64, device=d)
    _lib.call("hfa_unet_profile", ops._ptr(buf))
    task.head.logits(x)
    torch.cuda.synchronize()
    t = buf.cpu().numpy()
    names = {0: "conv1", 1: "conv2", 2: "down", 3: "up", 4: "head"}
    tot = (t[-1] - t[0]) / 100.0
    print(f"fused UNet, workgroup 0, T={T}: {tot * 1e-3:.3f} ms")
    for k, o in enumerate(fp.ops):
        us = (t[k + 1] - t[k]) / 100.0
        fl = sum(2.0 * (T >> o["level"]) * o["n"] * sg["taps"] * sg["cin"] for sg in o["segs"])
        print(f"  op {k:2d} {names[o['kind']]:5s} level {o['level']} N={o['n']:3d} K={[sg['taps'] * sg['cin'] for sg in o['segs']]}"
              f": {us:8.1f} us  {fl / us / 1e6:6.2f} TF/s f32-eq")


if __name__ == "__main__":
    main()
