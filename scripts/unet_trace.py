"""The chip-wide UNet head alone (split precision), 10 batches at the bench geometry, for a rocprof kernel trace:
rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 scripts/unet_trace.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.head.use_fused = os.environ.get("HFA_UNET_FUSED", "0") == "1"
    x = torch.randn(32, 864, 768, device=d) * 0.5
    for _ in range(13):
        task.head.logits(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
