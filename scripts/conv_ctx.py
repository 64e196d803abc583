"""Extractor convs in context: each split conv's time inside the real encoder forward (HIP events per launch,
config-2 batch, synthetic weights and audio as bench.py) against the same launch repeated in isolation on the same
tensors (run on the GPU box).  Prints one line per conv: in-forward median us, isolated median us."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hubertfa_amd import ops, synth  # noqa: E402
from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint  # noqa: E402


def main():
    dev = torch.device("cuda")
    ck = synth_checkpoint(encoder="cnhubert", model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=dev)
    task.on_predict_start()
    enc = task.unitsEncoder.model
    B, n = 32, 160000
    wav = torch.from_numpy(np.stack([synth.synth_audio(n, 16000, seed=i) for i in range(B)])).to(dev)

    calls = []                                     # (M, launch closure) of every split conv in one forward
    orig = ops.conv_gemm_split

    def spy(*a, **kw):
        r = orig(*a, **kw)
        calls.append((kw.get("M"), kw.get("K"), kw.get("Zb", 1), lambda: orig(*a, **kw)))
        return r

    times = {}

    class Probe:
        def __call__(self, name, work, launch, kind="flops", shape=None, units=None, label=None):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            launch()
            e.record()
            times.setdefault((name, work), []).append((s, e))

    with torch.no_grad():
        for _ in range(3):
            enc(wav)
        torch.cuda.synchronize()
        ops.PROBE = Probe()
        for _ in range(8):
            enc(wav)
        torch.cuda.synchronize()
        ops.PROBE = None
        ops.conv_gemm_split = spy
        enc(wav)
        ops.conv_gemm_split = orig
        torch.cuda.synchronize()

        def med(v):
            v = sorted(v)
            return v[len(v) // 2]

        for M, K, Zb, go in calls:
            if M is None or Zb != B:
                continue
            flops = 2.0 * M * 512 * K * Zb
            inf = [s.elapsed_time(e) * 1e3 for (nm, w), ev in times.items() if abs(w - flops) < 1 for s, e in ev]
            for _ in range(3):
                go()
            evs = []
            for _ in range(10):                    # back to back, no host sync between launches
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                go()
                e.record()
                evs.append((s, e))
            torch.cuda.synchronize()
            ts = [s.elapsed_time(e) * 1e3 for s, e in evs]
            print(f"conv M={M:6d} K={K:5d}: in forward {med(inf) if inf else float('nan'):8.1f} us "
                  f"({len(inf)} launches), isolated {med(ts):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
