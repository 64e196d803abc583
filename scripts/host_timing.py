"""Where does the host block while enqueueing one bench step?  Times each phase of task.submit (GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from hubertfa_amd import ops  # noqa: E402
from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ckpt = synth_checkpoint(encoder="cnhubert", model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, 1000)
    wav = torch.from_numpy(wav_np).to(dev)
    torch.cuda.set_sync_debug_mode(os.environ.get("SYNC_MODE", "warn"))
    T = {}
    orig_call = ops._lib.call

    def timed_call(name, *a):
        t = time.perf_counter()
        orig_call(name, *a)
        dt = time.perf_counter() - t
        if dt > 2e-3:
            print(f"   slow launch {name}: {dt * 1e3:.1f} ms", flush=True)
    ops._lib.call = timed_call
    pending = None
    for step in range(6):
        t0 = time.perf_counter()
        feats, n_frames, wl = task.encode_batch(wav, 16000)
        t1 = time.perf_counter()
        dev_out = task.decode_device(feats, n_frames, wl, ph, ws, pw)
        t2 = time.perf_counter()
        h = task.decoder.fetch(dev_out)
        t3 = time.perf_counter()
        if pending is not None:
            task.decoder.assemble(pending, ph, ws, pw)
        t4 = time.perf_counter()
        pending = h
        print(f"step {step}: encode {1e3 * (t1 - t0):.1f} ms, head+decode {1e3 * (t2 - t1):.1f}, "
              f"fetch {1e3 * (t3 - t2):.1f}, assemble(prev) {1e3 * (t4 - t3):.1f}", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
