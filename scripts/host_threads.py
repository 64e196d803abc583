"""Which host threads burn CPU around the pipelined config-2 step (GPU box): per-thread CPU ms (/proc) over (1) 2 s
idle after HIP initialisation, (2) 20 pipelined steps (task.submit + assemble, bench.py's loop), (3) 2 s idle after.
    python scripts/host_threads.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def show(label, a, b, secs):
    rows = bench.thread_cpu_diff(a, b, 1, top=8)
    print(f"{label} ({secs:.2f} s): " + ", ".join(f"{n} {ms:.0f} ms" for n, ms in rows), flush=True)


def main():
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    torch.zeros(1, device=d)
    t0, a = time.time(), bench.thread_cpu()
    time.sleep(2.0)
    show("idle after init", a, bench.thread_cpu(), time.time() - t0)
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)
    for _ in range(3):
        task.decoder.assemble(task.submit(wav, ph, ws, pw, wav_sr=16000), ph, ws, pw)
    torch.cuda.synchronize()
    t0, a = time.time(), bench.thread_cpu()
    pending = None
    for _ in range(20):
        h = task.submit(wav, ph, ws, pw, wav_sr=16000)
        if pending is not None:
            task.decoder.assemble(pending, ph, ws, pw)
        pending = h
    task.decoder.assemble(pending, ph, ws, pw)
    torch.cuda.synchronize()
    show("20 pipelined steps", a, bench.thread_cpu(), time.time() - t0)
    t0, a = time.time(), bench.thread_cpu()
    time.sleep(2.0)
    show("idle after", a, bench.thread_cpu(), time.time() - t0)
    names = {}
    for tid, (n, _) in bench.thread_cpu().items():
        names[n] = names.get(n, 0) + 1
    print("threads by name:", names, flush=True)


if __name__ == "__main__":
    main()
