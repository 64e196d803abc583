"""The pipelined config-2 step alone (task.submit + assemble, as bench.py's run()), for a rocprof kernel trace of
the encoder stream beside the side stream: rocprofv3 --kernel-trace -d OUT -o run -- python3 scripts/pipe_trace.py
[--steps 8]."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)
    pending = None
    for _ in range(args.steps):
        h = task.submit(wav, ph, ws, pw, wav_sr=16000)
        if pending is not None:
            task.decoder.assemble(pending, ph, ws, pw)
        pending = h
    task.decoder.assemble(pending, ph, ws, pw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
