"""The pipelined config-2 step (task.submit + assemble, exactly bench.py's run()) with a launch log, for per-shape
rooflines from a rocprofv3 kernel trace or PMC pass:

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- \
        python3 scripts/shape_trace.py --steps 6 --log OUT/launch_log.json
    python scripts/shape_table.py --trace OUT --log OUT/launch_log.json [--pmc PMC_DIR ...]

The log lists, in host launch order, every launch the ops layer reports to its probe hook during the LAST
``--steps`` steps (name, shape, algorithmic work); shape_table.py pairs them with the trace's dispatches (same
host order) to label each GEMM dispatch by its role (out-proj vs FFN2 share one instantiation and grid).
``--mode serial``: encoder + head + DP on one stream (no overlap); ``--mode encoder``: the encoder alone (what each
encoder kernel takes with nothing beside it: against ``pipe``, the per-kernel cost of the overlapped side stream)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


class LaunchLog:
    """ops.PROBE hook: records every reported launch (no timing, no extra GPU work)."""

    def __init__(self):
        self.name = "-"
        self.entries = []

    def __call__(self, name, work, launch, kind="flops", shape=None, units=None, label=None):
        self.entries.append({"name": name, "work": work, "kind": kind, "shape": list(shape) if shape else None,
                             "label": label})
        return launch()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--encoder", default="base", choices=["base", "large"])
    ap.add_argument("--mode", default="pipe", choices=["pipe", "serial", "encoder"])
    ap.add_argument("--log", required=True)
    args = ap.parse_args()
    import bench
    from hubertfa_amd import ops
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    enc = {"base": "cnhubert", "large": "cnhubert-large"}[args.encoder]
    ck = synth_checkpoint(encoder=enc, model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(args.batch, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)

    def run(k):
        if args.mode == "encoder":
            for _ in range(k):
                task.encode_batch(wav, 16000)
            return
        if args.mode == "serial":
            for _ in range(k):
                task.decoder.assemble(task.align_batch(wav, ph, ws, pw, wav_sr=16000, host=False), ph, ws, pw)
            return
        pending = None
        for _ in range(k):
            h = task.submit(wav, ph, ws, pw, wav_sr=16000)
            if pending is not None:
                task.decoder.assemble(pending, ph, ws, pw)
            pending = h
        task.decoder.assemble(pending, ph, ws, pw)

    run(args.warmup)
    torch.cuda.synchronize()
    log = LaunchLog()
    ops.PROBE = log
    run(args.steps)
    ops.PROBE = None
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(os.path.abspath(args.log)), exist_ok=True)
    with open(args.log, "w") as f:
        json.dump({"steps": args.steps, "batch": args.batch, "encoder": enc, "mode": args.mode,
                   "launches": log.entries}, f)
    print(f"logged {len(log.entries)} launches over {args.steps} steps", flush=True)


if __name__ == "__main__":
    main()
