"""Interleaved A/B of the pipelined config-2 step (bench.py's run(): task.submit + assemble, two streams) across
scheduling variants, on one box (add a variant as a setter in setters()):

    python scripts/pipe_ab.py --variants base,mask64 --rounds 4 --steps 20

Prints ms per step per variant per round and the median; with --encoder-only also the encoder alone."""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def hip_runtime():
    """The libamdhip64 this process already loaded (torch's): a second copy would be a second HIP runtime."""
    import ctypes
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def masked_stream(device, n_cus: int, total: int = 256):
    """A HIP stream restricted to n_cus of the chip's CUs, spread evenly: one block of 8 consecutive CU indices out of
    every total / n_cus blocks (one CU of each XCD under an XCD-interleaved numbering, an equal share of every XCD
    under a contiguous one)."""
    import ctypes
    hip = hip_runtime()
    stride = total // n_cus
    words = (ctypes.c_uint32 * (total // 32))()
    for i in range(total):
        if (i // 8) % stride == 0:
            words[i // 32] |= 1 << (i % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(total // 32), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(st.value, device=device)


def setters(task):
    plain = {}

    def side(kind):
        def f():
            if "plain" not in plain:
                plain["plain"] = getattr(task, "_side", None) or torch.cuda.Stream(task.device)
            if kind == "plain":
                task._side = plain["plain"]
            else:
                key = f"mask{kind}"
                if key not in plain:
                    plain[key] = masked_stream(task.device, kind)
                task._side = plain[key]
        return f

    return {
        "base": side("plain"),
        "mask64": side(64),
        "mask32": side(32),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,mask64")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--encoder-only", action="store_true")
    args = ap.parse_args()
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)
    S = setters(task)
    names = args.variants.split(",")

    def piped(k):
        pending = None
        for _ in range(k):
            h = task.submit(wav, ph, ws, pw, wav_sr=16000)
            if pending is not None:
                task.decoder.assemble(pending, ph, ws, pw)
            pending = h
        task.decoder.assemble(pending, ph, ws, pw)

    def enc(k):
        for _ in range(k):
            task.encode_batch(wav, 16000)

    def clock(fn, k):
        fn(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    res = {n: [] for n in names}
    res_enc = {n: [] for n in names}
    for r in range(args.rounds):
        for n in names:
            S[n]()
            res[n].append(clock(piped, args.steps))
            if args.encoder_only:
                res_enc[n].append(clock(enc, args.steps))
            S["base"]()
            print(f"round {r} {n}: pipelined {res[n][-1]:.3f} ms/step"
                  + (f", encoder alone {res_enc[n][-1]:.3f}" if args.encoder_only else ""), flush=True)
    for n in names:
        print(f"{n}: median pipelined {statistics.median(res[n]):.3f} ms/step "
              f"(min {min(res[n]):.3f}, max {max(res[n]):.3f})"
              + (f", encoder alone {statistics.median(res_enc[n]):.3f}" if args.encoder_only else ""), flush=True)


if __name__ == "__main__":
    main()
