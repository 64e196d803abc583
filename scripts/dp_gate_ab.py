"""Config 5 (one 300 s utterance, T = 25 839 frames, S = 1 801 states): where the 13 ms Viterbi forward should run
beside the next encoder (GPU box).  The DP's one workgroup holds a CU for its whole run, and every one-round GEMM
grid of the encoder that overlaps it waits for the tile that could not start there.  Compared, with HIP events:
  enc      the encoder alone
  dp       the forward DP alone
  whole    the DP in one launch on a side stream, started with the encoder (the shipped pipeline's overlap)
  gated    the DP in N step ranges (hfa_viterbi_forward_steps), range k enqueued on the side stream behind an event
           recorded right before the encoder's k-th attention launch (multi-round grids: a held CU costs them little)
and checks the gated DP's dp / bt / curr are bit-identical to the whole launch.
    python scripts/dp_gate_ab.py [--reps 3] [--segments 12,10] [--batch 1 --seconds 300 --words 600]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hubertfa_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--segments", default="12,10,6")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=300.0)
    ap.add_argument("--words", type=int, default=600)
    args = ap.parse_args()
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(args.batch, args.seconds, args.words, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)
    feats, n_frames, wl = task.encode_batch(wav, 16000)
    logits, _ = task.head_logits(feats, n_frames)
    dec = task.decoder
    frame, edge = logits[:, :, 2:].contiguous(), logits[:, :, 0].contiguous()
    B, Tl, V = frame.shape
    Ts = [dec.num_frames(w, Tl) for w in wl]
    ids = [dec.ph_ids(p) for p in ph]
    Smax = -(-max(len(i) for i in ids) // 8) * 8
    ids_pad = np.zeros((B, Smax), np.int32)
    for b, i in enumerate(ids):
        ids_pad[b, :len(i)] = i
    T_t = torch.tensor(Ts, dtype=torch.int32, device=d)
    S_t = torch.tensor([len(i) for i in ids], dtype=torch.int32, device=d)
    ids_t = torch.from_numpy(ids_pad).to(d)
    lat = ops.lattice_prologue(frame, edge, ids_t, T_t, S_t, init_dp=True)
    dp0, bt0, curr0 = lat.pop("dp"), lat.pop("bt"), lat.pop("curr")
    Tmax = dp0.shape[1]
    print(f"T = {Ts[0]}, S = {len(ids[0])}, Tmax = {Tmax}, Smax = {Smax}", flush=True)
    bufs = {"dp": dp0.clone(), "bt": bt0.clone(), "curr": curr0.clone()}

    def dp_range(a, c):
        ops.viterbi_forward(lat["prob_log"], lat["not_edge_log"], lat["edge_log"], bufs["curr"], bufs["dp"],
                            bufs["bt"], ids_t, T_t, S_t, steps=(a, c))

    def reset():
        bufs["dp"].copy_(dp0)
        bufs["curr"].copy_(curr0)

    side = torch.cuda.Stream(d)
    main = torch.cuda.current_stream(d)
    real_attn = ops.attention_split

    def clock(fn):
        ts = []
        for _ in range(args.reps + 1):
            reset()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            fn()
            side_done = torch.cuda.Event()
            side_done.record(side)
            main.wait_event(side_done)
            e1.record(main)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return min(ts[1:]), dict((k, v.clone()) for k, v in bufs.items())

    def enc():
        task.encode_batch(wav, 16000)

    def dp_alone():
        with torch.cuda.stream(side):
            side.wait_stream(main)
            dp_range(1, Tmax)

    def whole():
        with torch.cuda.stream(side):
            side.wait_stream(main)
            dp_range(1, Tmax)
        task.encode_batch(wav, 16000)

    def gated(nseg):
        edges = np.linspace(1, Tmax, nseg + 1).round().astype(int)
        todo = []

        def hooked(*a, **k):
            if todo:
                ev = torch.cuda.Event()
                ev.record(main)
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    dp_range(*todo.pop(0))
            return real_attn(*a, **k)

        def run():
            todo[:] = list(zip(edges[:-1], edges[1:]))
            side.wait_stream(main)
            ops.attention_split = hooked
            try:
                task.encode_batch(wav, 16000)
            finally:
                ops.attention_split = real_attn
            with torch.cuda.stream(side):
                while todo:
                    dp_range(*todo.pop(0))
        return run

    t_enc, _ = clock(enc)
    t_dp, _ = clock(dp_alone)
    t_whole, ref = clock(whole)
    print(f"encoder alone {t_enc:.2f} ms, DP alone {t_dp:.2f} ms, encoder + whole DP {t_whole:.2f} ms "
          f"(+{t_whole - t_enc:.2f})", flush=True)
    for nseg in (int(x) for x in args.segments.split(",")):
        t_g, got = clock(gated(nseg))
        same = True                      # (columns past S hold don't-care values that depend on the cuts)
        for b in range(B):
            T0, S0 = Ts[b], len(ids[b])
            same = same and (torch.equal(got["dp"][b, :T0, :S0], ref["dp"][b, :T0, :S0]) and
                             torch.equal(got["bt"][b, 1:T0, :S0], ref["bt"][b, 1:T0, :S0]) and
                             torch.equal(got["curr"][b, :S0], ref["curr"][b, :S0]))
        print(f"encoder + DP in {nseg} ranges gated at attention: {t_g:.2f} ms (+{t_g - t_enc:.2f}), "
              f"bit-identical {same}", flush=True)
        if not same:
            sys.exit(1)
    t_whole2, _ = clock(whole)
    print(f"encoder + whole DP again {t_whole2:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
