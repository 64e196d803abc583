"""One-wave Viterbi forward with U utterances per workgroup (U waves, one per SIMD; hfa_viterbi_tuning(200 + U) in
viterbi.hip of commit c574cbc, reverted): the DP holds B/U CUs instead of B while it runs beside the encoder.  Config-2 geometry by default;
encoder alone, then encoder + the DP in one launch beside it, for U = 1, 2, 4 (twice), dp / bt / curr checked
bit-identical to U = 1.
    python scripts/dp_upw_ab.py [--batch 32 --seconds 10 --words 30]"""
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--segments", default="12,10,6")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--words", type=int, default=30)
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

    from hubertfa_amd import _lib

    def with_u(u, fn):
        def run():
            _lib.lib().hfa_viterbi_tuning(200 + u)
            try:
                fn()
            finally:
                _lib.lib().hfa_viterbi_tuning(201)
        return run

    t_enc, _ = clock(enc)
    print(f"encoder alone {t_enc:.2f} ms", flush=True)
    ref = None
    for rep in range(2):
        for u in (1, 2, 4):
            t_dp, _ = clock(with_u(u, dp_alone))
            t_w, got = clock(with_u(u, whole))
            same = True
            if ref is None and u == 1:
                ref = got
            for b in range(B):
                T0, S0 = Ts[b], len(ids[b])
                same = same and (torch.equal(got["dp"][b, :T0, :S0], ref["dp"][b, :T0, :S0]) and
                                 torch.equal(got["bt"][b, 1:T0, :S0], ref["bt"][b, 1:T0, :S0]) and
                                 torch.equal(got["curr"][b, :S0], ref["curr"][b, :S0]))
            print(f"U = {u} utterances per workgroup: DP alone {t_dp:.3f} ms, encoder + DP {t_w:.2f} ms "
                  f"(+{t_w - t_enc:.2f}), bit-identical {same}", flush=True)
            if not same:
                sys.exit(1)


if __name__ == "__main__":
    main()
