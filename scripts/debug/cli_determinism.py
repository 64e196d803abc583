"""Debug: the CLI's batched (variable-length) and one-utterance paths, run repeatedly in one process, must give
identical predictions; counts f32 re-runs taken by the split range guard (GPU box).

python scripts/debug/cli_determinism.py [--reps 6]
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--exp", default="", help="comma list: sync, load, head")
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--wavck", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("--stages", action="store_true")
    ap.add_argument("--convs", action="store_true")
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--pipe", default="")
    ap.add_argument("--guard", action="store_true")
    ap.add_argument("--ldsprobe", default="")
    ap.add_argument("--keepstages", action="store_true")
    ap.add_argument("--sentinel", action="store_true")
    ap.add_argument("--only-c", default="", help="comma list of variants for stage C only: split, f32enc, cfgN")
    args = ap.parse_args()
    import infer
    import hubertfa_amd.g2p as g2p_mod
    from hubertfa_amd import synth
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    from hubertfa_amd.wav_io import write_wav
    import pathlib
    tmp = pathlib.Path(tempfile.mkdtemp())
    d = synth.synth_dictionary(n_words=40)
    dpath = tmp / "dict.txt"
    dpath.write_text("".join(f"{w}\t{' '.join(p)}\n" for w, p in d.items()))
    seg = tmp / "segments"
    seg.mkdir()
    for i, secs in enumerate((2.0, 2.0, 3.5, 2.7, 1.3)):
        write_wav(seg / f"u{i}.wav", synth.synth_audio(int(secs * 16000), seed=i), 16000)
        (seg / f"u{i}.lab").write_text(synth.synth_lab(5, d, seed=i))
    ck = tmp / "m.ckpt"
    synth_checkpoint(str(ck))
    g = g2p_mod.DictionaryG2P(dictionary=str(dpath))
    g.set_in_format("lab")
    rows = list(g.get_dataset(sorted(seg.rglob("*.wav"))))
    torch.set_grad_enabled(False)
    task = ForcedAlignmentTask.load_from_checkpoint(str(ck), device=torch.device("cuda"), hubert_model_path="synth:0")
    redo = {"n": 0}
    orig = task._align_f32

    def counted(*a, **k):
        redo["n"] += 1
        return orig(*a, **k)
    task._align_f32 = counted

    def key(preds):
        return {str(p[0]): (np.asarray(p[4]).tobytes(), np.asarray(p[2]).tobytes()) for p in preds}

    if args.exp:
        from hubertfa_amd import ops
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        from hubertfa_amd.wav_io import read_wav
        wavs = [read_wav(r_[0])[0][0] for r_ in rows]
        if "sync" in args.exp.split(","):       # pipelined submit, but the host waits for each batch
            orig_submit = task.submit

            def sub_sync(*a, **k):
                h = orig_submit(*a, **k)
                torch.cuda.synchronize()
                return h
            task.submit = sub_sync
            got, ref_, bad = [], None, 0
            orig_logits = task.head.logits

            def spy(feats, *a, **k):
                got.append(feats.clone())
                return orig_logits(feats, *a, **k)
            task.head.logits = spy
            for r in range(args.reps):
                got.clear()
                infer._predict(task, rows, 1)
                torch.cuda.synchronize()
                if ref_ is None:
                    ref_ = list(got)
                else:
                    bad += sum(not torch.equal(a, b) for a, b in zip(ref_, got))
            task.head.logits = orig_logits
            task.submit = orig_submit
            print(f"exp sync (cfg {args.cfg}): {bad} differing encoder outputs", flush=True)
        if "load" in args.exp.split(","):       # encoder alone on the main stream beside an unrelated side load
            side = torch.cuda.Stream()
            a = torch.randn(2048, 2048, device="cuda")
            bad = 0
            for i, w in enumerate(wavs):
                x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
                f0 = None
                for _ in range(args.reps):
                    with torch.cuda.stream(side):
                        for _ in range(6):
                            a = torch.tanh(a @ a)
                    feats = task.encode_batch(x, 16000)[0].clone()
                    if f0 is None:
                        f0 = feats
                    elif not torch.equal(f0, feats):
                        bad += 1
            torch.cuda.synchronize()
            print(f"exp load (cfg {args.cfg}): {bad} differing encoder outputs", flush=True)
        for mode in ("fetch", "upl", "fetchupl"):
            if mode not in args.exp.split(","):
                continue
            side = torch.cuda.Stream()
            r2 = rows[2]
            x0 = torch.from_numpy(np.ascontiguousarray(wavs[2])).cuda()[None]
            fh, nf, wl = task.encode_batch(x0, 16000)
            torch.cuda.synchronize()
            bad = 0
            for i, w in enumerate(wavs):
                f0 = None
                for _ in range(args.reps):
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        dv = task.decode_device(fh, nf, wl, [r2[1]], [r2[2]], [r2[3]])
                        if "fetch" in mode:
                            hnd = task.decoder.fetch(dv)
                    if "upl" in mode:
                        x = torch.from_numpy(np.ascontiguousarray(w)[None]).pin_memory().to("cuda", non_blocking=True)
                    else:
                        x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
                    feats = task.encode_batch(x, 16000)[0].clone()
                    if f0 is None:
                        f0 = feats
                    elif not torch.equal(f0, feats):
                        bad += 1
                    if "fetch" in mode:
                        hnd["event"].synchronize()
            torch.cuda.synchronize()
            print(f"exp {mode} (cfg {args.cfg}): {bad} differing encoder outputs", flush=True)
        for mode in ("dec", "full"):
            if mode not in args.exp.split(","):
                continue
            # encoder on main beside the lattice + Viterbi ("dec") or the whole decode_device ("full") on the side
            side = torch.cuda.Stream()
            r2 = rows[2]
            x0 = torch.from_numpy(np.ascontiguousarray(wavs[2])).cuda()[None]
            fh, nf, wl = task.encode_batch(x0, 16000)
            lg = task.head.logits(fh)[:, :nf]
            torch.cuda.synchronize()
            bad = 0
            for i, w in enumerate(wavs):
                x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
                f0 = None
                for _ in range(args.reps):
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        for _ in range(3):
                            if mode == "dec":
                                task.decoder.decode_batch(lg[:, :, 2:], lg[:, :, 0], wl, [r2[1]], [r2[2]], [r2[3]],
                                                          host=False)
                            else:
                                task.decode_device(fh, nf, wl, [r2[1]], [r2[2]], [r2[3]])
                    feats = task.encode_batch(x, 16000)[0].clone()
                    if f0 is None:
                        f0 = feats
                    elif not torch.equal(f0, feats):
                        bad += 1
            torch.cuda.synchronize()
            print(f"exp {mode} (cfg {args.cfg}): {bad} differing encoder outputs", flush=True)
        if "head" in args.exp.split(","):       # encoder on main beside the head's kernels on the side stream
            side = torch.cuda.Stream()
            x0 = torch.from_numpy(np.ascontiguousarray(wavs[2])).cuda()[None]
            fh = task.encode_batch(x0, 16000)[0]
            torch.cuda.synchronize()
            bad = 0
            for i, w in enumerate(wavs):
                x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
                f0 = None
                for _ in range(args.reps):
                    with torch.cuda.stream(side):
                        for _ in range(3):
                            task.head.logits(fh)
                    feats = task.encode_batch(x, 16000)[0].clone()
                    if f0 is None:
                        f0 = feats
                    elif not torch.equal(f0, feats):
                        bad += 1
            torch.cuda.synchronize()
            print(f"exp head (cfg {args.cfg}): {bad} differing encoder outputs", flush=True)
        return
    if args.pipe:
        # the CLI's pipeline re-done here with selectable side-stream work; compares the features the side sees
        from hubertfa_amd import ops
        from hubertfa_amd.wav_io import read_wav
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        wavs = [read_wav(r_[0])[0][0] for r_ in rows]
        order = sorted(range(len(wavs)), key=lambda i: -len(wavs[i]))
        side = torch.cuda.Stream()
        keep = []
        fixed = task.encode_batch(torch.from_numpy(np.ascontiguousarray(wavs[0])).cuda()[None], 16000)[0]
        torch.cuda.synchronize()
        # one recorded head pass: (name, fn, args, kwargs) of every op the UNet calls, for per-op replays
        import hubertfa_amd.unet as um
        real_ops = um.ops
        calls = []

        class _Rec:
            def __getattr__(self, k):
                f = getattr(real_ops, k)
                if not callable(f):
                    return f

                def g(*a, **kw):
                    calls.append((k, f, a, kw))
                    return f(*a, **kw)
                return g
        um.ops = _Rec()
        task.head.logits(fixed)
        um.ops = real_ops
        torch.cuda.synchronize()
        from collections import Counter
        print("head ops:", dict(Counter(c[0] for c in calls)), flush=True)
        for j, (k, f, a, kw) in enumerate(calls):
            if k == "conv_gemm_split":
                desc = {n: (tuple(v.shape) if isinstance(v, torch.Tensor) else v) for n, v in kw.items()}
                print(f"  call {j}: {k} args {[tuple(x.shape) for x in a if isinstance(x, torch.Tensor)]} {desc}",
                      flush=True)
        if args.ldsprobe:
            import ctypes
            lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "probes",
                                           "liblds_guard.so"))
            lib.lds_guard_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
            vstream = torch.cuda.Stream()
            for agg in args.ldsprobe.split(","):
                for kib, nblk in ((8, 256), (8, 512), (16, 256), (32, 256)):
                    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
                    first = torch.zeros(4, dtype=torch.int32, device="cuda")
                    torch.cuda.synchronize()
                    e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
                    e0.record(vstream)
                    lib.lds_guard_launch(nblk, kib, 20000, ctypes.c_void_p(bad.data_ptr()),
                                         ctypes.c_void_p(first.data_ptr()), ctypes.c_void_p(vstream.cuda_stream))
                    e1.record(vstream)
                    e2.record(side)
                    with torch.cuda.stream(side):
                        for _ in range(40):
                            if agg.startswith("conv"):
                                ops._lib.call("hfa_gemm_split_tuning", int(agg[4:]))
                                for k, f, a, kw in calls:
                                    if k == "conv_gemm_split":
                                        f(*a, **kw)
                            elif agg == "linear":
                                for k, f, a, kw in calls:
                                    if k == "linear_split":
                                        f(*a, **kw)
                            elif agg == "mm":
                                m = torch.randn(2048, 2048, device="cuda")
                                m = m @ m
                    e3.record(side)
                    torch.cuda.synchronize()
                    print(f"ldsprobe aggressor={agg} victim {nblk} x {kib} KiB: {int(bad.item())} changed words, "
                          f"first {first.tolist()}; victim {e0.elapsed_time(e1):.2f} ms, aggressor "
                          f"{e2.elapsed_time(e3):.2f} ms, victim start->aggressor start {e0.elapsed_time(e2):.2f} ms",
                          flush=True)
            return
        if args.guard:
            for cfg in (10, 9, 0):
                ops._lib.call("hfa_gemm_split_tuning", cfg)
                for j, (k, f, a, kw) in enumerate(calls):
                    if k != "conv_gemm_split":
                        continue
                    C = kw["C"]
                    G = 1 << 20
                    big = torch.empty(C.numel() + 2 * G, dtype=torch.float32, device=C.device)
                    big.view(torch.int32).fill_(0x7fc00001)
                    kw2 = dict(kw)
                    kw2["C"] = big[G:G + C.numel()].view(C.shape)
                    f(*a, **kw2)
                    torch.cuda.synchronize()
                    lo = (big[:G].view(torch.int32) != 0x7fc00001).nonzero()
                    hi = (big[G + C.numel():].view(torch.int32) != 0x7fc00001).nonzero()
                    if lo.numel() or hi.numel():
                        print(f"cfg {cfg} call {j}: guard writes below {lo.numel()} (first {lo[:3].flatten().tolist()}) "
                              f"above {hi.numel()} (first {hi[:3].flatten().tolist()})", flush=True)
            print("guard done", flush=True)
            return
        rec = None
        if args.keepstages:
            import hubertfa_amd.hubert as hm, hubertfa_amd.encoder as em, hubertfa_amd.resample as rm
            rec = []

            class _Keep:
                def __getattr__(self, k):
                    f = getattr(real_ops, k)
                    if not callable(f):
                        return f

                    def g(*a, **kw):
                        if k == "conv0" and args.sentinel:
                            x_ = a[0]
                            T0 = (x_.shape[1] - 10) // 5 + 1
                            o = torch.empty((2, x_.shape[0], T0, 512), dtype=torch.float16, device=x_.device)
                            o.view(torch.int16).fill_(0x7e01)           # f16 NaN sentinel
                            kw = dict(kw, out=o)
                        out = f(*a, **kw)
                        if torch.cuda.current_stream() == torch.cuda.default_stream():
                            t = out if isinstance(out, torch.Tensor) else None
                            for key in ("C", "Cs", "out"):
                                if t is None and isinstance(kw.get(key), torch.Tensor):
                                    t = kw[key]
                            if t is not None:
                                rec.append((k, t))
                        return out
                    return g
            for m in (hm, em, rm):
                m.ops = _Keep()
        for work in args.pipe.split(","):
            ref_ = None
            bad = 0
            ref_m, bad_m = None, 0
            if work.startswith("xcfg:"):
                ops._lib.call("hfa_gemm_split_tuning", int(work.split(":")[1]))
            if work.startswith("late:"):
                # side work of batch i enqueued after batch i+1's conv0 and waiting for it: the head overlaps the
                # rest of the next encoder instead of its conv0
                import hubertfa_amd.hubert as hm2
                ev = {}
                c0real = real_ops.conv0

                class _C0:
                    def __getattr__(self, k):
                        if k == "conv0":
                            def g(*a, **kw):
                                out = c0real(*a, **kw)
                                e = torch.cuda.Event()
                                e.record()
                                ev["c0"] = e
                                return out
                            return g
                        return getattr(real_ops, k)
                hm2.ops = _C0()
                for rep in range(args.reps):
                    seen, seen_main, prev = [], [], None
                    for i in order + [None]:
                        if i is not None:
                            w = wavs[i]
                            x = torch.from_numpy(np.ascontiguousarray(w)[None]).pin_memory().to("cuda",
                                                                                               non_blocking=True)
                            feats, nf, wl = task.encode_batch(x, 16000)
                            seen_main.append(feats.clone())
                            ready = torch.cuda.Event()
                            ready.record()
                        if prev is not None:
                            pf, pready = prev
                            with torch.cuda.stream(side):
                                side.wait_event(pready)
                                if i is not None:
                                    side.wait_event(ev["c0"])
                                pf.record_stream(side)
                                for k, f, a, kw in calls:
                                    if k == "conv_gemm_split":
                                        f(*a, **kw)
                        prev = (feats, ready) if i is not None else None
                    torch.cuda.synchronize()
                    if ref_ is None:
                        ref_m = seen_main
                        ref_ = True
                    else:
                        bad_m += sum(not torch.equal(a, b) for a, b in zip(ref_m, seen_main))
                hm2.ops = real_ops
                print(f"pipe work={work} cfg {args.cfg}: {bad_m} differing features (main clone) over "
                      f"{args.reps - 1} x {len(order)}", flush=True)
                continue
            for rep in range(args.reps):
                seen, pend = [], None
                seen_main = []
                for i in order:
                    w, r_ = wavs[i], rows[i]
                    x = torch.from_numpy(np.ascontiguousarray(w)[None]).pin_memory().to("cuda", non_blocking=True)
                    feats, nf, wl = task.encode_batch(x, 16000)
                    seen_main.append(feats.clone())
                    ready = torch.cuda.Event()
                    ready.record()
                    if work == "headkeep":
                        keep.append(feats)
                    with torch.cuda.stream(side):
                        side.wait_event(ready)
                        if work != "headkeep":
                            feats.record_stream(side)
                        seen.append(feats.clone())
                        if work in ("head", "headkeep"):
                            task.head.logits(feats)
                        elif work == "headcopy":
                            task.head.logits(seen[-1])
                        elif work == "headfixed":
                            task.head.logits(fixed)
                        elif work.startswith("idx:"):
                            k, f, a, kw = calls[int(work[4:])]
                            f(*a, **kw)
                        elif work.startswith("op:"):
                            for k, f, a, kw in calls:
                                if k == work[3:]:
                                    f(*a, **kw)
                        elif work.startswith("xcfg:"):      # xcfg:<main cfg>:<side cfg> -- conv GEMM replays
                            _, mc, sc = work.split(":")
                            ops._lib.call("hfa_gemm_split_tuning", int(sc))
                            for k, f, a, kw in calls:
                                if k == "conv_gemm_split":
                                    f(*a, **kw)
                            ops._lib.call("hfa_gemm_split_tuning", int(mc))
                        elif work == "dec":
                            task.decode_device(feats, nf, wl, [r_[1]], [r_[2]], [r_[3]])
                        elif work == "fetch":
                            h = task.decoder.fetch(task.decode_device(feats, nf, wl, [r_[1]], [r_[2]], [r_[3]]))
                        done = torch.cuda.Event()
                        done.record()
                    if pend is not None:
                        pend.synchronize()
                    pend = done
                torch.cuda.synchronize()
                if rec is not None:
                    if rep == 0:
                        rec0 = list(rec)
                    else:
                        for j, ((n0, t0), (n1, t1)) in enumerate(zip(rec0, rec)):
                            if not torch.equal(t0, t1):
                                nz = (t0 != t1).nonzero()
                                if n0 == "conv0":
                                    for q in nz[:8].tolist():
                                        print(f"    at {q}: ref {float(t0[tuple(q)])} got {float(t1[tuple(q)])}",
                                              flush=True)
                                print(f"  rep {rep}: first differing op #{j} of {len(rec)}: {n0} shape "
                                      f"{tuple(t0.shape)}, {nz.shape[0]} elements, dim-2 idx "
                                      f"{nz[:, -2].unique().tolist()[:6]}, prev ops "
                                      f"{[q[0] for q in rec0[max(0, j - 3):j]]}", flush=True)
                                break
                    rec.clear()
                if ref_ is None:
                    ref_, ref_m = seen, seen_main
                else:
                    bad += sum(not torch.equal(a, b) for a, b in zip(ref_, seen))
                    bad_m += sum(not torch.equal(a, b) for a, b in zip(ref_m, seen_main))
            print(f"pipe work={work} cfg {args.cfg}: {bad} differing features (side clone), {bad_m} (main clone) "
                  f"over {args.reps - 1} x {len(order)}", flush=True)
        return
    if args.poison:
        # serial: every torch.empty filled with NaN / 0xFF garbage; any output change = a read of unwritten memory
        from hubertfa_amd import ops
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        from hubertfa_amd.wav_io import read_wav
        wavs = [read_wav(r_[0])[0][0] for r_ in rows]
        real_empty = torch.empty

        def run():
            outs = []
            for w, r_ in zip(wavs, rows):
                x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
                fe, nf, wl = task.encode_batch(x, 16000)
                dev = task.decode_device(fe, nf, wl, [r_[1]], [r_[2]], [r_[3]])
                T = int(dev["T"][0])
                outs.append((fe.clone(), dev["lattice"]["prob_log"][0, :T, :len(r_[1])].clone()))
            torch.cuda.synchronize()
            return outs
        base = run()
        for fill in ("nan", "big", "ff"):
            def poisoned(*a, **k):
                t = real_empty(*a, **k)
                if t.is_cuda:
                    if fill == "ff" or not t.is_floating_point():
                        t.view(torch.uint8).fill_(0xFF) if t.numel() and t.is_contiguous() else None
                    else:
                        t.fill_(float("nan") if fill == "nan" else 3.0e4)
                return t
            torch.empty = poisoned
            try:
                got = run()
            finally:
                torch.empty = real_empty
            for i, ((f0, p0), (f1, p1)) in enumerate(zip(base, got)):
                if not torch.equal(f0, f1) or not torch.equal(p0, p1):
                    nz = (f0 != f1).nonzero()
                    print(f"poison {fill}: utt {i} features equal {torch.equal(f0, f1)} ({nz.shape[0]} differ, rows "
                          f"{nz[:, 1].unique().tolist()[:8]}), lattice equal {torch.equal(p0, p1)}", flush=True)
        print("poison done", flush=True)
        return
    if args.stages:
        # light tracing: clone the extractor, positional and every layer output of the encoder (main stream)
        from hubertfa_amd import ops
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        enc = task.unitsEncoder.model
        log = []
        fe, po, ly = enc.feature_extractor, enc.positional, enc.layer

        def fe_(*a, **k):
            out = fe(*a, **k)
            log.append(("extractor", out.clone()))
            return out

        def po_(*a, **k):
            out = po(*a, **k)
            log.append(("positional", out.clone()))
            return out

        def ly_(*a, **k):
            out = ly(*a, **k)
            log.append(("layer", out[0].clone()))
            return out
        enc.feature_extractor, enc.positional, enc.layer = fe_, po_, ly_
        if args.convs:
            import hubertfa_amd.hubert as hm
            c0, cg = hm.ops.conv0, hm.ops.conv_gemm_split

            class _O:
                pass
            o2 = _O()
            o2.__dict__.update({k: getattr(hm.ops, k) for k in dir(hm.ops) if not k.startswith("__")})

            def c0_(*a, **k):
                out = c0(*a, **k)
                log.append(("conv0", out.clone()))
                return out

            def cg_(*a, **k):
                out = cg(*a, **k)
                t = k.get("Cs") if k.get("Cs") is not None else k.get("C")
                log.append((f"conv_gemm_split", t.clone()))
                return out
            o2.conv0, o2.conv_gemm_split = c0_, cg_
            hm.ops = o2
        per_call = 14 + (7 if args.convs else 0)
        runs = []
        for r in range(args.reps):
            log.clear()
            infer._predict(task, rows, 1)
            torch.cuda.synchronize()
            runs.append(list(log))
        ref_ = runs[0]
        for r, run in enumerate(runs[1:], 1):
            for j, ((n0, t0), (n1, t1)) in enumerate(zip(ref_, run)):
                if not torch.equal(t0, t1):
                    nz = (t0 != t1).nonzero()
                    print(f"rep {r}: first differing stage #{j % per_call} ({n0}) of encoder call {j // per_call}: "
                          f"shape {tuple(t0.shape)}: {nz.shape[0]} elements, rows {int(nz[:, -2].min())}.."
                          f"{int(nz[:, -2].max())}, channels {int(nz[:, -1].min())}..{int(nz[:, -1].max())}, "
                          f"max |diff| {float((t0 - t1).abs().max()):.3e}", flush=True)
                    break
        print("stages done", flush=True)
        return
    if args.trace:
        # per-op exact checksums of every main-stream op output, pipelined CLI path: first op that diverges
        from hubertfa_amd import ops
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        import inspect
        log = []

        def cks(t):
            if not isinstance(t, torch.Tensor) or not t.is_cuda:
                return None
            v = t.detach().contiguous()
            v = v.view(torch.int16) if v.element_size() == 2 else v.view(torch.int32) if v.element_size() == 4 else None
            if v is None:
                return None
            v = v.reshape(-1).to(torch.int64)
            w = torch.arange(v.numel(), device=v.device) % 1009 + 1
            return torch.stack([v.sum(), (v * w).sum()])

        def wrap(name, fn):
            def inner(*a, **k):
                out = fn(*a, **k)
                if torch.cuda.current_stream() == torch.cuda.default_stream():
                    tgt = out if isinstance(out, torch.Tensor) else k.get("C", k.get("Cs", k.get("out")))
                    c = cks(tgt)
                    if c is not None:
                        log.append((name, tuple(tgt.shape), c))
                return out
            return inner
        for name, fn in list(vars(ops).items()):
            if inspect.isfunction(fn) and not name.startswith("_") and fn.__module__ == ops.__name__:
                setattr(ops, name, wrap(name, fn))
        runs = []
        for r in range(args.reps):
            log.clear()
            infer._predict(task, rows, 1)
            torch.cuda.synchronize()
            runs.append([(n, sh, tuple(c.tolist())) for n, sh, c in log])
        ref_ = runs[0]
        for r, run in enumerate(runs[1:], 1):
            if len(run) != len(ref_):
                print(f"rep {r}: op count {len(run)} vs {len(ref_)}")
            for j, (x, y) in enumerate(zip(ref_, run)):
                if x != y:
                    ctx = [f"{q[0]}{q[1]}" for q in ref_[max(0, j - 3):j]]
                    print(f"rep {r}: first differing op #{j} {x[0]} {x[1]} (after {ctx})", flush=True)
                    break
        print(f"trace done: {len(ref_)} ops per run", flush=True)
        return
    if args.wavck:
        # pipelined CLI path: checksum of each batch's uploaded waveform (on the stream, after the H2D copy) and
        # the encoder output the head receives
        from hubertfa_amd import ops
        task.on_predict_start()
        ops._lib.call("hfa_gemm_split_tuning", args.cfg)
        wk, fk = [], []
        orig_submit, orig_logits = task.submit, task.head.logits
        keep = []
        orig_encode = task.encode_batch

        def enc_keep(*a, **k):
            out = orig_encode(*a, **k)
            if args.variant == "keep":
                keep.append(out[0])            # features never return to the allocator
            return out
        task.encode_batch = enc_keep

        def sub(waves, *a, **k):
            if args.variant == "serial" and getattr(task, "_side", None) is not None:
                torch.cuda.current_stream().wait_stream(task._side)
            wk.append(waves.double().sum())
            return orig_submit(waves, *a, **k)

        def spy(feats, *a, **k):
            fk.append(feats.clone())
            return orig_logits(feats, *a, **k)
        task.submit, task.head.logits = sub, spy
        ref_w = ref_f = None
        for r in range(args.reps):
            wk.clear()
            fk.clear()
            infer._predict(task, rows, 1)
            torch.cuda.synchronize()
            w = [float(x) for x in wk]
            if ref_w is None:
                ref_w, ref_f = w, list(fk)
                continue
            dw = [j for j in range(len(w)) if w[j] != ref_w[j]]
            df = [j for j in range(len(fk)) if not torch.equal(fk[j], ref_f[j])]
            print(f"rep {r}: waves differ in batches {dw}, features differ in batches {df}", flush=True)
            for j in df:
                a, b = ref_f[j], fk[j]
                nz = (a != b).nonzero()
                ts = nz[:, 1]
                print(f"   batch {j}: shape {tuple(a.shape)} {nz.shape[0]} elements differ, frames "
                      f"{int(ts.min())}..{int(ts.max())} ({ts.unique().numel()} frames), channels "
                      f"{nz[:, 2].unique().numel()}, max |diff| {float((a - b).abs().max()):.3e}, "
                      f"max |ref| {float(a.abs().max()):.3e}", flush=True)
        return
    if args.only_c:
        from hubertfa_amd import ops
        task.on_predict_start()
        enc = task.unitsEncoder.model
        for v in args.only_c.split(","):
            enc.precision = "f32" if v == "f32enc" else "split"
            ops._lib.call("hfa_gemm_split_tuning", int(v[3:]) if v.startswith("cfg") else 0)
            feats_ref, bad = None, 0
            orig_logits = task.head.logits
            got = []

            def spy(feats, *a, **k):
                got.append(feats.clone())
                return orig_logits(feats, *a, **k)
            task.head.logits = spy
            for r in range(args.reps):
                got.clear()
                infer._predict(task, rows, 1)
                torch.cuda.synchronize()
                if feats_ref is None:
                    feats_ref = list(got)
                else:
                    bad += sum(not torch.equal(a, b) for a, b in zip(feats_ref, got))
            task.head.logits = orig_logits
            print(f"variant {v}: {bad} differing encoder outputs over {args.reps - 1} x {len(feats_ref)}", flush=True)
        return
    # A: encoder alone, per utterance, repeated (one stream)
    from hubertfa_amd.wav_io import read_wav
    wavs = [read_wav(r_[0])[0][0] for r_ in rows]
    bad = 0
    for i, w in enumerate(wavs):
        x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
        f0 = None
        for _ in range(args.reps * 3):
            feats = task.encode_batch(x, 16000)[0].clone()
            if f0 is None:
                f0 = feats
            elif not torch.equal(f0, feats):
                bad += 1
    print(f"A encoder-only repeats: {bad} mismatching runs", flush=True)
    # B1: head logits from fixed features, repeated; B2: the lattice's valid region through align_batch
    bad1 = bad2 = 0
    for i, (w, r_) in enumerate(zip(wavs, rows)):
        x = torch.from_numpy(np.ascontiguousarray(w)).cuda()[None]
        feats, n_frames, wl = task.encode_batch(x, 16000)
        l0 = None
        for _ in range(args.reps * 2):
            lg = task.head.logits(feats)[:, :n_frames].clone()
            if l0 is None:
                l0 = lg
            elif not torch.equal(l0, lg):
                bad1 += 1
                dif = (l0 != lg).nonzero()
                print(f"  u{i}: head logits differ at {dif.shape[0]} places, first {dif[:3].tolist()}, "
                      f"max {float((l0 - lg).abs().max()):.3e}", flush=True)
        p0 = None
        S = len(r_[1])
        for _ in range(args.reps * 2):
            dev = task.align_batch(x, [r_[1]], [r_[2]], [r_[3]], wav_sr=16000, host=False)
            T = int(dev["T"][0])
            pl = dev["lattice"]["prob_log"][0, :T, :S].clone()
            if p0 is None:
                p0 = pl
            elif not torch.equal(p0, pl):
                bad2 += 1
    print(f"B1 head-logit repeats: {bad1} mismatching runs; B2 lattice repeats: {bad2}", flush=True)
    # C: the pipelined CLI path; the head's inputs (encoder features) and outputs are stashed per utterance
    stash = {}
    orig_logits = task.head.logits

    def logits_spy(feats, *a, **k):
        out = orig_logits(feats, *a, **k)
        stash.setdefault("cur", []).append((feats.clone(), out.clone()))
        return out
    task.head.logits = logits_spy
    ref_st = None
    ref = None
    for r in range(args.reps):
        stash.clear()
        infer._predict(task, rows, 1)
        torch.cuda.synchronize()
        cur = stash["cur"]
        if ref_st is None:
            ref_st = cur
        else:
            for j, ((f0, l0), (f1, l1)) in enumerate(zip(ref_st, cur)):
                if not torch.equal(f0, f1) or not torch.equal(l0, l1):
                    print(f"  C rep {r} batch {j}: feats equal {torch.equal(f0, f1)}, logits equal "
                          f"{torch.equal(l0, l1)}", flush=True)
    print("C done", flush=True)
    task.head.logits = orig_logits
    for r in range(args.reps):
        for bs in (32, 1):
            redo["n"] = 0
            k = key(infer._predict(task, rows, bs))
            if ref is None:
                ref = k
            diff = [n for n in k if k[n] != ref[n]]
            print(f"rep {r} batch_size {bs}: f32 re-runs {redo['n']}, differing utterances {diff}", flush=True)


if __name__ == "__main__":
    main()
