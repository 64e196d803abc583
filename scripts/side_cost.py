"""What the side stream costs the pipelined config-2 step, decomposed (verdict r05 item 3): power or occupancy?

The pipelined step runs batch i's UNet head + lattice + Viterbi (the "side pass") on a side stream beside batch i+1's
encoder; the step is ~0.8-0.9 ms longer than the encoder alone.  Two timing-only stand-ins for the side pass separate
the candidate causes:
  Z  the same side pass on all-zero weights and inputs: the same kernels, grids, instructions and bytes, minimal
     switching energy (MFMA/VALU on zeros);
  R  a replay of the side pass's kernel sequence by scripts/probes/occupy.hip: for each side kernel a grid of the
     same workgroups holding the same LDS bytes and VGPR count for the kernel's own duration, doing only s_sleep --
     the side pass's CU occupancy with (almost) none of its power.
If E+R ~ E+S and E+Z ~ E+S, the cost is occupancy; if E+Z << E+S and E+R << E+S, it is power.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 scripts/side_cost.py --mode trace
    python scripts/side_cost.py --mode build --trace OUT --out replay.json
    python scripts/side_cost.py --mode ab --replay replay.json
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OCC_LIB = os.path.join(REPO, "scripts", "probes", "_build", "libocc.so")
MARK = "FillFunctor<short>"


def setup(zero=False):
    import torch
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda", 0)
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)
    zt = None
    if zero:
        zsd = {k: torch.zeros_like(v) for k, v in ck["state_dict"].items()}
        zt = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=zsd, device=d)
    return torch, d, task, zt, wav, ph, ws, pw


def mode_trace(a):
    torch, d, task, _zt, wav, ph, ws, pw = setup()
    feats, n_frames, wl = task.encode_batch(wav, 16000)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        torch.full((4099,), 7, dtype=torch.int16, device=d)          # the marker between passes
        torch.cuda.synchronize()
        task.decoder.fetch(task.decode_device(feats, n_frames, wl, ph, ws, pw))
        torch.cuda.synchronize()
    torch.full((4099,), 7, dtype=torch.int16, device=d)
    torch.cuda.synchronize()
    print("traced", a.reps, "side passes", flush=True)


def mode_build(a):
    rows = []
    for f in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if MARK in r["Kernel_Name"]]
    assert len(marks) >= 2, f"need >= 2 markers, found {len(marks)}"
    passes = [rows[i + 1:j] for i, j in zip(marks[:-1], marks[1:])]
    last = passes[-1]
    t0 = int(last[0]["Start_Timestamp"])
    seq = []
    for r in last:
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        vg = int(r["VGPR_Count"]) + int(r.get("Accum_VGPR_Count") or 0)
        seq.append({"name": r["Kernel_Name"][:120], "wgs": (grid + wg - 1) // wg, "block": wg,
                    "lds": int(r["LDS_Block_Size"]), "vgprs": vg,
                    "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                    "start_us": (int(r["Start_Timestamp"]) - t0) / 1e3})
    span = (int(last[-1]["End_Timestamp"]) - t0) / 1e3
    busy = sum(k["us"] for k in seq)
    out = {"passes_traced": len(passes), "kernels": len(seq), "span_us": span, "kernel_us": busy, "sequence": seq}
    json.dump(out, open(a.out, "w"), indent=1)
    print(f"{len(seq)} kernels, span {span:.0f} us, kernel time {busy:.0f} us -> {a.out}")
    for k in sorted(seq, key=lambda k: -k["us"])[:12]:
        print(f"  {k['us']:8.1f} us  wgs {k['wgs']:5d} x {k['block']:4d}  lds {k['lds']:6d}  vgpr {k['vgprs']:3d}  {k['name'][:70]}")


def mode_ab(a):
    torch, d, task, zt, wav, ph, ws, pw = setup(zero=True)
    from hubertfa_amd import ops
    rep = json.load(open(a.replay))["sequence"]
    occ = ctypes.CDLL(OCC_LIB)
    occ.occ_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                               ctypes.c_void_p, ctypes.c_void_p]
    slots = torch.zeros(len(rep), dtype=torch.int64, device=d)
    feats, n_frames, wl = task.encode_batch(wav, 16000)
    zfeats = torch.zeros_like(feats)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()

    def real(f2):
        task.decoder.fetch(task.decode_device(f2, n_frames, wl, ph, ws, pw))

    def real_cap(cap):
        def run(f2):
            with ops.grid_cap(cap):
                task.decoder.fetch(task.decode_device(f2, n_frames, wl, ph, ws, pw))
        return run

    def zero(_f2):
        zt.decoder.fetch(zt.decode_device(zfeats, n_frames, wl, ph, ws, pw))

    def replay(_f2, scale=1.0):
        s = torch.cuda.current_stream().cuda_stream
        slots.zero_()
        for i, k in enumerate(rep):
            rc = occ.occ_launch(k["wgs"], k["block"], k["lds"], k["vgprs"], k["us"] * scale,
                                slots[i:i + 1].data_ptr(), s)
            assert rc == 0, rc

    def replay_cap(cap, gemm_cap=None):
        """every kernel's grid capped at `cap` workgroups; `gemm_cap`: the GEMM and GroupNorm kernels' at that
        instead (what a persistent UNet GEMM / capped GroupNorm would hold)"""
        def run(_f2):
            s = torch.cuda.current_stream().cuda_stream
            slots.zero_()
            for i, k in enumerate(rep):
                c = cap
                if gemm_cap is not None and ("gemm_split" in k["name"] or "gn_rows" in k["name"]):
                    c = gemm_cap
                occ.occ_launch(min(k["wgs"], c), k["block"], k["lds"], k["vgprs"], k["us"],
                               slots[i:i + 1].data_ptr(), s)
        return run

    def replay_nolds(_f2):
        s = torch.cuda.current_stream().cuda_stream
        slots.zero_()
        for i, k in enumerate(rep):
            occ.occ_launch(k["wgs"], k["block"], 0, 64, k["us"], slots[i:i + 1].data_ptr(), s)

    def clock(fn, k):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    def piped(side_work):
        def run():
            f2, _, _ = task.encode_batch(wav, 16000)
            ev = torch.cuda.Event()
            ev.record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev)
                f2.record_stream(side)
                side_work(f2)
        return run

    def alone(side_work):
        def run():
            with torch.cuda.stream(side):
                side_work(feats)
        return run
    arms = {"E": lambda: task.encode_batch(wav, 16000), "E+S": piped(real),
            "E+S(cap 256)": piped(real_cap(256)), "E+S(cap 512)": piped(real_cap(512)),
            "E+S(cap 1024)": piped(real_cap(1024)),
            "E+Z": piped(zero),
            "E+R": piped(replay), "E+R x1.5": piped(lambda f2: replay(f2, 1.5)),
            "E+R(no LDS, 64 VGPR)": piped(replay_nolds),
            "E+R(wgs<=1024)": piped(replay_cap(1024)), "E+R(wgs<=256)": piped(replay_cap(256)),
            "E+R(rows<=512)": piped(replay_cap(512, 10 ** 9)),
            "E+R(rows<=512, gemm/gn<=256)": piped(replay_cap(512, 256)),
            "E+R(rows<=512, gemm/gn<=128)": piped(replay_cap(512, 128)),
            "S alone": alone(real), "S(cap 256) alone": alone(real_cap(256)), "S(cap 512) alone": alone(real_cap(512)),
            "Z alone": alone(zero), "R alone": alone(replay),
            "R(wgs<=256) alone": alone(replay_cap(256))}
    res = {k: [] for k in arms}
    for _ in range(a.rounds):
        for name, fn in arms.items():
            res[name].append(clock(fn, a.steps))
    med = {k: statistics.median(v) for k, v in res.items()}
    e = med["E"]
    out = {"steps": a.steps, "rounds": a.rounds, "median_ms": med, "all_ms": res,
           "cost_ms": {k: med[k] - e for k in arms if k.startswith("E+")}}
    c = out["cost_ms"]
    out["share_of_side_cost"] = {"zero_operands (same work, no switching)": c["E+Z"] / c["E+S"] if c["E+S"] else None,
                                 "occupancy replay (no work)": c["E+R"] / c["E+S"] if c["E+S"] else None}
    print(json.dumps(out), flush=True)
    for k, v in med.items():
        print(f"{k:24s} {v:8.3f} ms" + (f"   cost {v - e:+.3f} ms" if k.startswith("E+") else ""), file=sys.stderr)


def mode_calib(a):
    """The sleeper's own timing: one workgroup for 100 / 1000 us, a 27 648-workgroup grid for 29 us, 55 launches of
    1 us (the per-launch cost of the replay: a memset + a kernel)."""
    import torch
    d = torch.device("cuda", 0)
    occ = ctypes.CDLL(OCC_LIB)
    occ.occ_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                               ctypes.c_void_p, ctypes.c_void_p]
    slots = torch.zeros(64, dtype=torch.int64, device=d)
    s = torch.cuda.current_stream().cuda_stream

    def t(fn, n=5):
        slots.zero_()
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            slots.zero_()
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3
    cases = {"1 wg 100 us": lambda: occ.occ_launch(1, 64, 0, 64, 100.0, slots.data_ptr(), s),
             "1 wg 1000 us": lambda: occ.occ_launch(1, 64, 0, 64, 1000.0, slots.data_ptr(), s),
             "27648 x 256, 8 vgpr, 29 us": lambda: occ.occ_launch(27648, 256, 0, 8, 29.0, slots.data_ptr(), s),
             "448 x 256, 64 KiB, 88 vgpr, 100 us": lambda: occ.occ_launch(448, 256, 65536, 88, 100.0, slots.data_ptr(), s),
             "55 x (1 wg, 1 us)": lambda: [occ.occ_launch(1, 64, 0, 64, 1.0, slots[i:i + 1].data_ptr(), s) for i in range(55)]}
    for k, fn in cases.items():
        print(f"{k:40s} {t(fn):9.1f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", required=True, choices=["trace", "build", "ab", "calib"])
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--trace")
    ap.add_argument("--out", default="replay.json")
    ap.add_argument("--replay")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    {"trace": mode_trace, "build": mode_build, "ab": mode_ab, "calib": mode_calib}[a.mode](a)


if __name__ == "__main__":
    main()
