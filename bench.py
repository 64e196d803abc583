#!/usr/bin/env python
"""bench.py — BASELINE.json config 2: B=32 x 10 s 16 kHz utterances, Hubert-base (cnhubert), 1 MI355X.

One step = the whole infer path for one batch, wave in HBM -> phoneme boundaries on the host:
  16k->44.1k sinc resample (load_wav) -> 44.1k->16k sinc resample (UnitsEncoder) -> Hubert-base (7 convs,
  projection, positional conv, 12 post-LN layers) -> nearest-frame gather -> UNet + head -> lattice prologue
  -> Viterbi DP -> backtrack -> device->host copy -> interval/word assembly (+ RCCL gather of boundary arrays
  when N > 1).  Arithmetic is f32-class: every dense contraction (GEMMs, convs, attention) carries its f32
  operands as split-f16 plane pairs on the f16 MFMA (three exact partial products, f32 accumulation; a batch
  whose values leave f16 range re-runs on the f32 MFMA), everything else is f32.  Weights are seeded synthetic (no checkpoint
  offline), inputs are synthetic harmonic audio + 30 two-phone words (S = 91).

Multi-GPU: one process per GPU (torch.distributed.run); each rank aligns its own B utterances (weak scaling);
the only collective is the boundary-array all_gather.  Timing: barrier + synchronize on both sides of exactly
K steps, max over ranks.

Also reported (rank 0):
  * roofline of the dominant kernel (the MFMA instantiation with the most FLOPs per step, today the split-f16
    implicit GEMM with the GELU epilogue: CNN extractor conv1..5 and the FFN up-projections): algorithmic FLOPs
    per launch / average launch time (HIP events on the launching stream over the timed steps) against the
    f32-equivalent peak of its arithmetic (split-f16: 2516.6 / 3 TFLOP/s; f32 MFMA: 157.3);
  * cpu_baseline (N = 1 only): the CPU oracle (torch-CPU fp32 modules on the host threads + the C Viterbi) on a
    bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "aligned audio sec/sec (RTF^-1) + frames/sec, Hubert-base, 1/2/4/8 MI355X"
F32_MFMA_PEAK_TFLOPS = 157.3
# split-f16 GEMM (gemm_split_kernel): 3 exact f16 x f16 partial products per f32-equivalent MAC on
# v_mfma_f32_16x16x32_f16 (1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz = 2516.6 TFLOP/s dense), so the
# f32-equivalent ceiling of the scheme is a third of that.  The opt-in f16 mode (--precision f16: instantiations
# ending in ", true>") runs one product per MAC: its ceiling is the f16 dense peak itself.
F16_MFMA_PEAK_TFLOPS = 2516.6
SPLIT_F32EQ_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
RANDOM_DATA_F16_TFLOPS = 1247.0    # MI355X_MICROARCH.md 'DVFS give-back' (1): bf16 GEMM on random data, measured


def mfma_peak(kernel: str) -> float:
    if kernel.startswith("gemm_split_kernel") and kernel.endswith(", true>"):
        return F16_MFMA_PEAK_TFLOPS
    split = kernel.startswith("gemm_split_kernel") or kernel.startswith("attn_fwd_split")
    return SPLIT_F32EQ_PEAK_TFLOPS if split else F32_MFMA_PEAK_TFLOPS
HBM_PEAK_GBPS = 8000.0             # MI355X HBM3E, MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU per step")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--words", type=int, default=30)
    ap.add_argument("--cpu-sample-s", type=float, default=15.0, help="CPU baseline time budget (seconds)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sustained-s", type=float, default=10.0,
                    help="N = 1: after the timed steps, run this many seconds of continuous steps and report the first "
                         "and last 2 s (0: skip)")
    ap.add_argument("--encoder", default="base", choices=["base", "large", "soft"],
                    help="base = cnhubert (config 2/3), large = cnhubert-large 24L/1024 (config 4), soft = hubertsoft")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo only for rehearsals")
    ap.add_argument("--device", type=int, default=None, help="force every rank onto this device (rehearsal)")
    ap.add_argument("--probe", default="auto",
                    help="kernel instantiation to time; auto = the one carrying the most FLOPs in a warmup census")
    ap.add_argument("--serial", action="store_true", help="one stream per step (no head/encoder overlap)")
    ap.add_argument("--no-held-dp", action="store_true",
                    help="run a long lattice's DP in one launch behind its head (A/B of task.defer_dp_frames)")
    ap.add_argument("--precision", default="split", choices=["split", "f16"],
                    help="split: f32-class split-f16x3 (the headline); f16: opt-in fast mode, one f16 product per MAC "
                         "in the encoder's split GEMMs (f16-class accuracy, not the reference's f32)")
    ap.add_argument("--chunk-seconds", type=float, default=None,
                    help="long-form: encode overlapping windows of this length (config 5 chunked; B=1 only)")
    ap.add_argument("--two-stage-resample", action="store_true",
                    help="run the 16 k -> 44.1 k -> 16 k resampling as its two stages (A/B of the one-pass chain)")
    ap.add_argument("--defer-dp-frames", type=int, default=None,
                    help="task.defer_dp_frames (hold lattices of at least this many DP frames for the next encoder's "
                         "attention launches; A/B of the threshold)")
    ap.add_argument("--side-grid-cap", type=int, default=None,
                    help="task.side_grid_cap (workgroups per launch of the side pass's row kernels; A/B of the cap)")
    ap.add_argument("--no-config3", action="store_true",
                    help="N > 1: skip the extra BASELINE config-3 measurement (global batch 512) after the timed steps")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="N = 1 headline runs: skip the config4 / config5 blocks measured after the timed steps")
    ap.add_argument("--host-input", action="store_true",
                    help="waves start in host memory and are uploaded inside every step (task.upload, as infer.py) (PCIe-inclusive "
                         "rate; the headline value keeps inputs resident in HBM)")
    ap.add_argument("--probe-every", type=int, default=1,
                    help="time the dominant kernel's launches (HIP events) in every N-th timed step only")
    ap.add_argument("--probe-secondary", action="store_true",
                    help="also time the secondary kernels inside the timed region (else in an untimed pipelined pass)")
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "r06", "traffic_r06.json"),
                    help="PMC-derived HBM bytes per launch of the probed kernel (written by scripts/pmc_traffic.py)")
    ap.add_argument("--pmc-file", default=os.path.join(REPO, "profiles", "r06", "pmc_r06.json"),
                    help="PMC-derived MFMA busy and clock per kernel (written by scripts/pmc_kernels.py)")
    return ap.parse_args()


def make_inputs(B, seconds, words, seed0):
    import numpy as np
    from hubertfa_amd import synth
    n16 = int(round(seconds * 16000))
    wav = np.stack([synth.synth_audio(n16, 16000, seed=seed0 + i) for i in range(B)])
    d = synth.synth_dictionary(n_words=400)
    two = sorted(w for w, p in d.items() if len(p) == 2)
    r = synth.rng(seed0 + 12345)
    ph_seqs, word_seqs, p2ws = [], [], []
    for i in range(B):
        ws = [two[int(j)] for j in r.integers(0, len(two), words)]
        ph, p2w = ["SP"], [-1]
        for wi, w in enumerate(ws):
            for p in d[w]:
                ph.append(p)
                p2w.append(wi)
            ph.append("SP")
            p2w.append(-1)
        ph_seqs.append(ph)
        word_seqs.append(ws)
        p2ws.append(p2w)
    return wav, ph_seqs, word_seqs, p2ws


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(wav, ph_seqs, word_seqs, p2ws, ckpt, budget_s, encoder="cnhubert"):
    """CPU oracle on a bounded sample (whole utterances until the budget is spent), with the per-stage split SURVEY
    §8(d) asks for (resample, Hubert, gather + UNet + head, decode) and the C Viterbi alone on one core per
    utterance (the numba-equivalent: forward_pass + backtrack, alignment_decoder.py:170-230, 269-288)."""
    import numpy as np
    import torch
    from hubertfa_amd import synth
    from oracle import decode as odec, hubert_cpu, resample as ores
    hp = ckpt["hyper_parameters"]
    import yaml
    vocab = yaml.safe_load(hp["vocab_text"])
    arch = {"cnhubert": synth.arch_cnhubert_base, "cnhubert-large": synth.arch_cnhubert_large,
            "hubertsoft": synth.arch_hubertsoft}[encoder]()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    ua = synth.UNetArch(input_dims=arch.out_channels, vocab_size=vocab["vocab_size"])
    usd = {k: v.numpy() for k, v in ckpt["state_dict"].items()}
    threads = torch.get_num_threads()
    stages = {"resample": 0.0, "hubert": 0.0, "unet_head": 0.0, "decode": 0.0}
    done, t0 = 0, time.perf_counter()
    last = None
    while time.perf_counter() - t0 < budget_s:   # cycle over the batch until the budget is spent
        i = done % len(wav)
        ta = time.perf_counter()
        x16 = torch.from_numpy(wav[i:i + 1])
        x44 = ores.resample(x16, 16000, 44100, 6)
        xr = ores.resample(x44, 44100, 16000, 128)
        tb = time.perf_counter()
        units = hubert_cpu.hubert_forward(arch, sd, xr)
        tc = time.perf_counter()
        n44 = x44.shape[-1]
        n_frames = n44 // 512 + 1
        ratio = (512 / 44100) / (320 / 16000)
        idx = torch.clamp(torch.round(ratio * torch.arange(n_frames)).long(), max=units.shape[1] - 1)
        feats = units[:, idx]
        logits = hubert_cpu.unet_head_forward(ua, usd, feats)
        td = time.perf_counter()
        r = odec.decode(vocab, logits[:, :, 2:], logits[:, :, 0], n44 / 44100, ph_seqs[i], word_seqs[i], p2ws[i])
        te = time.perf_counter()
        for k, dt in zip(stages, (tb - ta, tc - tb, td - tc, te - td)):
            stages[k] += dt
        last = (np.array([vocab["vocab"][p] for p in ph_seqs[i]]), r[5]["ph_prob_log"], r[5]["edge_prob"])
        done += 1
    el = time.perf_counter() - t0
    # the C Viterbi alone (single-threaded C, -O2 -ffp-contract=off): lattice prep + forward_pass + backtrack of one
    # utterance, repeated for >= 1 s
    ids, ppl, ep = last
    n_v, tv = 0, time.perf_counter()
    while n_v < 3 or time.perf_counter() - tv < 1.0:
        odec._decode(ids, ppl, ep)
        n_v += 1
    v_ms = 1e3 * (time.perf_counter() - tv) / n_v
    secs = done * wav.shape[1] / 16000
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"value": secs / el, "unit": "audio_s/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "os_cpu_count": os.cpu_count(), "affinity_cpus": affinity, "torch_threads": threads,
            "stages_ms_per_utterance": {k: 1e3 * v / max(done, 1) for k, v in stages.items()},
            "viterbi_1core_ms_per_utterance": v_ms, "viterbi_T": int(ppl.shape[0]), "viterbi_S": int(len(ids)),
            "viterbi_1core_us_per_time_step": 1e3 * v_ms / max(int(ppl.shape[0]), 1),
            "sample": f"{done} x {wav.shape[1] / 16000:.0f} s utterances of the same workload, sequential B=1 "
                      f"(oracle: torch-CPU fp32 resample + {encoder} + UNet on {threads} torch threads, C Viterbi "
                      f"on 1 core), {el:.1f} s wall",
            "note": "cores = torch intra-op threads used (torch.get_num_threads(); the box's share of a larger node: "
                    "os_cpu_count is the whole machine, affinity_cpus what this process may run on); the C Viterbi "
                    "is single-threaded like the reference's numba forward_pass"}


def config_name(encoder: str, world: int, B: int, seconds: float = 10.0) -> str:
    """Which BASELINE.json config this run's geometry is (configs[1..4]); weak scaling keeps B per GPU fixed."""
    if seconds >= 60:
        return f"config 5 geometry (long-form, {seconds:g} s, {B} per GPU)"
    if encoder == "large":
        return "config 4 geometry" + ("" if world * B == 256 else f" (global batch {world * B}, config 4 is 256)")
    if world == 1:
        return "config 2" if B == 32 else f"config 2 geometry (B={B}, config 2 is 32)"
    return "config 3 geometry" + ("" if world * B == 512 else f" (global batch {world * B}, config 3 is 512)")


def step_breakdown(task, wav, ph_seqs, word_seqs, p2ws, k, step_s):
    """What the side stream (UNet head + lattice + Viterbi + D2H, overlapped with the next batch's encoder) costs
    the pipelined step: the same k steps with the encoder alone (main stream, nothing beside it), and the head + DP
    alone on the encoder's output (serial).  Outside the timed region."""
    import torch
    from hubertfa_amd import ops
    feats, n_frames, wl = task.encode_batch(wav, 16000)
    torch.cuda.synchronize()

    def clock(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3
    enc_ms = clock(lambda: task.encode_batch(wav, 16000))
    head_ms = clock(lambda: task.decoder.fetch(task.decode_device(feats, n_frames, wl, ph_seqs, word_seqs, p2ws)))
    # the side stream's two parts, each overlapped alone with the encoder as in task.submit
    side = torch.cuda.Stream()
    logits = task.head.logits(feats)[:, :n_frames]
    frame, edge = logits[:, :, 2:], logits[:, :, 0]

    def piped(side_work):
        def run():
            f2, _, _ = task.encode_batch(wav, 16000)
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(side):
                side.wait_event(ev)
                f2.record_stream(side)      # the next iteration's encoder must not reuse f2 under the side stream
                side_work(f2)
        return run
    unet_piped = clock(piped(lambda f2: task.head.logits(f2)))
    dp_piped = clock(piped(lambda f2: task.decoder.fetch(task.decoder.decode_batch(frame, edge, wl, ph_seqs, word_seqs,
                                                                                      p2ws, host=False))))
    torch.cuda.synchronize()
    task.head.flag.zero_()                  # nothing from these measurement runs may reach the later steps' guard
    ops.split_flag(task.device).zero_()
    return {"pipelined_step_ms": step_s * 1e3, "encoder_only_ms": enc_ms, "head_dp_only_ms": head_ms,
            "side_stream_cost_ms": step_s * 1e3 - enc_ms, "encoder_plus_unet_ms": unet_piped,
            "encoder_plus_lattice_dp_ms": dp_piped,
            "note": "encoder_only / head_dp_only: the step's two halves run alone, serially, k steps each; "
                    "side_stream_cost = pipelined step - encoder alone (what overlapping the head costs the encoder); "
                    "encoder_plus_unet / encoder_plus_lattice_dp: the encoder with only that part of the side stream "
                    "beside it"}


def chunk_agreement(task, wav, ph_seqs, word_seqs, p2ws, chunk_seconds):
    """Chunked long-form against its anchor, the unchunked run of the same utterances (the
    reference encodes each wave whole, tools/encoder.py:36-60): per utterance, the share of phone boundaries whose
    frame is within 0 / 2 / 5 DP frames of the unchunked run's, and the largest per-frame log-prob difference on
    the [T, S] lattice (and its mean).  Outside the timed region."""
    import numpy as np
    import torch
    full = task.align_batch(wav, ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False)
    chnk = task.align_batch(wav, ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False, chunk_seconds=chunk_seconds)
    torch.cuda.synchronize()
    out = []
    for b in range(len(ph_seqs)):
        T, S = full["T"][b], len(ph_seqs[b])
        dl = (full["lattice"]["prob_log"][b, :T, :S] - chnk["lattice"]["prob_log"][b, :T, :S]).abs()
        n_a, n_b = int(full["n"][b]), int(chnk["n"][b])
        ia, ta = full["ph_idx_seq"][b, :n_a].cpu().numpy(), full["ph_time_int"][b, :n_a].cpu().numpy()
        ib, tb = chnk["ph_idx_seq"][b, :n_b].cpu().numpy(), chnk["ph_time_int"][b, :n_b].cpu().numpy()
        common, xa, xb = np.intersect1d(ia, ib, return_indices=True)
        d = np.abs(ta[xa].astype(np.int64) - tb[xb].astype(np.int64))
        out.append({"T": int(T), "states": S, "boundaries": int(n_a), "boundaries_chunked": int(n_b),
                    "phones_in_both": int(len(common)),
                    "within_0": float(np.mean(d == 0)) if len(d) else None,
                    "within_2": float(np.mean(d <= 2)) if len(d) else None,
                    "within_5": float(np.mean(d <= 5)) if len(d) else None,
                    "max_frame_shift": int(d.max()) if len(d) else None,
                    "max_logprob_diff": float(dl.max()), "mean_logprob_diff": float(dl.mean())})
    return {"chunk_seconds": chunk_seconds, "anchor": "the unchunked run of the same utterance (the reference "
            "encodes each wave whole, tools/encoder.py:36-60)", "utterances": out,
            "note": "random-init weights: the agreement says little about a trained model's; it measures what the "
                    "windows' lost attention context changes on this workload"}


def config3_batch(args, world: int) -> int:
    """Per-GPU batch of BASELINE config 3 (512 x 10 s over the node) when this multi-GPU run's own global batch is
    not already 512; 0 when there is nothing extra to measure."""
    if world <= 1 or args.encoder != "base" or args.seconds != 10.0 or args.chunk_seconds is not None:
        return 0
    if world * args.batch == 512 or 512 % world or args.no_config3:
        return 0
    return 512 // world


def sustained(run, seconds, audio_per_step, headline_ms, window_s=2.0):
    """Sustained throughput (verdict r05 item 2): ``seconds`` of continuous pipelined steps right after the timed
    region, one HIP event on the launching stream at the start of every step.  The interval between two steps'
    events is that step's share of the device's time (the host keeps the stream fed), so the first and the last
    ``window_s`` seconds of intervals show whether the 20-step headline rate holds as the chip heats; ``wall`` is the
    whole run's wall clock.  Outside the timed region."""
    import torch
    evs = []

    def mark():
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        evs.append(ev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(10 ** 9, on_step=mark, until=t0 + seconds)
    end = torch.cuda.Event(enable_timing=True)
    end.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    evs.append(end)
    step_events = [evs[i].elapsed_time(evs[i + 1]) for i in range(len(evs) - 1)]      # ms

    def window(ms_list):
        acc, out = 0.0, []
        for m in ms_list:
            if acc >= window_s * 1e3:
                break
            out.append(m)
            acc += m
        return out
    first, last = window(step_events), window(step_events[::-1])
    mean = lambda x: sum(x) / len(x)  # noqa: E731
    f_ms, l_ms = mean(first), mean(last)
    return {"seconds": wall, "steps": len(step_events), "ms_per_step": 1e3 * wall / len(step_events),
            "value": audio_per_step * len(step_events) / wall, "unit": "audio_s/s",
            "first_window_ms_per_step": f_ms, "last_window_ms_per_step": l_ms,
            "first_window_value": audio_per_step / f_ms * 1e3, "last_window_value": audio_per_step / l_ms * 1e3,
            "window_s": window_s, "min_step_ms": min(step_events), "max_step_ms": max(step_events),
            "last_vs_headline": headline_ms / l_ms,
            "note": "continuous pipelined config-2 steps (bench's own loop) right after the timed region; per-step "
                    "times are the intervals between HIP events recorded on the launching stream at each step's start, "
                    "the last one ends at the drained pipeline; wall includes the final drain"}


def host_io(wav_np, res, seconds, budget_s=3.0):
    """file I/O and TextGrid writing, reported beside (not inside) the timed wave->boundaries path:
    read the batch as 16-bit WAV files (wav_io.read_wav, the CLI's native reader) and write its TextGrids + confidence.csv
    (post_processing + Exporter, the CLI's writer) in a temporary directory, on the host; ms per batch."""
    import tempfile
    from hubertfa_amd.export_tool import Exporter
    from hubertfa_amd.post_processing import post_processing
    from hubertfa_amd.wav_io import read_wav, write_wav
    B = wav_np.shape[0]
    with tempfile.TemporaryDirectory() as td:
        paths = [os.path.join(td, f"utt{b:04d}.wav") for b in range(B)]
        for p, x in zip(paths, wav_np):
            write_wav(p, x, 16000)
        t_read, n = 0.0, 0
        while n == 0 or (t_read < budget_s / 2 and n < 20):
            t0 = time.perf_counter()
            for p in paths:
                read_wav(p)
            t_read += time.perf_counter() - t0
            n += 1
        preds = [(p, seconds, r["confidence"], r["ph_seq"], r["ph_intervals"], r["word_seq"], r["word_intervals"])
                 for p, r in zip(paths, res)]
        Exporter(*post_processing(list(preds)), os.path.join(td, "warm")).export(["textgrid", "confidence"])
        t_write, m = 0.0, 0
        while m == 0 or (t_write < budget_s / 2 and m < 20):
            pp, log = post_processing(list(preds))
            t0 = time.perf_counter()
            Exporter(pp, log, os.path.join(td, "out")).export(["textgrid", "confidence"])
            t_write += time.perf_counter() - t0
            m += 1
    return {"wav_read_ms_per_batch": 1e3 * t_read / n, "textgrid_write_ms_per_batch": 1e3 * t_write / m,
            "files_per_batch": B, "note": "host only, one thread, outside the timed region (infer.py decodes a batch's "
                                          "files on a thread pool into its pinned upload buffer, and on one GPU "
                                          "writes each batch's TextGrids, while the GPU runs the neighbouring batch)"}


SECONDARY = ("viterbi_forward_kernel", "hfa_conv0_split", "hfa_conv0_f32", "attn_fwd_split16_kernel", "attn_fwd_split_kernel",
             "attn_fwd_f32_kernel")
SECONDARY_NOTE = {"hfa_conv0_split": "one hfa_conv0_split call: conv0_gram_kernel + conv0_gram_stats_kernel + "
                                     "conv0_packed_kernel (statistics and the apply pass)",
                  "hfa_conv0_f32": "one hfa_conv0_f32 call (the f32 path: statistics + the VALU apply pass)"}


def secondary_rooflines(iso, pipe, T, S):
    """SURVEY §8(d) secondary figures: the DP (HBM-accounted latency-bound scan, also µs per time step),
    conv0+GroupNorm+GELU (HBM) and flash attention (MFMA), timed with HIP events.  The roofline numbers come from
    ``iso``: two serial steps after the timed region, one stream, nothing overlapping.  ``pipe`` adds each
    kernel's average duration inside the timed, two-stream pipeline, where the head + DP share the chip with the
    next batch's encoder (so their wall time there is longer than the kernel needs)."""
    out = []
    for name in SECONDARY:
        ps = iso.summary(name)
        if not ps["launches"]:
            continue
        rate = ps["avg_work"] / (ps["avg_ms"] * 1e-3)
        if name.startswith("attn_fwd"):
            e = {"kernel": name, "bound": "mfma", "achieved": rate / 1e12, "peak": mfma_peak(name),
                 "unit": "TFLOP/s", "frac": rate / 1e12 / mfma_peak(name)}
        else:
            e = {"kernel": name, "bound": "hbm" if name != "viterbi_forward_kernel" else "latency",
                 "achieved": rate / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": rate / 1e9 / HBM_PEAK_GBPS,
                 "bytes_per_launch": ps["avg_work"]}
            if name == "viterbi_forward_kernel":
                e["us_per_time_step"] = ps["total_ms"] * 1e3 / ps["units"] if ps["units"] else ps["avg_ms"] * 1e3 / T
                e["states"] = S
        pp = pipe.summary(name)
        if name in SECONDARY_NOTE:
            e["covers"] = SECONDARY_NOTE[name]
        e.update({"launches": ps["launches"], "avg_launch_ms": ps["avg_ms"], "timing": "isolated serial steps",
                  "in_pipeline_avg_launch_ms": pp["avg_ms"] if pp["launches"] else None})
        out.append(e)
    return out


def thread_cpu():
    """{native thread id: (name, user + system CPU seconds)} of this process (Linux /proc; {} elsewhere)."""
    out = {}
    base = f"/proc/{os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    tck = os.sysconf("SC_CLK_TCK")
    for t in tids:
        try:
            with open(f"{base}/{t}/stat") as f:
                st = f.read()
            name = st[st.index("(") + 1:st.rindex(")")]
            fields = st[st.rindex(")") + 2:].split()
            out[int(t)] = (name, (int(fields[11]) + int(fields[12])) / tck)
        except (OSError, ValueError, IndexError):
            continue
    return out


def thread_cpu_diff(a, b, steps, top=5):
    """The busiest threads' CPU ms per step between two thread_cpu() snapshots."""
    import threading
    main_id = threading.get_native_id()
    rows = []
    for tid, (name, t1) in b.items():
        d = t1 - a.get(tid, (name, 0.0))[1]
        if d > 0:
            rows.append(("main" if tid == main_id else name, round(1e3 * d / max(steps, 1), 2)))
    rows.sort(key=lambda r: -r[1])
    return rows[:top]


def launcher_cmd(gpus: int, argv, port: int):
    """The torch.distributed.run command that starts ``gpus`` ranks of this script with the same arguments."""
    return [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def check_world(args, env=None):
    """``--gpus N`` against the launch: None when this process is a rank of the right world (or a one-GPU run), else
    "launch" (no WORLD_SIZE and N > 1: start N ranks) or an error message (a rank count other than N, too few
    visible devices).  Reads no device state beyond the count (torch.cuda.device_count() does not initialise HIP)."""
    env = os.environ if env is None else env
    if args.gpus < 1:
        return f"--gpus {args.gpus}: at least one GPU"
    if "WORLD_SIZE" in env:
        w = int(env["WORLD_SIZE"])
        if w != args.gpus:
            return f"--gpus {args.gpus} but this launch has WORLD_SIZE={w} ranks"
        return None
    if args.gpus == 1:
        return None
    if args.device is None:
        import torch
        n = torch.cuda.device_count()
        if n < args.gpus:
            return (f"--gpus {args.gpus}: only {n} GPU(s) visible (HIP_VISIBLE_DEVICES / the node); pass --device D to "
                    f"rehearse {args.gpus} ranks on one GPU")
    return "launch"


def launch_ranks(args) -> int:
    """Start ``--gpus`` ranks of this script under torch.distributed.run as a CHILD process (never exec: nothing here
    has touched the GPU, and the ranks do it themselves), relay its output (rank 0 prints the one JSON line) and
    return its exit code.  SIGTERM / SIGINT are passed on to the child's process group."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.Popen(launcher_cmd(args.gpus, sys.argv[1:], port), start_new_session=True)

    def relay(sig, _frame):
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, relay)
    return p.wait()


def device_census(dev, world):
    """What the collective layer saw: the process group's world size and every rank's device and PCI address,
    gathered to every rank (outside the timed region)."""
    import torch
    import torch.distributed as dist
    pr = torch.cuda.get_device_properties(dev)
    mine = {"rank": dist.get_rank() if world > 1 else 0, "device": int(dev.index), "name": pr.name,
            "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
            "visible": os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))}
    if world == 1:
        return {"world_size": 1, "backend": None, "ranks": [mine]}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": allr,
            "distinct_devices": len({r["pci"] for r in allr})}


def main():
    args = parse()
    verdict = check_world(args)
    if verdict == "launch":
        sys.exit(launch_ranks(args))
    if verdict is not None:
        print(f"bench.py: {verdict}", file=sys.stderr, flush=True)
        sys.exit(2)
    import numpy as np
    import torch
    import torch.distributed as dist
    from hubertfa_amd import ops
    from hubertfa_amd.distributed import env_rank_world, gather_boundaries
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint

    rank, world, local = env_rank_world()
    if args.device is not None:          # rehearsal of the N>1 path on a 1-GPU box (all ranks on one device)
        local = args.device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    encoder = {"base": "cnhubert", "large": "cnhubert-large", "soft": "hubertsoft"}[args.encoder]
    ckpt = synth_checkpoint(encoder=encoder, model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    if args.two_stage_resample:
        task.chain_resample = False
    if args.side_grid_cap is not None:
        task.side_grid_cap = args.side_grid_cap
    if args.defer_dp_frames is not None:
        task.defer_dp_frames = args.defer_dp_frames
    if args.no_held_dp:
        task.defer_dp_frames = None
    if args.precision == "f16":
        task.unitsEncoder.model.f16 = True
    B = args.batch
    wav_np, ph_seqs, word_seqs, p2ws = make_inputs(B, args.seconds, args.words, seed0=1000 * (rank + 1))
    wav = wav_dev = torch.from_numpy(wav_np).to(dev)
    wav_host = torch.from_numpy(wav_np).pin_memory() if args.host_input else None
    inputs = (wav_dev, wav_host, ph_seqs, word_seqs, p2ws)

    def launch(inp, tk):
        """GPU half of one step (+ the boundary gather) and the async D2H of its results: the encoder on the main
        stream, head + DP on a side stream overlapping the next step's encoder (task.submit).  With --host-input the
        step starts with task.upload of its waves (the CLI's pinned non-blocking H2D)."""
        wav_d, wav_h, ph, ws, pw = inp
        wav = tk.upload(wav_h) if wav_h is not None else wav_d
        if args.serial:
            dev_out = tk.align_batch(wav, ph, ws, pw, wav_sr=16000, host=False, chunk_seconds=args.chunk_seconds)
            if world > 1:
                gather_boundaries(dev_out, uniform=True)
            return tk.decoder.fetch(dev_out)
        return tk.submit(wav, ph, ws, pw, wav_sr=16000,
                           on_device=(lambda d: gather_boundaries(d, uniform=True)) if world > 1 else None,
                           chunk_seconds=args.chunk_seconds)

    def finish(handle, inp, tk):
        return tk.decoder.assemble(handle, *inp[2:])

    def run(k, inp=inputs, tk=task, on_step=None, until=None):
        """k steps, software-pipelined: the host assembles batch i while the GPU runs batch i+1 -- or, when
        task.submit holds a batch's DP for the next encoder's attention launches (a long lattice), batch i-1: batch
        i's results land near the end of encoder i+1, and waiting for them there would leave the GPU idle while the
        host assembles and enqueues the next step.  ``on_step`` runs before each step's launch; ``until`` (a
        perf_counter time) ends the loop early (the sustained block)."""
        pending, res = [], None
        for _ in range(k):
            if until is not None and time.perf_counter() >= until:
                break
            if on_step is not None:
                on_step()
            t0, c0, p0 = time.perf_counter(), time.thread_time(), time.process_time()
            h = launch(inp, tk)
            t1, c1 = time.perf_counter(), time.thread_time()
            pending.append(h)
            while len(pending) > (2 if "resolve" in h else 1):
                res = finish(pending.pop(0), inp, tk)
            host_t.append((t1 - t0, time.perf_counter() - t1, c1 - c0, time.thread_time() - c1,
                           time.process_time() - p0))
        while pending:
            res = finish(pending.pop(0), inp, tk)
        return res

    def timed(k, inp=inputs, tk=task, on_step=None):
        """exactly k steps between barrier + synchronize pairs -> (results, max seconds over ranks)."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = run(k, inp, tk, on_step=on_step)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([e], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            e = float(tt.item())
        return r, e

    host_t = []   # per step: enqueue / wait + assemble wall seconds, their CPU seconds (this thread), process CPU

    census = ops.KernelProbe(None)
    ops.PROBE = census
    res = run(max(args.warmup, 1))
    ops.PROBE = None
    torch.cuda.synchronize()
    probe_name = census.dominant() if args.probe == "auto" else args.probe
    # the dominant kernel is timed live in the timed steps (every --probe-every-th step); each timed launch adds two
    # event records to the stream, so the secondary kernels are timed in a separate untimed pipelined pass below
    probe = ops.KernelProbe(probe_name, extra=SECONDARY if args.probe_secondary else ())
    ops.PROBE = probe
    thr0 = thread_cpu()
    step_i = [0]
    # the cyclic collector's pauses inside the timed region (generation, ms): a full collection over the process's
    # heap stalls the launching thread (host_cpu.gc_pauses)
    import gc
    gc_log, gc_t = [], {}

    def gc_cb(phase, info):
        if phase == "start":
            gc_t["t"] = time.perf_counter()
        elif "t" in gc_t:
            gc_log.append((info["generation"], 1e3 * (time.perf_counter() - gc_t.pop("t"))))
    gc.callbacks.append(gc_cb)

    step_ev = []                      # one event per timed step at its start (the launching stream)

    def sample_step():
        probe.active = step_i[0] % max(args.probe_every, 1) == 0
        step_i[0] += 1
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        step_ev.append(ev)
    res, el = timed(args.steps, on_step=sample_step)
    thr1 = thread_cpu()
    gc.callbacks.remove(gc_cb)
    ops.PROBE = None
    probe.active = True
    pipe = probe
    if not args.probe_secondary:       # the secondary kernels' in-pipeline durations: the same loop, untimed
        pipe = ops.KernelProbe("-", extra=SECONDARY)
        ops.PROBE = pipe
        run(min(args.steps, 5))
        torch.cuda.synchronize()
        ops.PROBE = None

    devices = device_census(dev, world)
    n_frames = res[0]["T"]
    audio_s = world * B * args.seconds * args.steps
    value = audio_s / el
    frames_ps = world * B * n_frames * args.steps / el
    ps = probe.summary()
    achieved = ps["avg_flops"] / (ps["avg_ms"] * 1e-3) / 1e12 if ps["launches"] else None
    hub_flops = task.unitsEncoder.model.flops(int(round(args.seconds * 16000)))
    head_flops = task.head.flops(task.head.padded_len(n_frames))

    pmc = None
    if os.path.exists(args.pmc_file):
        try:
            with open(args.pmc_file) as f:
                pmc = json.load(f).get("kernels", {}).get(probe_name)
        except Exception:  # noqa: BLE001
            pmc = None
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            with open(args.traffic_file) as f:
                tj = json.load(f)
            if tj.get("kernel") == probe_name:
                traffic = tj.get("bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    out = {
        "metric": METRIC, "value": value, "unit": "audio_s/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 (split-f16x3)" if args.precision == "split" else "f16 (opt-in fast mode)",
        "data": "synthetic",
        "arithmetic": ("f32 operands as split-f16 pairs (x = x1 + 2^-11 x2) on v_mfma_f32_16x16x32_f16, 3 exact products "
                       "per f32 MAC, f32 accumulate; norms/softmax/DP in f32 (DP f32/f64 as the reference)"
                       if args.precision == "split" else
                       "opt-in fast mode: encoder GEMMs on the f16 high planes alone (one product per MAC, f32 "
                       "accumulate); attention, grouped positional conv and UNet head split-f16x3; norms/softmax/DP f32"),
        "config": {"workload": f"{config_name(args.encoder, world, B, args.seconds)}"
                               f"{'' if args.chunk_seconds is None else f', chunked {args.chunk_seconds:g} s windows'}: "
                               f"B={B} x {args.seconds:g} s 16 kHz utterances per GPU, "
                               f"{ {'base': 'Hubert-base (cnhubert arch)', 'large': 'Hubert-large (cnhubert-large arch)', 'soft': 'HubertSoft'}[args.encoder]}"
                               f" + UNet head + Viterbi; full infer path wave({'host, H2D in the step' if args.host_input else 'HBM'})->boundaries(host), host assembly "
                               f"pipelined one batch behind the GPU",
                   "encoder": encoder, "do_normalize": bool(task.unitsEncoder.model.arch.do_normalize),
                   "global_batch": world * B, "seconds_per_utterance": args.seconds, "dp_frames": n_frames,
                   "states": len(ph_seqs[0]), "parallelism": f"utterance-dp{world}", "precision": args.precision},
        "frames_per_s": frames_ps,
        "ranks": devices,
        "hubert_frames_per_s": world * B * task.unitsEncoder.model.frame_lengths(int(round(args.seconds * 16000)))
                               * args.steps / el,
        "realtime_factor": value,
        "encoder_tflops": world * B * (hub_flops + head_flops) * args.steps / el / 1e12,
        "roofline": {"bound": "mfma", "kernel": probe_name, "achieved": achieved, "peak": mfma_peak(probe_name),
                     "unit": "TFLOP/s", "frac": achieved / mfma_peak(probe_name) if achieved else None,
                     "peak_basis": ("f16 MFMA dense peak (one-product f16 mode)" if probe_name.endswith(", true>")
                                    else "f32-equivalent FLOPs of the split-f16 scheme: 3 f16 MFMA products per f32 "
                                    "MAC, 2516.6 TF f16 dense / 3" if probe_name.startswith("gemm_split_kernel")
                                    else "f32 MFMA dense peak"),
                     "traffic": traffic, "launches": ps["launches"], "avg_launch_ms": ps["avg_ms"],
                     "timed_steps_probed": len(range(0, args.steps, max(args.probe_every, 1))),
                     "flops_per_launch": ps["avg_flops"],
                     "mfma_busy": pmc.get("mfma_busy") if pmc else None,
                     "clock_ghz": pmc.get("clock_ghz") if pmc else None,
                     "pmc_source": os.path.relpath(args.pmc_file, REPO) if pmc else None},
    }
    if probe_name.startswith("gemm_split_kernel") and achieved:
        # context, not the contract's peak: MI355X_MICROARCH.md 'DVFS give-back' item 1 measures a plain bf16 GEMM
        # on random data at 1247 TF/s (the chip holds ~1.9 GHz under dense MFMA load), the rate a random-data f16
        # MFMA loop can sustain; the split scheme's f32-equivalent share of it is a third (one product: all of it)
        rd = RANDOM_DATA_F16_TFLOPS / (1 if probe_name.endswith(", true>") else 3)
        out["roofline"]["random_data_mfma_rate"] = rd
        out["roofline"]["frac_of_random_data_rate"] = achieved / rd
    if len(step_ev) > 2:
        # where the timed region's time goes: step-start to step-start intervals on the device, and what the wall clock
        # holds beyond them (the drain: the last batch's side pass + assembly after the last step's start)
        iv = [step_ev[i].elapsed_time(step_ev[i + 1]) for i in range(len(step_ev) - 1)]
        srt = sorted(iv)
        out["timed_step_profile"] = {
            "first_interval_ms": iv[0], "median_interval_ms": srt[len(srt) // 2], "max_interval_ms": srt[-1],
            "sum_intervals_ms": sum(iv), "wall_ms": el * 1e3, "wall_minus_intervals_ms": el * 1e3 - sum(iv),
            "note": "device time between consecutive timed steps' starts; wall_minus_intervals = the last step, its "
                    "drain and the host work around the timed region"}
    if world == 1 and args.sustained_s > 0 and args.chunk_seconds is None:
        n0 = len(host_t)
        out["sustained"] = sustained(run, args.sustained_s, B * args.seconds, out["ms_per_step"])
        del host_t[n0:]
    c3 = config3_batch(args, world)
    if c3:
        # BASELINE config 3 (512 x 10 s over the node) measured after the weak-scaling region, whose per-GPU batch
        # stays at config 2's 32 so the driver's N = 1..8 curve compares equal per-GPU work
        inp3 = make_inputs(c3, args.seconds, args.words, seed0=7000 * (rank + 1))
        inp3 = (torch.from_numpy(inp3[0]).to(dev), None) + inp3[1:]
        run(1, inp3)
        _, el3 = timed(args.steps, inp3)
        out["config3"] = {"workload": f"config 3: global batch {world * c3} x {args.seconds:g} s ({c3} per GPU, "
                                      f"{world} GPUs), same path and timing protocol", "per_gpu_batch": c3,
                          "global_batch": world * c3, "steps": args.steps, "ms_per_step": el3 / args.steps * 1e3,
                          "value": world * c3 * args.seconds * args.steps / el3, "unit": "audio_s/s",
                          "frames_per_s": world * c3 * n_frames * args.steps / el3}
    def extra_block(workload, tk, b, seconds, words, steps, warmup):
        """Another BASELINE config on this GPU after the headline's timed region, with the same path and protocol
        (warmup census of the MFMA kernels, then exactly ``steps`` timed steps between synchronises): its rate, DP
        frames/s, the dominant GEMM's and the attention's fractions of the split ceiling (HIP events)."""
        n0 = len(host_t)
        x = make_inputs(b, seconds, words, seed0=5000)
        inp = (torch.from_numpy(x[0]).to(dev), None) + x[1:]
        cen = ops.KernelProbe(None)
        ops.PROBE = cen
        run(warmup, inp, tk)
        ops.PROBE = None
        torch.cuda.synchronize()
        name = cen.dominant()
        attn = ops.attention_split_probe_name()
        pr = ops.KernelProbe(name, extra=(attn,))
        ops.PROBE = pr
        r, e = timed(steps, inp, tk)
        ops.PROBE = None
        del host_t[n0:]
        blk = {"workload": workload, "per_gpu_batch": b, "seconds_per_utterance": seconds, "states": len(x[1][0]),
               "steps": steps, "warmup": warmup, "ms_per_step": e / steps * 1e3,
               "value": b * seconds * steps / e, "unit": "audio_s/s",
               "frames_per_s": b * r[0]["T"] * steps / e, "dp_frames": r[0]["T"]}
        for key, kname in (("dominant_kernel", name), ("attention", attn)):
            s = pr.summary(kname)
            if s["launches"]:
                ach = s["avg_flops"] / (s["avg_ms"] * 1e-3) / 1e12
                blk[key] = {"kernel": kname, "achieved": ach, "peak": mfma_peak(kname), "unit": "TFLOP/s",
                            "frac": ach / mfma_peak(kname), "avg_launch_ms": s["avg_ms"], "launches": s["launches"]}
        torch.cuda.synchronize()
        return blk

    if (world == 1 and not args.no_extra_configs and args.encoder == "base" and args.seconds == 10.0 and B == 32
            and args.chunk_seconds is None and not args.serial and args.precision == "split" and not args.host_input):
        # BASELINE configs 4 and 5 on this GPU, driver-observed in the same line (verdict r04 item 4): config 4's
        # per-GPU shard (Hubert-large 24L, 32 x 10 s) and config 5 unchunked (one 300 s utterance, the reference's
        # whole-wave encoding, tools/encoder.py:36-60; its DP held for the next encoder's attention launches)
        ck4 = synth_checkpoint(encoder="cnhubert-large", model_path="synth:0", seed=1)
        t4 = ForcedAlignmentTask(**ck4["hyper_parameters"], state_dict=ck4["state_dict"], device=dev)
        t4.on_predict_start()
        xs = max(3, min(args.steps, 10))
        out["config4"] = extra_block("config 4 geometry: Hubert-large (cnhubert-large arch, 24 layers) + UNet head + "
                                     "Viterbi, 32 x 10 s per GPU (config 4 is 256 over 8 GPUs)", t4, 32, 10.0,
                                     args.words, xs, 2)
        del t4
        out["config5"] = extra_block("config 5: one 300 s utterance, unchunked (whole-wave encoding), Hubert-base, "
                                     "600 two-phone words (S = 1801), 1 GPU", task, 1, 300.0, 600, 10, 2)
    if args.chunk_seconds is not None:
        out["chunk_agreement"] = chunk_agreement(task, wav_dev, ph_seqs, word_seqs, p2ws, args.chunk_seconds)
    if world == 1 and args.chunk_seconds is None and not args.serial:
        out["step_breakdown"] = step_breakdown(task, wav_dev, ph_seqs, word_seqs, p2ws, args.steps, el / args.steps)
    iso = ops.KernelProbe("-", extra=SECONDARY)       # isolated serial steps for the secondary rooflines
    ops.PROBE = iso
    for _ in range(2):
        torch.cuda.synchronize()
        task.decoder.assemble(task.align_batch(wav_dev, ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False,
                                               chunk_seconds=args.chunk_seconds), ph_seqs, word_seqs, p2ws)
    torch.cuda.synchronize()
    ops.PROBE = None
    out["secondary"] = secondary_rooflines(iso, pipe, n_frames, len(ph_seqs[0]))
    ht = host_t[max(args.warmup, 1):max(args.warmup, 1) + args.steps]      # the timed steps
    avg = lambda i: 1e3 * sum(h[i] for h in ht) / max(len(ht), 1)  # noqa: E731
    out["host_cpu"] = {
        "enqueue_cpu_ms_per_step": avg(2), "assemble_cpu_ms_per_step": avg(3), "process_cpu_ms_per_step": avg(4),
        "enqueue_wall_ms_per_step": avg(0), "wait_assemble_wall_ms_per_step": avg(1),
        "threads_cpu_ms_per_step": thread_cpu_diff(thr0, thr1, args.steps),
        "gc_pauses": {"collections": len(gc_log), "by_generation": [sum(1 for g, _ in gc_log if g == k) for k in range(3)],
                      "max_ms": max((d for _, d in gc_log), default=0.0), "total_ms": sum(d for _, d in gc_log)},
        "note": "rank 0's host cost per timed step: CPU seconds of the launching thread for the GPU half's enqueue "
                "(ctypes launches, allocator, events) and for the previous batch's wait + interval assembly, and "
                "the whole process's CPU (all threads; per thread over the timed region in threads_cpu_ms_per_step, "
                "'main' = the launching thread); the GPU step is ms_per_step"}
    if rank == 0:
        import contextlib
        with contextlib.redirect_stdout(sys.stderr):         # the writers' progress prints stay off the JSON line
            out["host_io"] = host_io(wav_np, res, args.seconds)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wav_np, ph_seqs, word_seqs, p2ws, ckpt, args.cpu_sample_s, encoder)
    if rank == 0:
        ht = host_t[-args.steps:]
        print(f"host per step: enqueue {1e3 * sum(h[0] for h in ht) / len(ht):.2f} ms, wait+assemble "
              f"{1e3 * sum(h[1] for h in ht) / len(ht):.2f} ms", file=sys.stderr, flush=True)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
