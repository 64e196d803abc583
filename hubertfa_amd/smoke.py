"""One small end-to-end invocation of the hot path on cuda:0, checked against the CPU oracle
(used by ``__graft_entry__.smoke()``; the oracle import is local to this checker)."""
from __future__ import annotations

import numpy as np
import torch


def run_smoke(seconds: float = 2.0, B: int = 2) -> dict:
    import yaml
    from . import synth
    from .task import ForcedAlignmentTask, synth_checkpoint
    from oracle import decode as odec, hubert_cpu, resample as ores   # checker only

    assert torch.cuda.is_available(), "smoke() needs a GPU"
    dev = torch.device("cuda", 0)
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    vocab = yaml.safe_load(ckpt["hyper_parameters"]["vocab_text"])
    n16 = int(seconds * 16000)
    wav = np.stack([synth.synth_audio(n16, seed=50 + i) for i in range(B)])
    d = synth.synth_dictionary()
    labs = [synth.synth_lab(6, d, seed=60 + i).split(" ") for i in range(B)]
    ph_seqs, p2ws = [], []
    for ws in labs:
        ph, pw = ["SP"], [-1]
        for wi, w in enumerate(ws):
            for p in d[w]:
                ph.append(p)
                pw.append(wi)
            ph.append("SP")
            pw.append(-1)
        ph_seqs.append(ph)
        p2ws.append(pw)
    res = task.align_batch(torch.from_numpy(wav).to(dev), ph_seqs, labs, p2ws, wav_sr=16000)
    torch.cuda.synchronize()

    # CPU oracle of the same utterances
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    ua = synth.UNetArch(vocab_size=vocab["vocab_size"])
    usd = {k: v.numpy() for k, v in ckpt["state_dict"].items()}
    n_match = 0
    for b in range(B):
        x44 = ores.resample(torch.from_numpy(wav[b:b + 1]), 16000, 44100, 6)
        units = hubert_cpu.hubert_forward(arch, sd, ores.resample(x44, 44100, 16000, 128))
        n44 = x44.shape[-1]
        nf = n44 // 512 + 1
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(nf)).long(),
                          max=units.shape[1] - 1)
        logits = hubert_cpu.unet_head_forward(ua, usd, units[:, idx])
        ref = odec.decode(vocab, logits[:, :, 2:], logits[:, :, 0], n44 / 44100, ph_seqs[b], labs[b], p2ws[b])
        assert list(ref[0]) == list(res[b]["ph_seq"]), "phone sequence differs from the oracle"
        n_match += int(np.array_equal(ref[5]["tint"], res[b]["ph_time_int"]))
        np.testing.assert_allclose(res[b]["ph_intervals"], ref[1], atol=2 * 512 / 44100)
    assert n_match == B, f"boundary indices matched the oracle on only {n_match}/{B} utterances"
    print(f"smoke OK: {B} x {seconds:g} s, boundary-exact utterances {n_match}/{B}")
    return {"utterances": B, "boundary_exact": n_match}
