"""The torch-CPU float oracle is pinned against outputs of the reference modules (gen_golden.py).

Tolerances are what the data supports: the oracle runs the same torch-CPU ops as transformers / the reference
modules, so it matches them to a few f32 ulps of the activations (measured 0 - 4e-6 on the 1 s goldens,
3e-6 on the 10 s base units, 1.1e-5 - 2.0e-5 on the 10 s per-frame log-probs, boundaries bit-exact)."""
import os

import numpy as np
import torch

from hubertfa_amd import synth
from oracle import hubert_cpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_oracle_hf_base_matches_reference():
    z = np.load(os.path.join(GOLDEN, "hubert_hf_base.npz"))
    arch = synth.arch_cnhubert_base(do_normalize=True)
    sd = synth.synth_hubert_state_dict(arch, seed=11)
    out = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(z["wav"])[None])[0].numpy()
    np.testing.assert_allclose(out, z["hf_base_out"], atol=2e-5, rtol=0)


def test_oracle_hf_large_matches_reference():
    z = np.load(os.path.join(GOLDEN, "hubert_hf_large.npz"))
    arch = synth.arch_cnhubert_large(layers=2, do_normalize=False)
    sd = synth.synth_hubert_state_dict(arch, seed=12)
    out = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(z["input"])[None])[0].numpy()
    np.testing.assert_allclose(out, z["out"], atol=2e-5, rtol=0)


def test_oracle_hubertsoft_matches_reference():
    z = np.load(os.path.join(GOLDEN, "hubert_soft.npz"))
    arch = synth.arch_hubertsoft()
    sd = synth.synth_hubert_state_dict(arch, seed=13)
    out = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(z["wav"])[None])[0].numpy()
    np.testing.assert_allclose(out, z["out"], atol=2e-5, rtol=0)


def test_oracle_unet_head_matches_reference():
    z = np.load(os.path.join(GOLDEN, "unet_head.npz"))
    ua = synth.UNetArch()
    sd = synth.synth_unet_state_dict(ua, seed=21)
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        out = hubert_cpu.unet_head_forward(ua, sd, torch.from_numpy(x))[0].numpy()
        np.testing.assert_allclose(out, z[f"T{T}_logits"], atol=1e-4, rtol=0)


def test_oracle_10s_vs_reference():
    """BASELINE config-2 geometry, the whole lattice: oracle.hubert_cpu (base 12L, large 24L, hubertsoft) -> the
    grid gather -> UNet + head -> oracle.decode against the reference's own 10 s run (tests/golden/e2e_10s.npz):
    units to 2e-5, per-frame log-probs to 5e-5, boundaries bit-exact.  This is the pin that lets the GPU tests
    use the oracle at sizes the fixtures do not cover (batches, 24 layers x B, 300 s)."""
    import json
    from oracle import decode as odec
    z = np.load(os.path.join(GOLDEN, "e2e_10s.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "e2e_10s.json")))
    wav = torch.from_numpy(z["wav16_s16"].astype(np.float32) / 32768.0)[None]
    vocab = synth.synth_vocab(62)
    ids = np.array([vocab["vocab"][p] for p in meta["ph_seq"]])
    n44 = meta["n44"]
    nf = n44 // 512 + 1
    for name, arch in (("base", synth.arch_cnhubert_base()), ("large", synth.arch_cnhubert_large()),
                       ("soft", synth.arch_hubertsoft())):
        units = hubert_cpu.hubert_forward(arch, synth.synth_hubert_state_dict(arch, seed=0), wav)
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(nf)).long(),
                          max=units.shape[1] - 1)
        g = units[:, idx]
        if name == "base":
            np.testing.assert_allclose(g[0].numpy(), z["base_units"], atol=2e-5, rtol=0)
        ua = synth.UNetArch(input_dims=arch.out_channels, vocab_size=vocab["vocab_size"])
        lg = hubert_cpu.unet_head_forward(ua, synth.synth_unet_state_dict(ua, seed=1), g)
        ph, ph_iv, w, w_iv, conf, ex = odec.decode(vocab, lg[:, :, 2:], lg[:, :, 0], n44 / 44100, meta["ph_seq"],
                                                   meta["word_seq"], meta["ph_idx_to_word_idx"])
        err = float(np.abs(ex["ph_prob_log"][:, ids] - z[f"{name}_ph_prob_log"][:, ids]).max())
        assert err < 5e-5, (name, err)
        assert np.array_equal(ex["idx"], z[f"{name}_ph_idx_seq"]), name
        assert np.array_equal(ex["tint"], z[f"{name}_ph_time_int"]), name
        assert list(ph) == meta["encoders"][name]["ph_seq_pred"] and list(w) == meta["encoders"][name]["word_seq_pred"]
        np.testing.assert_allclose(ph_iv, z[f"{name}_ph_intervals"], atol=1e-6)
        np.testing.assert_allclose(conf, meta["encoders"][name]["confidence"], rtol=1e-5)
