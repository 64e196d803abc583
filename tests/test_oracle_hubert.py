"""The torch-CPU float oracle is pinned against outputs of the reference modules (gen_golden.py)."""
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
    np.testing.assert_allclose(out, z["hf_base_out"], atol=2e-4, rtol=0)


def test_oracle_hf_large_matches_reference():
    z = np.load(os.path.join(GOLDEN, "hubert_hf_large.npz"))
    arch = synth.arch_cnhubert_large(layers=2, do_normalize=False)
    sd = synth.synth_hubert_state_dict(arch, seed=12)
    out = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(z["input"])[None])[0].numpy()
    np.testing.assert_allclose(out, z["out"], atol=2e-4, rtol=0)


def test_oracle_hubertsoft_matches_reference():
    z = np.load(os.path.join(GOLDEN, "hubert_soft.npz"))
    arch = synth.arch_hubertsoft()
    sd = synth.synth_hubert_state_dict(arch, seed=13)
    out = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(z["wav"])[None])[0].numpy()
    np.testing.assert_allclose(out, z["out"], atol=2e-4, rtol=0)


def test_oracle_unet_head_matches_reference():
    z = np.load(os.path.join(GOLDEN, "unet_head.npz"))
    ua = synth.UNetArch()
    sd = synth.synth_unet_state_dict(ua, seed=21)
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        out = hubert_cpu.unet_head_forward(ua, sd, torch.from_numpy(x))[0].numpy()
        np.testing.assert_allclose(out, z[f"T{T}_logits"], atol=1e-4, rtol=0)
