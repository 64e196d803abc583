"""Model-level parity of the HIP Hubert encoders and UNet lattice head.

1. Against the reference's own outputs (tests/golden, produced by gen_golden.py from the reference modules).
2. At BASELINE config sizes (10 s utterances, batched) against the torch-CPU oracle (oracle/hubert_cpu.py,
   itself pinned to the goldens by tests/test_oracle_hubert.py).
Tolerances (abs, on O(1) post-LN activations): 1e-3 for 12-layer encoders, 2e-4 for the UNet logits; the
north-star bar for per-frame log-probs is 1e-4 (test_pipeline_gpu.py).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _maxerr(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def test_hf_base_vs_reference_golden():
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    z = np.load(os.path.join(GOLDEN, "hubert_hf_base.npz"))
    arch = synth.arch_cnhubert_base(do_normalize=True)
    enc = HubertEncoder(arch, synth.synth_hubert_state_dict(arch, seed=11))
    wav = torch.from_numpy(z["wav"])[None].cuda()
    feats = enc.feature_extractor(torch.from_numpy(z["hf_base_input"])[None].cuda())
    e_feat = _maxerr(feats[0].cpu().numpy(), z["hf_base_feats"].T)
    out = enc(wav)[0].cpu().numpy()
    e_out = _maxerr(out, z["hf_base_out"])
    print(f"hf base: feature extractor max err {e_feat:.2e}, final {e_out:.2e}")
    assert e_feat < 1e-4 and e_out < 1e-3


def test_hf_large_vs_reference_golden():
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    z = np.load(os.path.join(GOLDEN, "hubert_hf_large.npz"))
    arch = synth.arch_cnhubert_large(layers=2, do_normalize=False)
    enc = HubertEncoder(arch, synth.synth_hubert_state_dict(arch, seed=12))
    out = enc(torch.from_numpy(z["input"])[None].cuda())[0].cpu().numpy()
    e = _maxerr(out, z["out"])
    print(f"hf large(2L): max err {e:.2e}")
    assert e < 1e-3


def test_hubertsoft_vs_reference_golden():
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    z = np.load(os.path.join(GOLDEN, "hubert_soft.npz"))
    arch = synth.arch_hubertsoft()
    enc = HubertEncoder(arch, synth.synth_hubert_state_dict(arch, seed=13))
    out = enc(torch.from_numpy(z["wav"])[None].cuda())[0].cpu().numpy()
    e = _maxerr(out, z["out"])
    print(f"hubertsoft: max err {e:.2e}")
    assert out.shape == z["out"].shape and e < 1e-3


def test_unet_head_vs_reference_golden():
    from hubertfa_amd import synth
    from hubertfa_amd.unet import LatticeHead
    z = np.load(os.path.join(GOLDEN, "unet_head.npz"))
    ua = synth.UNetArch()
    head = LatticeHead(ua, synth.synth_unet_state_dict(ua, seed=21))
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        Tp = head.padded_len(T)
        xp = np.zeros((1, Tp, ua.input_dims), np.float32)
        xp[:, :T] = x
        lg = head.logits(torch.from_numpy(xp).cuda())[0, :T].cpu().numpy()
        e = _maxerr(lg, z[f"T{T}_logits"])
        print(f"unet T={T}: max err {e:.2e}")
        assert e < 2e-4


def test_full_size_batch_vs_oracle():
    """Config 2 geometry (10 s @16 kHz) at B=2: HIP encoder + gather + UNet vs the CPU oracle."""
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    from oracle import hubert_cpu
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    enc = HubertEncoder(arch, sd)
    wav = np.stack([synth.synth_audio(160000, seed=s) for s in (1, 2)])
    got = enc(torch.from_numpy(wav).cuda()).cpu().numpy()
    ref = hubert_cpu.hubert_forward(arch, sd, torch.from_numpy(wav)).numpy()
    e = _maxerr(got, ref)
    print(f"10 s x2 hubert base: max err {e:.2e}")
    assert got.shape == (2, 499, 768) and e < 2e-3
