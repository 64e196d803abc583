"""The north-star bars against the REFERENCE ITSELF at BASELINE config-2 geometry (one 10 s utterance: 160 000
encoder samples, N44 = 441 000, 862 grid frames, T = 861 DP frames, S = 88 states, V = 63).

tests/golden/e2e_10s.npz holds what the reference computed (tests/golden/gen_golden.py gen_e2e10s): its
UnitsEncoder (tools/encoder.py:36-60) over HF HubertModel base 12L / HF Hubert-large 24L stable-LN / bshall
HubertSoft, its UNetBackbone + head and forward split (forced_alignment.py:284-292), its AlignmentDecoder.decode
(tools/alignment_decoder.py:26-143) — with the product's default synthetic weights (synth:0 encoders, the
synth_checkpoint(seed=1) UNet/head).  The same 16 kHz wave is fed to the HIP encoder here; the resamplers in front
of it stay unpinned (torchaudio is absent), so the grid is built from N44 exactly as encoder.py:56-59 does.

Bars: per-frame log-probs (ph_prob_log at the sequence's phones) within 1e-4 of the reference's; ph_idx_seq and
ph_time_int bit-exact; word / phone sequences identical; intervals and confidence to f32 round-off.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LOGPROB_TOL = 1e-4
ENCODERS = {"base": "cnhubert", "large": "cnhubert-large", "soft": "hubertsoft"}


def _fixture():
    z = np.load(os.path.join(GOLDEN, "e2e_10s.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "e2e_10s.json")))
    return z, meta


def _task(name, precision):
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    ck = synth_checkpoint(encoder=ENCODERS[name], model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=torch.device("cuda"))
    task.on_predict_start()
    task.unitsEncoder.model.precision = task.head.precision = precision
    return task


def _gpu_path(task, wav16, meta):
    """16 kHz wave -> HIP Hubert -> grid gather -> UNet + head -> lattice prologue -> Viterbi -> boundaries."""
    from hubertfa_amd import ops
    n44 = meta["n44"]
    ue = task.unitsEncoder
    x = torch.from_numpy(wav16)[None].cuda()
    units = ue.model(x)                                               # [1, L, C]
    n_frames, ratio = ue.grid(n44, 44100, 512)                        # encoder.py:56-57 at the 44.1 kHz grid
    feats = ops.units_gather(units.contiguous(), n_frames, task.head.padded_len(n_frames), ratio)
    args = ([meta["ph_seq"]], [meta["word_seq"]], [meta["ph_idx_to_word_idx"]])
    dev_out = task.decode_device(feats, n_frames, [n44 / 44100], *args)
    lattice = dev_out["lattice"]["prob_log"][0].cpu().numpy()
    res = task.decoder.assemble(dev_out, *args)[0]
    return units[0].cpu().numpy(), feats[0, :n_frames].cpu().numpy(), lattice, res


@pytest.mark.parametrize("precision", ["split", "f32"])
@pytest.mark.parametrize("name", ["base", "large", "soft"])
def test_10s_vs_reference(name, precision):
    z, meta = _fixture()
    wav16 = z["wav16_s16"].astype(np.float32) / 32768.0
    task = _task(name, precision)
    units, feats, lattice, res = _gpu_path(task, wav16, meta)
    vocab = task.vocab
    ids = np.array([vocab["vocab"][p] for p in meta["ph_seq"]])
    ref_pl = z[f"{name}_ph_prob_log"][:, ids]
    T = ref_pl.shape[0]
    assert res["T"] == T == 861
    if name == "base":                     # the gathered Hubert units themselves (f32-class contractions)
        uerr = float(np.abs(feats - z["base_units"]).max())
        assert uerr < 2e-3, f"units error {uerr:.2e}"
    err = float(np.abs(lattice[:T, :len(ids)] - ref_pl).max())
    print(f"[{name}/{precision}] per-frame log-prob error vs the reference: {err:.2e}")
    assert err < LOGPROB_TOL, f"{name}/{precision}: per-frame log-prob error {err:.2e} > {LOGPROB_TOL}"
    assert np.array_equal(res["ph_idx_seq"], z[f"{name}_ph_idx_seq"]), "phone path differs from the reference"
    assert np.array_equal(res["ph_time_int"], z[f"{name}_ph_time_int"]), "boundary frames differ from the reference"
    enc = meta["encoders"][name]
    assert list(res["ph_seq"]) == enc["ph_seq_pred"] and list(res["word_seq"]) == enc["word_seq_pred"]
    np.testing.assert_allclose(res["ph_intervals"], z[f"{name}_ph_intervals"], atol=1e-5)
    np.testing.assert_allclose(res["word_intervals"], z[f"{name}_word_intervals"], atol=1e-5)
    # frame confidence = exp(dp[t, s_t] - dp[t-1, s_t-1]) is a sum of lattice terms that include
    # log(1 - edge + 1e-6): where the edge probability rounds to ~1 in f32, one ulp of it (6e-8) moves that term by
    # up to 0.06 — the reference's own formula is that ill-conditioned there.  So: both exp's underflow together,
    # 98 % of the frames agree to 1e-3 in the log domain, and the utterance confidence to 1e-3.
    fc, rc = res["frame_confidence"].astype(np.float64), z[f"{name}_frame_confidence"].astype(np.float64)
    tiny = 1e-30
    mism = (fc > tiny) != (rc > tiny)                 # underflow disagreements only right at the threshold
    assert np.all(np.maximum(fc[mism], rc[mism]) < 1e-25)
    both = (fc > tiny) & (rc > tiny)
    lg = np.abs(np.log(fc[both]) - np.log(rc[both]))
    print(f"[{name}/{precision}] log frame-confidence error: median {np.median(lg):.1e}, "
          f"{(lg > 1e-3).mean() * 100:.1f} % above 1e-3, max {lg.max():.1e}")
    assert (lg > 1e-3).mean() < 0.02
    np.testing.assert_allclose(res["confidence"], enc["confidence"], rtol=1e-3)


def test_10s_reference_lattice_through_gpu_dp():
    """Given the reference's own lattice (its ph_prob_log and its f64 edge_prob, captured at _decode's entry), the
    HIP forward pass + backtrack reproduce its boundaries bit-exactly and its frame confidences to expf's round-off
    at T = 861 (the DP's parity does not depend on the encoder)."""
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    from hubertfa_amd import synth
    z, meta = _fixture()
    vocab = synth.synth_vocab(62)
    dec = AlignmentDecoder(vocab, {"hop_length": 512, "sample_rate": 44100})
    ids = np.array([vocab["vocab"][p] for p in meta["ph_seq"]])
    for name in ENCODERS:
        idx, tint, fconf = dec._decode(ids, z[f"{name}_ph_prob_log"], z[f"{name}_edge_prob"])
        assert np.array_equal(idx, z[f"{name}_ph_idx_seq"]) and np.array_equal(tint, z[f"{name}_ph_time_int"]), name
        np.testing.assert_allclose(fconf, z[f"{name}_frame_confidence"], rtol=2e-6, atol=1e-7)
