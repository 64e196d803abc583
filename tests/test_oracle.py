"""The CPU oracle is pinned against the reference's own outputs (tests/golden/*, made by gen_golden.py)."""
import json
import os

import numpy as np
import pytest

from oracle import decode as od

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dp_cases():
    z = np.load(os.path.join(GOLDEN, "dp_cases.npz"))
    return z, int(z["n"])


def test_oracle_forward_pass_bit_exact():
    z, n = _dp_cases()
    for c in range(n):
        p = f"c{c}_"
        ids = z[p + "ids"].astype(np.int64)
        pl, E, nE, curr, dp, bt, pad = od.lattice_inputs(ids, z[p + "ph_prob_log"], z[p + "edge_prob"])
        T, S = dp.shape
        d2, b2, c2 = od.forward_pass(T, S, pl, nE, E, curr, dp, bt, ids, pad)
        assert np.array_equal(d2.view(np.int32), z[p + "dp"].view(np.int32)), f"dp mismatch case {c}"
        assert np.array_equal(b2, z[p + "bt"].astype(np.int32)), f"bt mismatch case {c}"
        assert np.array_equal(c2.view(np.int64), z[p + "curr"].view(np.int64)), f"curr mismatch case {c}"


def test_oracle_backtrack_matches_reference():
    z, n = _dp_cases()
    for c in range(n):
        p = f"c{c}_"
        idx, tint, fc = od._decode(z[p + "ids"].astype(np.int64), z[p + "ph_prob_log"], z[p + "edge_prob"])
        assert np.array_equal(idx, z[p + "ph_idx_seq"]), c
        assert np.array_equal(tint, z[p + "ph_time_int"]), c
        np.testing.assert_allclose(fc, z[p + "frame_confidence"], rtol=2e-6, atol=0, equal_nan=True)


def test_oracle_decode_matches_reference():
    import torch
    meta = json.load(open(os.path.join(GOLDEN, "decode_cases.json")))
    z = np.load(os.path.join(GOLDEN, "decode_cases.npz"))
    vocab = meta["vocab"]
    for ci, case in enumerate(meta["cases"]):
        lt = torch.from_numpy(z[f"c{ci}_logits"])
        ph, ph_iv, w, w_iv, conf, extra = od.decode(vocab, lt[:, :, 2:], lt[:, :, 0], case["wav_length"],
                                                    case["ph_seq"], case["word_seq"], case["ph_idx_to_word_idx"])
        assert list(ph) == case["ph_seq_pred"]
        assert list(w) == case["word_seq_pred"]
        assert np.array_equal(extra["idx"], z[f"c{ci}_ph_idx_seq"])
        assert np.array_equal(extra["tint"], z[f"c{ci}_ph_time_int"])
        np.testing.assert_allclose(ph_iv, z[f"c{ci}_ph_intervals"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(w_iv, z[f"c{ci}_word_intervals"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(conf, case["total_confidence"], rtol=1e-5)
