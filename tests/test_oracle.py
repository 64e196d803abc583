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


def test_wav_readers_against_scipy(tmp_path):
    """The WAV container decoding, cross-checked with an independent parser (scipy.io.wavfile, the one present here;
    torchaudio is absent): files written by scipy in int16 / int32 / uint8 / float32 / float64, mono and stereo, odd
    lengths, read by the numpy restatement (oracle/wav_read.py) and by libhfa's native reader (host code, no GPU),
    equal scipy's samples under torchaudio's documented normalisation (int16 / 2^15, int32 / 2^31, uint8 (x-128)/128,
    floats as stored).  Pins the container parsing and the scaling formulas; torchaudio's own output stays unpinned."""
    wavfile = pytest.importorskip("scipy.io.wavfile")
    from oracle.wav_read import read_wav_np
    rng = np.random.default_rng(3)
    scale = {np.int16: 2.0 ** 15, np.int32: 2.0 ** 31}
    native = None
    try:
        from hubertfa_amd import _lib, wav_io
        if os.path.exists(_lib.LIB_PATH):
            native = wav_io.read_wav
    except Exception:  # noqa: BLE001 — torch / the library absent: the restatement alone is checked
        native = None
    for dt in (np.int16, np.int32, np.uint8, np.float32, np.float64):
        for ch in (1, 2):
            n = int(rng.integers(1, 5000))
            if dt is np.uint8:
                x = rng.integers(0, 256, (n, ch)).astype(dt)
            elif dt in scale:
                info = np.iinfo(dt)
                x = rng.integers(info.min, info.max, (n, ch), endpoint=True).astype(dt)
            else:
                x = rng.uniform(-1, 1, (n, ch)).astype(dt)
            if ch == 1:
                x = x[:, 0]
            p = tmp_path / f"{np.dtype(dt).name}_{ch}.wav"
            wavfile.write(p, 22050, x)
            sr, y = wavfile.read(p)
            y = y.reshape(n, ch).T
            if dt is np.uint8:
                want = (y.astype(np.float32) - 128.0) / 128.0
            elif dt in scale:
                want = (y.astype(np.float64) / scale[dt]).astype(np.float32)
            else:
                want = y.astype(np.float32)
            got, gsr = read_wav_np(p)
            assert gsr == sr == 22050 and got.dtype == np.float32 and np.array_equal(got, want), (dt, ch)
            if native is not None:
                got2, sr2 = native(p)
                assert sr2 == 22050 and np.array_equal(got2, want), (dt, ch)
