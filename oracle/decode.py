"""TEST INFRASTRUCTURE ONLY — numpy + C restatement of AlignmentDecoder (tools/alignment_decoder.py).

``forward_pass`` / ``backtrack`` call the C oracle (viterbi_oracle.c); ``decode`` restates the host logic of
``AlignmentDecoder.decode`` (:26-143) with torch-CPU softmax/log_softmax/sigmoid exactly as the reference calls
them (:56-71).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.hfa_oracle_forward.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, P, P, P, ctypes.c_int]
        L.hfa_oracle_forward.restype = None
        L.hfa_oracle_backtrack.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
        L.hfa_oracle_backtrack.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def forward_pass(T, S, prob_log, not_edge_prob_log, edge_prob_log, curr_ph_max_prob_log, dp, backtrack_s,
                 ph_seq_id, prob3_pad_len):
    """In-place numpy semantics of AlignmentDecoder.forward_pass (alignment_decoder.py:170-230)."""
    pl = np.ascontiguousarray(prob_log, np.float32)
    nE = np.ascontiguousarray(not_edge_prob_log, np.float32)
    E = np.ascontiguousarray(edge_prob_log, np.float32)
    cu = np.ascontiguousarray(curr_ph_max_prob_log, np.float64)
    d = np.ascontiguousarray(dp, np.float32)
    bt = np.ascontiguousarray(backtrack_s, np.int32)
    ids = np.ascontiguousarray(ph_seq_id, np.int32)
    lib().hfa_oracle_forward(int(T), int(S), _p(pl), _p(nE), _p(E), _p(cu), _p(d), _p(bt), _p(ids),
                             int(prob3_pad_len))
    return d, bt, cu


def backtrack(dp, bt, ph_seq_id):
    T, S = dp.shape
    d = np.ascontiguousarray(dp, np.float32)
    b = np.ascontiguousarray(bt, np.int32)
    ids = np.ascontiguousarray(ph_seq_id, np.int32)
    idx = np.zeros(T, np.int32)
    tint = np.zeros(T, np.int32)
    fc = np.zeros(T, np.float32)
    n = lib().hfa_oracle_backtrack(T, S, _p(d), _p(b), _p(ids), _p(idx), _p(tint), _p(fc))
    return idx[:n], tint[:n], fc


def lattice_inputs(ph_seq_id, ph_prob_log, edge_prob):
    """_decode's lattice preparation and DP initialisation (alignment_decoder.py:239-257)."""
    S = len(ph_seq_id)
    T = ph_prob_log.shape[0]
    prob_log = ph_prob_log[:, ph_seq_id]
    E = np.log(edge_prob + 1e-6).astype("float32")
    nE = np.log(1 - edge_prob + 1e-6).astype("float32")
    curr = np.full(S, -np.inf)
    dp = np.full((T, S), -np.inf, dtype="float32")
    bt = np.full_like(dp, -1, dtype="int32")
    dp[0, 0] = prob_log[0, 0]
    curr[0] = prob_log[0, 0]
    if ph_seq_id[0] == 0 and prob_log.shape[-1] > 1:
        dp[0, 1] = prob_log[0, 1]
        curr[1] = prob_log[0, 1]
    pad = 2 if S >= 2 else 1
    return prob_log, E, nE, curr, dp, bt, pad


def _decode(ph_seq_id, ph_prob_log, edge_prob):
    T = ph_prob_log.shape[0]
    S = len(ph_seq_id)
    prob_log, E, nE, curr, dp, bt, pad = lattice_inputs(ph_seq_id, ph_prob_log, edge_prob)
    dp, bt, curr = forward_pass(T, S, prob_log, nE, E, curr, dp, bt, ph_seq_id, pad)
    return backtrack(dp, bt, ph_seq_id)


def decode(vocab, ph_frame_logits, ph_edge_logits, wav_length, ph_seq, word_seq=None, ph_idx_to_word_idx=None,
           hop_length=512, sample_rate=44100):
    """Restatement of AlignmentDecoder.decode (alignment_decoder.py:26-143); logits are torch CPU tensors."""
    import torch

    frame_length = hop_length / sample_rate
    ph_seq_id = np.array([vocab["vocab"][ph] for ph in ph_seq])
    ph_mask = np.zeros(vocab["vocab_size"])
    ph_mask[ph_seq_id] = 1
    ph_mask[0] = 1
    ph_mask = torch.from_numpy(ph_mask)
    if word_seq is None:
        word_seq = ph_seq
        ph_idx_to_word_idx = np.arange(len(ph_seq))
    if wav_length is not None:
        n = int((wav_length * sample_rate + 0.5) / hop_length)
        ph_frame_logits = ph_frame_logits[:, :n, :]
        ph_edge_logits = ph_edge_logits[:, :n]
    ph_mask = ph_mask.unsqueeze(0).unsqueeze(0).logical_not() * 1e9
    x = ph_frame_logits.float() - ph_mask.float()
    ph_prob_log = torch.log_softmax(x, dim=-1).squeeze(0).numpy().astype("float32")
    e = ((torch.sigmoid(ph_edge_logits.float()) - 0.1) / 0.8).clamp(0.0, 1.0).squeeze(0).numpy().astype("float32")
    T = ph_prob_log.shape[0]
    edge_diff = np.concatenate((np.diff(e, axis=0), [0]), axis=0)
    edge_prob = (e + np.concatenate(([0], e[:-1]))).clip(0, 1)
    idx, tint, fc = _decode(ph_seq_id, ph_prob_log, edge_prob)
    total_conf = np.exp(np.mean(np.log(fc + 1e-6)) / 3)
    frac = (edge_diff[tint] / 2).clip(-0.5, 0.5)
    tp = frame_length * np.concatenate([tint.astype("float32") + frac, [T]])
    iv = np.stack([tp[:-1], tp[1:]], axis=1)
    ph_pred, ph_iv, w_pred, w_iv = [], [], [], []
    last = -1
    for i, pi in enumerate(idx):
        if ph_seq[pi] == "SP":
            continue
        ph_pred.append(ph_seq[pi])
        ph_iv.append(iv[i, :])
        wi = ph_idx_to_word_idx[pi]
        if wi == last:
            w_iv[-1][1] = iv[i, 1]
        else:
            w_pred.append(word_seq[wi])
            w_iv.append([iv[i, 0], iv[i, 1]])
            last = wi
    return (np.array(ph_pred), np.array(ph_iv).clip(min=0, max=None), np.array(w_pred),
            np.array(w_iv).clip(min=0, max=None), total_conf, dict(idx=idx, tint=tint, fc=fc, edge_prob=edge_prob,
                                                                    ph_prob_log=ph_prob_log, edge_diff=edge_diff))
