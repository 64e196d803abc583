"""Host-side interval/word assembly of the alignment decoder (reference: tools/alignment_decoder.py:97-138).

numpy only (no torch): the host half of decoding, used by AlignmentDecoder.assemble, by the CLI's streamed export
(infer.py, from the raw boundary records) and by rank 0 after the multi-GPU gather; alignment_decoder re-exports
these names.
"""
from __future__ import annotations

import numpy as np


def assemble_intervals(ph_idx_seq, ph_time_int, edge_diff, T, frame_length, ph_seq, word_seq, ph_idx_to_word_idx):
    """Fractional boundaries and word grouping (alignment_decoder.py:103-138), numpy f64 as the reference.

    The phone / word loop of the reference runs as array operations (the host assembles every batch of the pipelined
    step while the GPU runs the next one, and the last batch's assembly is exposed): SP phones dropped by a mask, a
    word opened wherever the word index changes between kept phones, closed at its last phone.  The loop form
    (assemble_intervals_loop, the reference's statement order) is the fallback where the two could differ: a kept
    phone without a word (index -1, where the reference's first merge would index an empty list)."""
    ph_time_int = np.asarray(ph_time_int)
    edge_diff = np.asarray(edge_diff, dtype=np.float64)
    ph_time_fractional = (edge_diff[ph_time_int] / 2).clip(-0.5, 0.5)
    ph_time_pred = frame_length * np.concatenate([ph_time_int.astype("float32") + ph_time_fractional, [T]])
    ph_intervals = np.stack([ph_time_pred[:-1], ph_time_pred[1:]], axis=1)
    return _phones_words(ph_intervals, np.asarray(ph_idx_seq, dtype=np.int64), ph_seq, word_seq, ph_idx_to_word_idx)


def assemble_intervals_loop(ph_idx_seq, ph_time_int, edge_diff, T, frame_length, ph_seq, word_seq,
                            ph_idx_to_word_idx):
    """assemble_intervals in the reference's own statement order (alignment_decoder.py:103-138): the fallback and the
    check (tests/test_host.py) of the array form."""
    ph_time_int = np.asarray(ph_time_int)
    edge_diff = np.asarray(edge_diff, dtype=np.float64)
    ph_time_fractional = (edge_diff[ph_time_int] / 2).clip(-0.5, 0.5)
    ph_time_pred = frame_length * np.concatenate([ph_time_int.astype("float32") + ph_time_fractional, [T]])
    ph_intervals = np.stack([ph_time_pred[:-1], ph_time_pred[1:]], axis=1)
    return _assemble_loop(ph_intervals, ph_idx_seq, ph_seq, word_seq, ph_idx_to_word_idx)


def _assemble_loop(ph_intervals, ph_idx_seq, ph_seq, word_seq, ph_idx_to_word_idx):
    ph_seq_pred, ph_intervals_pred, word_seq_pred, word_intervals_pred = [], [], [], []
    word_idx_last = -1
    for i, ph_idx in enumerate(ph_idx_seq):
        if ph_seq[ph_idx] == "SP":
            continue
        ph_seq_pred.append(ph_seq[ph_idx])
        ph_intervals_pred.append(ph_intervals[i, :])
        word_idx = ph_idx_to_word_idx[ph_idx]
        if word_idx == word_idx_last:
            word_intervals_pred[-1][1] = ph_intervals[i, 1]
        else:
            word_seq_pred.append(word_seq[word_idx])
            word_intervals_pred.append([ph_intervals[i, 0], ph_intervals[i, 1]])
            word_idx_last = word_idx
    return (np.array(ph_seq_pred), np.array(ph_intervals_pred).clip(min=0, max=None), np.array(word_seq_pred),
            np.array(word_intervals_pred).clip(min=0, max=None))


def _phones_words(ph_intervals, idx, ph_seq, word_seq, ph_idx_to_word_idx):
    """assemble_intervals' phone / word selection from the [n, 2] phone intervals (array form; loop fallback)."""
    keep = np.fromiter((ph_seq[i] != "SP" for i in idx.tolist()), dtype=bool, count=len(idx))
    sel = np.flatnonzero(keep)
    if len(sel) == 0:
        return np.array([]), np.array([]), np.array([]), np.array([])
    kept = idx[sel].tolist()
    w = np.fromiter((ph_idx_to_word_idx[i] for i in kept), dtype=np.int64, count=len(kept))
    if (w < 0).any():
        return _assemble_loop(ph_intervals, idx, ph_seq, word_seq, ph_idx_to_word_idx)
    ph_iv = ph_intervals[sel]
    first = np.flatnonzero(np.concatenate([[True], w[1:] != w[:-1]]))
    last = np.concatenate([first[1:] - 1, [len(w) - 1]])
    word_iv = np.stack([ph_iv[first, 0], ph_iv[last, 1]], axis=1)
    return (np.array([ph_seq[i] for i in kept]), ph_iv.clip(min=0, max=None),
            np.array([word_seq[k] for k in w[first].tolist()]), word_iv.clip(min=0, max=None))


def batch_results(Ts, idx_h, tint_h, n_h, fc_h, ed_h, ph_seqs, word_seqs, p2ws, frame_length: float) -> list:
    """utterance_result for a whole batch of raw boundary arrays as they leave the GPU (idx / tint [B, >= n], n [B],
    frame_confidence / edge_diff [B, >= T] f32): the fractional boundaries of every utterance in one set of array
    operations (elementwise, so each value is the per-utterance form's, bit for bit), the phone / word selection and
    the confidence per utterance.  Returns the records utterance_result returns."""
    B = len(ph_seqs)
    T = np.asarray(list(Ts[:B]), dtype=np.int64)
    n = np.asarray(n_h[:B], dtype=np.int64)
    cols = np.arange(idx_h.shape[1])[None, :]
    valid = cols < n[:, None]
    tint = np.where(valid, tint_h[:B], 0).astype(np.int64)
    ed = np.take_along_axis(ed_h[:B], tint, axis=1).astype(np.float64)
    ed = np.where(tint == (T - 1)[:, None], 0.0, ed)          # edge_diff's last frame is 0 (alignment_decoder.py:83)
    body = frame_length * (tint.astype("float32") + (ed / 2).clip(-0.5, 0.5))
    ends = frame_length * T.astype(np.float64)
    out = []
    for b in range(B):
        k, Tb = int(n[b]), int(T[b])
        ph_seq = ph_seqs[b]
        ws = word_seqs[b] if word_seqs is not None and word_seqs[b] is not None else ph_seq
        pw = p2ws[b] if p2ws is not None and p2ws[b] is not None else np.arange(len(ph_seq))
        tp = np.concatenate([body[b, :k], ends[b:b + 1]])
        iv = np.stack([tp[:-1], tp[1:]], axis=1)
        idx = idx_h[b, :k].astype(np.int64)
        rec = dict(T=Ts[b], ph_idx_seq=idx, ph_time_int=tint_h[b, :k].astype(np.int64),
                   frame_confidence=fc_h[b, :Tb].copy(), edge_diff=ed_h[b, :Tb].copy())
        ph_p, ph_iv, w_p, w_iv = _phones_words(iv, idx, ph_seq, ws, pw)
        out.append(dict(rec, ph_seq=ph_p, ph_intervals=ph_iv, word_seq=w_p, word_intervals=w_iv,
                        confidence=total_confidence(rec["frame_confidence"])))
    return out


def total_confidence(frame_confidence: np.ndarray):
    return np.exp(np.mean(np.log(frame_confidence + 1e-6)) / 3)  # (:97)


def utterance_result(rec: dict, ph_seq, word_seq, ph_idx_to_word_idx, frame_length: float) -> dict:
    """One utterance's decode outputs from its raw boundary record — T, ph_idx_seq [n], ph_time_int [n],
    frame_confidence [T] and edge_diff [T] (f32 as computed on the GPU; the last frame's entry is replaced by
    0 as :83) — so every consumer of the raw arrays (the batched decoder, the multi-GPU gather on rank 0) builds
    bit-identical intervals."""
    T = rec["T"]
    ed = np.asarray(rec["edge_diff"])
    edge_diff = np.concatenate([ed[:T - 1].astype(np.float64), [0.0]]) if T > 0 else np.zeros(0)
    ph_p, ph_iv, w_p, w_iv = assemble_intervals(rec["ph_idx_seq"], rec["ph_time_int"], edge_diff, T, frame_length,
                                                ph_seq, word_seq, ph_idx_to_word_idx)
    return dict(rec, ph_seq=ph_p, ph_intervals=ph_iv, word_seq=w_p, word_intervals=w_iv,
                confidence=total_confidence(rec["frame_confidence"]))
