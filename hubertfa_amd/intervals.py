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


def batch_tables(ph_seqs, word_seqs, p2ws) -> dict:
    """The transcript side of a batch's host assembly (batch_results): the batch's phone and word tables concatenated
    (names, lengths, SP mask, word map, offsets).  They depend on the transcripts only, so a pipelined caller builds
    them while the GPU runs the batch (task.submit) and the assembly after the results land is left with the path
    arrays alone.  ``src`` keeps the three sequences, so a table is used only for the very objects it was built from."""
    B = len(ph_seqs)
    wss = [word_seqs[b] if word_seqs is not None and word_seqs[b] is not None else ph_seqs[b] for b in range(B)]
    pw0 = [p2ws[b] if p2ws is not None and p2ws[b] is not None else np.arange(len(ph_seqs[b])) for b in range(B)]
    n_ph = np.fromiter(map(len, ph_seqs), dtype=np.int64, count=B)
    pws = [np.asarray(p, dtype=np.int64) for p in pw0]
    odd = np.fromiter((len(p) != k for p, k in zip(pws, n_ph.tolist())), dtype=bool, count=B)
    pws = [np.zeros(k, np.int64) if o else p for p, k, o in zip(pws, n_ph.tolist(), odd.tolist())]
    n_w = np.fromiter(map(len, wss), dtype=np.int64, count=B)
    ph_flat = [p for s in ph_seqs for p in s]
    w_flat = [x for s in wss for x in s]
    ph_names = np.array(ph_flat + [""])          # one spare entry: the target of out-of-range paths
    return dict(src=(ph_seqs, word_seqs, p2ws), wss=wss, pw0=pw0, odd=odd, n_ph=n_ph, n_w=n_w,
                ph_off=np.concatenate([[0], np.cumsum(n_ph)[:-1]]), w_off=np.concatenate([[0], np.cumsum(n_w)[:-1]]),
                ph_names=ph_names, w_names=np.array(w_flat + [""]),
                ph_len=np.fromiter(map(len, ph_flat), dtype=np.int64, count=len(ph_flat)),
                w_len=np.fromiter(map(len, w_flat), dtype=np.int64, count=len(w_flat)),
                is_sp=np.append(ph_names[:-1] == "SP", False), pw_flat=np.concatenate(pws + [np.zeros(1, np.int64)]),
                n_flat=len(ph_flat))


def batch_results(Ts, idx_h, tint_h, n_h, fc_h, ed_h, ph_seqs, word_seqs, p2ws, frame_length: float,
                  tables: dict | None = None) -> list:
    """utterance_result for a whole batch of raw boundary arrays as they leave the GPU (idx / tint [B, >= n], n [B],
    frame_confidence / edge_diff [B, >= T] f32).  The batch is assembled as one flat phone list: each path position
    indexes the batch's concatenated phone table (SP mask, word index offset per utterance, name lengths), the kept
    phones and the word openings are selected once for the batch, and each utterance's record is slices of the
    result (every value elementwise as the per-utterance form, bit for bit; string dtypes sized per utterance as
    np.array sizes them).  An utterance whose path leaves its own tables (a kept phone without a word, an index out of
    range) is assembled alone by _phones_words, whose loop form raises as the reference does."""
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
    # each phone interval is [its start, the next phone's start or the utterance's end] (:103-108)
    nxt = np.empty_like(body)
    nxt[:, :-1] = body[:, 1:]
    hasn = np.flatnonzero(n > 0)
    nxt[hasn, n[hasn] - 1] = ends[hasn]

    # the transcript side (batch_tables), built here unless the caller built it for these very sequences
    src = tables["src"] if tables is not None else None
    if src is None or src[0] is not ph_seqs or src[1] is not word_seqs or src[2] is not p2ws:
        tables = batch_tables(ph_seqs, word_seqs, p2ws)
    wss, pw0, odd, n_ph, n_w = tables["wss"], tables["pw0"], tables["odd"], tables["n_ph"], tables["n_w"]
    ph_off, w_off, ph_names, w_names = tables["ph_off"], tables["w_off"], tables["ph_names"], tables["w_names"]
    ph_len, w_len, is_sp, pw_flat = tables["ph_len"], tables["w_len"], tables["is_sp"], tables["pw_flat"]
    n_flat = tables["n_flat"]

    # the batch's paths as one flat list of (utterance, phone) in path order
    rows, pos = np.nonzero(valid)
    loc = idx_h[:B][rows, pos].astype(np.int64)
    bad_ix = (loc < 0) | (loc >= n_ph[rows])
    g = np.where(bad_ix, n_flat, loc + ph_off[rows])
    kept = ~is_sp[g]
    w_loc = pw_flat[g]
    bad = bad_ix | (kept & ((w_loc < 0) | (w_loc >= n_w[rows])))
    alone = odd.copy()                    # a word map not one entry per phone: that utterance alone
    alone[rows[bad]] = True

    sel = np.flatnonzero(kept & ~alone[rows])
    ks, kp, kg = rows[sel], pos[sel], g[sel]
    kw = w_loc[sel] + w_off[ks]
    ph_iv = np.stack([body[ks, kp], nxt[ks, kp]], axis=1).clip(min=0, max=None)
    opens = np.concatenate([[True], (kw[1:] != kw[:-1]) | (ks[1:] != ks[:-1])]) if len(sel) else np.zeros(0, bool)
    first = np.flatnonzero(opens)
    last = np.concatenate([first[1:] - 1, [len(sel) - 1]]) if len(first) else first
    word_iv = np.stack([ph_iv[first, 0], ph_iv[last, 1]], axis=1)
    fw = kw[first]
    ph_cnt = np.bincount(ks, minlength=B)
    w_cnt = np.bincount(ks[first], minlength=B)
    ph_end, w_end = np.cumsum(ph_cnt), np.cumsum(w_cnt)
    has_p, has_w = np.flatnonzero(ph_cnt), np.flatnonzero(w_cnt)
    ph_wid, w_wid = np.ones(B, np.int64), np.ones(B, np.int64)     # per utterance: np.array's '<U' width
    if len(has_p):
        ph_wid[has_p] = np.maximum(np.maximum.reduceat(ph_len[kg], (ph_end - ph_cnt)[has_p]), 1)
    if len(has_w):
        w_wid[has_w] = np.maximum(np.maximum.reduceat(w_len[fw], (w_end - w_cnt)[has_w]), 1)
    ph_sel, w_sel = ph_names[kg], w_names[fw]
    # total_confidence per row, for the rows of each length at once: the mean along each row of a [rows, T] block is
    # the 1-D mean of that row (numpy's pairwise sum over the contiguous axis), bit for bit
    log_fc = np.log(fc_h[:B] + 1e-6)
    conf = [None] * B
    for Tv in set(T.tolist()):
        rws = np.flatnonzero(T == Tv)
        cv = np.exp(np.mean(log_fc[rws, :Tv], axis=1) / 3)
        for j, r in enumerate(rws.tolist()):
            conf[r] = cv[j]
    idx64, tint64 = idx_h[:B].astype(np.int64), tint_h[:B].astype(np.int64)
    ph_end, w_end, ph_cnt, w_cnt = ph_end.tolist(), w_end.tolist(), ph_cnt.tolist(), w_cnt.tolist()
    ph_wid, w_wid, alone, n, T = ph_wid.tolist(), w_wid.tolist(), alone.tolist(), n.tolist(), T.tolist()

    out = []
    for b in range(B):
        k, Tb = n[b], T[b]
        idx = idx64[b, :k].copy()
        if alone[b]:
            tp = np.concatenate([body[b, :k], ends[b:b + 1]])
            res = _phones_words(np.stack([tp[:-1], tp[1:]], axis=1), idx, ph_seqs[b], wss[b], pw0[b])
        elif ph_cnt[b] == 0:
            res = np.array([]), np.array([]), np.array([]), np.array([])
        else:
            p0, p1, w0, w1 = ph_end[b] - ph_cnt[b], ph_end[b], w_end[b] - w_cnt[b], w_end[b]
            res = (ph_sel[p0:p1].astype(f"<U{ph_wid[b]}"), ph_iv[p0:p1], w_sel[w0:w1].astype(f"<U{w_wid[b]}"),
                   word_iv[w0:w1])
        out.append(dict(T=Ts[b], ph_idx_seq=idx, ph_time_int=tint64[b, :k].copy(),
                        frame_confidence=fc_h[b, :Tb].copy(), edge_diff=ed_h[b, :Tb].copy(), ph_seq=res[0],
                        ph_intervals=res[1], word_seq=res[2], word_intervals=res[3],
                        confidence=conf[b]))
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
