"""Host tail of the infer path (reference: tools/post_processing.py:1-105).

``fill_small_gaps``: a leading gap < MIN_SP_LENGTH snaps to 0; an inner gap < SP_MERGE_LENGTH is closed towards an
``AP`` neighbour (both AP: meet in the middle; neither AP: meet in the middle only if < MIN_SP_LENGTH); a trailing
gap < MIN_SP_LENGTH extends the last interval to the end.  ``add_SP`` then fills every remaining gap with ``SP``.
Intervals are mutated in place like the reference (numpy f64 [n, 2]).  Per-utterance errors are collected into
the error log instead of aborting the batch.
"""
from __future__ import annotations

MIN_SP_LENGTH = 0.1
SP_MERGE_LENGTH = 0.3


def add_SP(word_seq, word_intervals, wav_length, add_phone="SP"):
    if len(word_seq) == 0:
        return [add_phone], [[0, wav_length]]
    seq, ivs = [add_phone], [[0, word_intervals[0, 0]]]
    # rows as Python floats (the same f64 values): iterating numpy rows costs ~2 us per interval
    rows = word_intervals.tolist() if hasattr(word_intervals, "tolist") else word_intervals
    for word, (start, end) in zip(word_seq, rows):
        if ivs[-1][1] < start:
            seq.append(add_phone)
            ivs.append([ivs[-1][1], start])
        seq.append(word)
        ivs.append([start, end])
    if ivs[-1][1] < wav_length:
        seq.append(add_phone)
        ivs.append([ivs[-1][1], wav_length])
    if word_intervals[0, 0] <= 0:
        seq, ivs = seq[1:], ivs[1:]
    return seq, ivs


def fill_small_gaps(word_seq, word_intervals, wav_length):
    iv = word_intervals
    # the reference's loop on the rows as Python floats (the same f64 values and arithmetic: numpy element access
    # costs ~0.3 us per read), the changed values written back into the caller's array in place as the reference's
    # own element writes leave it
    f64 = hasattr(iv, "tolist")
    rows = iv.tolist() if f64 else iv
    if 0 < rows[0][0] < MIN_SP_LENGTH:
        rows[0][0] = 0
    for i in range(len(word_seq) - 1):
        left_end, right_start = rows[i][1], rows[i + 1][0]
        if not left_end < right_start:
            continue
        gap = right_start - left_end
        if gap >= SP_MERGE_LENGTH:
            continue
        left_ap, right_ap = word_seq[i] == "AP", word_seq[i + 1] == "AP"
        if left_ap and right_ap:
            mid = (left_end + right_start) / 2
            rows[i][1] = mid
            rows[i + 1][0] = mid
        elif left_ap:
            rows[i][1] = right_start
        elif right_ap:
            rows[i + 1][0] = left_end
        elif gap < MIN_SP_LENGTH:
            mid = (left_end + right_start) / 2
            rows[i][1] = mid
            rows[i + 1][0] = mid
    if rows[-1][1] < wav_length and wav_length - rows[-1][1] < MIN_SP_LENGTH:
        rows[-1][1] = wav_length
    if f64:
        iv[...] = rows
    return word_seq, iv


def post_process_one(prediction, add_phone="SP"):
    """One utterance -> (processed prediction, None), or (None, [wav_path, exception]) for the error log."""
    wav_path, wav_length, confidence, ph_seq, ph_intervals, word_seq, word_intervals = prediction
    try:
        word_seq, word_intervals = fill_small_gaps(word_seq, word_intervals, wav_length)
        ph_seq, ph_intervals = fill_small_gaps(ph_seq, ph_intervals, wav_length)
        word_seq, word_intervals = add_SP(word_seq, word_intervals, wav_length, add_phone)
        ph_seq, ph_intervals = add_SP(ph_seq, ph_intervals, wav_length, add_phone)
        return [wav_path, wav_length, confidence, ph_seq, ph_intervals, word_seq, word_intervals], None
    except Exception as e:  # noqa: BLE001 — collected, never aborts the batch
        return None, [wav_path, e]


def post_processing(predictions, add_phone="SP"):
    print("Post-processing...")
    res, error_log = [], []
    for pred in predictions:
        r, err = post_process_one(pred, add_phone)
        if err is None:
            res.append(r)
        else:
            error_log.append(err)
    return res, error_log
