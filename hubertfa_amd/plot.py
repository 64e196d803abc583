"""Validation figure of one alignment (reference: tools/plot.py plot_for_valid, called by AlignmentDecoder.plot at
tools/alignment_decoder.py:152-168).  Host-only matplotlib; imported on demand (the infer path never plots).

Top: the mel spectrogram with a red line at every phone boundary (a boundary shared by two phones drawn once, none
at the first frame or past the last), the non-SP phone names alternating above (black) and inside (white) the top
edge, and the frame confidence as a filled curve.  Bottom: the per-frame probabilities of the sequence's phones,
the aligned phone index per frame (red) and the edge probability (filled).  The same figure, element for element, as
the reference draws (tests/golden/plot.json)."""
from __future__ import annotations

import numpy as np


def plot_for_valid(melspec, ph_seq, ph_intervals, frame_confidence, ph_frame_prob, ph_frame_id_gt, edge_prob):
    import matplotlib.pyplot as plt
    names = [p.split("/")[-1] for p in ph_seq]
    n_mels, n_frames = melspec.shape[-2], melspec.shape[-1]
    frames = np.arange(n_frames)
    fig, (top, bottom) = plt.subplots(2)
    top.imshow(melspec[0], origin="lower", aspect="auto")
    for k, (start, end) in enumerate(ph_intervals):
        opens = k == 0 or ph_intervals[k - 1, 1] != start       # not already drawn as the previous phone's end
        if opens and start > 0:
            top.axvline(start, color="r", linewidth=1)
        if end < n_frames:
            top.axvline(end, color="r", linewidth=1)
        if names[k] == "SP":
            continue
        x = (start + end) / 2 - len(names[k]) * n_frames / 275
        y, colour = (n_mels + 1, "black") if k % 2 else (n_mels - 6, "white")
        top.text(x, y, names[k], fontsize=11, color=colour)
    conf = frame_confidence * n_mels
    top.plot(frames, conf, color="black", linewidth=1, alpha=0.6)
    top.fill_between(frames, conf, color="black", alpha=0.3)
    bottom.imshow(ph_frame_prob.T, origin="lower", aspect="auto", interpolation="nearest")
    bottom.plot(frames, ph_frame_id_gt, color="red", linewidth=1.5)
    edge = edge_prob * ph_frame_prob.shape[-1]
    bottom.plot(frames, edge, color="black", linewidth=1)
    bottom.fill_between(frames, edge, color="black", alpha=0.3)
    fig.set_size_inches(13, 7)
    fig.subplots_adjust(hspace=0)
    fig.subplots_adjust(left=0.05, right=0.95, top=0.95, bottom=0.05)
    return fig


def phone_index_per_frame(ph_idx_seq, ph_time_int, n_frames: int) -> np.ndarray:
    """The aligned phone index of every frame (alignment_decoder.py:153-160): the path's index steps added at the
    frames where they happen, then summed up."""
    steps = np.zeros(n_frames, dtype="int32")
    idx = np.asarray(ph_idx_seq)
    np.add.at(steps, np.asarray(ph_time_int), np.diff(np.concatenate([[0], idx])).astype("int32"))
    return np.cumsum(steps)
