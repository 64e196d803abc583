"""Thin torch wrappers over the libhfa C-ABI: tensors -> raw device pointers + the current HIP stream.

PyTorch is plumbing here (device memory, streams); every op below launches a hand-written gfx950 kernel from
libhfa.so.  Inputs must already be on the GPU — there is no CPU path and no silent fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_P = ctypes.c_void_p


def _ptr(t: torch.Tensor | None):
    return _P(0) if t is None else _P(t.data_ptr())


def _stream(device=None):
    return _P(torch.cuda.current_stream(device).cuda_stream)


def _need(t: torch.Tensor, dtype, name: str, contiguous: bool = True):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise _lib.HFALibraryError(f"{name}: must be a GPU tensor (no CPU fallback), got {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t


# ------------------------------------------------------------------------------------------------------------
# Alignment decoder (viterbi.hip)
# ------------------------------------------------------------------------------------------------------------
def viterbi_forward(prob_log, not_edge_log, edge_log, curr, dp, bt, ph_seq_id, T, S, pad=None):
    """In-place batched forward_pass (alignment_decoder.py:170-230).

    prob_log/dp [B,Tmax,Smax] f32 (dp row 0 pre-initialised), bt [B,Tmax,Smax] int8, curr [B,Smax] f64,
    not_edge_log/edge_log [B,Tmax] f32, ph_seq_id [B,Smax] i32, T/S/pad [B] i32.
    """
    B, Tmax, Smax = prob_log.shape
    for t, dt, n in ((prob_log, torch.float32, "prob_log"), (not_edge_log, torch.float32, "not_edge_log"),
                     (edge_log, torch.float32, "edge_log"), (curr, torch.float64, "curr"),
                     (dp, torch.float32, "dp"), (bt, torch.int8, "bt"), (ph_seq_id, torch.int32, "ph_seq_id"),
                     (T, torch.int32, "T"), (S, torch.int32, "S")):
        _need(t, dt, n)
    if pad is not None:
        _need(pad, torch.int32, "pad")
    assert dp.shape == prob_log.shape and bt.shape == prob_log.shape
    assert curr.shape == (B, Smax) and ph_seq_id.shape == (B, Smax)
    assert not_edge_log.shape == (B, Tmax) and edge_log.shape == (B, Tmax)
    _lib.call("hfa_viterbi_forward", B, Tmax, Smax, _ptr(T), _ptr(S), _ptr(pad), _ptr(prob_log),
              _ptr(not_edge_log), _ptr(edge_log), _ptr(curr), _ptr(dp), _ptr(bt), _ptr(ph_seq_id),
              _stream(prob_log.device))


def viterbi_backtrack(dp, bt, ph_seq_id, T, S):
    """Batched end-state + backtrack + frame confidence (alignment_decoder.py:263-288).

    Returns (ph_idx_seq [B,Tmax] i32, ph_time_int [B,Tmax] i32, n [B] i32, frame_conf [B,Tmax] f32);
    row b is valid up to n[b] (ascending t) / T[b].
    """
    B, Tmax, Smax = dp.shape
    _need(dp, torch.float32, "dp")
    _need(bt, torch.int8, "bt")
    _need(ph_seq_id, torch.int32, "ph_seq_id")
    _need(T, torch.int32, "T")
    _need(S, torch.int32, "S")
    dev = dp.device
    idx = torch.empty((B, Tmax), dtype=torch.int32, device=dev)
    tint = torch.empty((B, Tmax), dtype=torch.int32, device=dev)
    n = torch.empty((B,), dtype=torch.int32, device=dev)
    fc = torch.empty((B, Tmax), dtype=torch.float32, device=dev)
    _lib.call("hfa_viterbi_backtrack", B, Tmax, Smax, _ptr(T), _ptr(S), _ptr(dp), _ptr(bt), _ptr(ph_seq_id),
              _ptr(idx), _ptr(tint), _ptr(n), _ptr(fc), _stream(dev))
    return idx, tint, n, fc


def lattice_prologue(frame_logits, edge_logits, ph_seq_id, T, S, want_frame_probs: bool = False):
    """Mask + log_softmax/softmax + edge sigmoid/diff/prob + gather to the [T,S] lattice (alignment_decoder.py
    :35-84, 239-242).  frame_logits [B,Tl,V] and edge_logits [B,Tl] may be strided views (last dim unit stride).
    """
    B, Tl, V = frame_logits.shape
    Smax = ph_seq_id.shape[1]
    _need(frame_logits, torch.float32, "frame_logits", contiguous=False)
    _need(edge_logits, torch.float32, "edge_logits", contiguous=False)
    if frame_logits.stride(2) != 1:
        raise ValueError("frame_logits: last dim must have unit stride")
    _need(ph_seq_id, torch.int32, "ph_seq_id")
    _need(T, torch.int32, "T")
    _need(S, torch.int32, "S")
    Tmax = Tl
    dev = frame_logits.device
    out = {
        "prob_log": torch.empty((B, Tmax, Smax), dtype=torch.float32, device=dev),
        "edge_log": torch.empty((B, Tmax), dtype=torch.float32, device=dev),
        "not_edge_log": torch.empty((B, Tmax), dtype=torch.float32, device=dev),
        "edge_diff": torch.empty((B, Tmax), dtype=torch.float32, device=dev),
        "edge_prob": torch.empty((B, Tmax), dtype=torch.float64, device=dev),
        "ph_prob_log": torch.empty((B, Tmax, V), dtype=torch.float32, device=dev) if want_frame_probs else None,
        "ph_frame_pred": torch.empty((B, Tmax, V), dtype=torch.float32, device=dev) if want_frame_probs else None,
    }
    _lib.call("hfa_lattice_prologue", B, Tmax, V, Smax, _ptr(T), _ptr(S), _ptr(frame_logits),
              frame_logits.stride(1), frame_logits.stride(0), _ptr(edge_logits), edge_logits.stride(1),
              edge_logits.stride(0), _ptr(ph_seq_id), _ptr(out["ph_prob_log"]), _ptr(out["ph_frame_pred"]),
              _ptr(out["prob_log"]), _ptr(out["edge_log"]), _ptr(out["not_edge_log"]), _ptr(out["edge_diff"]),
              _ptr(out["edge_prob"]), _stream(dev))
    return out
