"""Thin torch wrappers over the libhfa C-ABI: tensors -> raw device pointers + the current HIP stream.

PyTorch is plumbing here (device memory, streams); every op below launches a hand-written gfx950 kernel from
libhfa.so.  Inputs must already be on the GPU — there is no CPU path and no silent fallback.
"""
from __future__ import annotations

import contextlib
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
def viterbi_forward(prob_log, not_edge_log, edge_log, curr, dp, bt, ph_seq_id, T, S, pad=None, steps=None):
    """In-place batched forward_pass (alignment_decoder.py:170-230).

    prob_log/dp [B,Tmax,Smax] f32 (dp row 0 pre-initialised), bt [B,Tmax,Smax] int8, curr [B,Smax] f64,
    not_edge_log/edge_log [B,Tmax] f32, ph_seq_id [B,Smax] i32, T/S/pad [B] i32.  ``steps`` (t_begin, t_end):
    only those time steps, continuing from dp row t_begin - 1 and curr (consecutive ranges = one whole call).
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

    t0, t1 = (1, max(Tmax, 1)) if steps is None else (int(steps[0]), int(steps[1]))

    def launch():
        _lib.call("hfa_viterbi_forward_steps", B, Tmax, Smax, _ptr(T), _ptr(S), _ptr(pad), _ptr(prob_log),
                  _ptr(not_edge_log), _ptr(edge_log), _ptr(curr), _ptr(dp), _ptr(bt), _ptr(ph_seq_id), t0, t1,
                  _stream(prob_log.device))
    if PROBE is None:
        return launch()
    # SURVEY §8(d) algorithmic bytes: prob_log in + dp out (4 B each) + bt out (1 B) per cell, 8 B edge terms
    # per frame; counted on the padded planes (exact when every utterance of the batch fills them).  A step range
    # (a held DP, task.submit) counts its own time steps: ``units`` carries them, so the per-step figures hold.
    n = max(t1 - t0, 0) if steps is not None else Tmax
    PROBE("viterbi_forward_kernel", B * (9.0 * n * Smax + 8.0 * n), launch, kind="bytes", units=n)


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


def lattice_prologue(frame_logits, edge_logits, ph_seq_id, T, S, want_frame_probs: bool = False,
                     init_dp: bool = False):
    """Mask + log_softmax/softmax + edge sigmoid/diff/prob + gather to the [T,S] lattice (alignment_decoder.py
    :35-84, 239-242).  frame_logits [B,Tl,V] and edge_logits [B,Tl] may be strided views (last dim unit stride).
    ``init_dp``: also allocate the DP's dp / bt / curr and write _decode's initialisation (:244-254) in the same
    launch (out["dp"], out["bt"], out["curr"], ready for viterbi_forward)."""
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
        "dp": torch.empty((B, Tmax, Smax), dtype=torch.float32, device=dev) if init_dp else None,
        "bt": torch.empty((B, Tmax, Smax), dtype=torch.int8, device=dev) if init_dp else None,
        "curr": torch.empty((B, Smax), dtype=torch.float64, device=dev) if init_dp else None,
    }
    _lib.call("hfa_lattice_prologue", B, Tmax, V, Smax, _ptr(T), _ptr(S), _ptr(frame_logits),
              frame_logits.stride(1), frame_logits.stride(0), _ptr(edge_logits), edge_logits.stride(1),
              edge_logits.stride(0), _ptr(ph_seq_id), _ptr(out["ph_prob_log"]), _ptr(out["ph_frame_pred"]),
              _ptr(out["prob_log"]), _ptr(out["edge_log"]), _ptr(out["not_edge_log"]), _ptr(out["edge_diff"]),
              _ptr(out["edge_prob"]), _ptr(out["dp"]), _ptr(out["curr"]), _stream(dev))
    return out


def viterbi_init(prob_log, ph_seq_id, T, S):
    """_decode's dp / bt / curr initialisation (alignment_decoder.py:244-254) for a lattice that did not come
    through lattice_prologue: returns (dp, bt, curr) ready for viterbi_forward."""
    B, Tmax, Smax = prob_log.shape
    _need(prob_log, torch.float32, "prob_log")
    _need(ph_seq_id, torch.int32, "ph_seq_id")
    _need(T, torch.int32, "T")
    _need(S, torch.int32, "S")
    dev = prob_log.device
    dp = torch.empty((B, Tmax, Smax), dtype=torch.float32, device=dev)
    bt = torch.empty((B, Tmax, Smax), dtype=torch.int8, device=dev)
    curr = torch.empty((B, Smax), dtype=torch.float64, device=dev)
    _lib.call("hfa_viterbi_init", B, Tmax, Smax, _ptr(T), _ptr(S), _ptr(prob_log), _ptr(ph_seq_id), _ptr(dp),
              _ptr(curr), _stream(dev))
    return dp, bt, curr


# ------------------------------------------------------------------------------------------------------------
# Encoder kernels (gemm.hip, attention.hip, norm.hip, conv.hip, misc.hip)
# ------------------------------------------------------------------------------------------------------------
EPI_NONE, EPI_GELU = 0, 1
GEMM_F16 = 0x100          # hfa.h HFA_GEMM_F16: opt-in one-product f16 arithmetic on the split GEMM
ACT_NONE, ACT_GELU, ACT_HARDSWISH = 0, 1, 2

_P_, _I_, _LL_, _F_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
_lib.register("hfa_conv_gemm_f32", [_I_, _I_, _I_, _I_, _I_, _P_, _LL_, _LL_, _I_, _I_, _I_, _I_, _I_, _P_, _LL_, _I_,
                                    _P_, _LL_, _P_, _LL_, _LL_, _I_, _P_, _LL_, _LL_, _I_, _I_, _P_])
_lib.register("hfa_gemm_tuning", [_I_, _I_])
_lib.register("hfa_gemm_kernel_name", [_I_, _I_, _I_, _I_, _I_, _P_, _LL_, _LL_, _I_, _I_, _I_, _I_, _I_, _P_, _LL_,
                                       _I_, _P_, _LL_, _P_, _LL_, _LL_, _I_, _P_, _LL_, _LL_, _I_, _I_], ctypes.c_char_p)
_lib.register("hfa_conv_gemm_split", [_I_, _I_, _I_, _I_, _I_, _P_, _LL_, _LL_, _LL_, _I_, _I_, _I_, _I_, _I_, _P_,
                                       _LL_, _LL_, _I_, _P_, _LL_, _P_, _LL_, _LL_, _I_, _P_, _LL_, _P_, _P_, _LL_,
                                       _LL_, _LL_, _I_, _I_, _P_, _P_])
_lib.register("hfa_gemm_split_kernel_name", [_I_, _I_, _I_, _I_, _I_, _I_, _I_], ctypes.c_char_p)
_lib.register("hfa_gemm_split_tuning", [_I_])
_lib.register("hfa_split_f16", [_I_, _I_, _P_, _LL_, _P_, _LL_, _LL_, _P_, _P_])
_lib.register("hfa_gemm_f32", [_I_, _I_, _I_, _P_, _I_, _P_, _I_, _P_, _P_, _I_, _P_, _I_, _I_, _P_])
_lib.register("hfa_attention_f32", [_I_, _I_, _I_, _I_, _F_, _P_, _LL_, _I_, _P_, _LL_, _I_, _P_, _LL_, _I_, _P_,
                                    _LL_, _I_, _P_, _P_])
_lib.register("hfa_attention_split", [_I_, _I_, _I_, _I_, _F_, _P_, _LL_, _LL_, _I_, _P_, _LL_, _LL_, _I_, _P_, _LL_,
                                      _LL_, _I_, _P_, _LL_, _LL_, _I_, _P_, _P_])
_lib.register("hfa_attention_split_tuning", [_I_])
_lib.register("hfa_attention_split_form", [_I_])
_lib.register("hfa_attention_split_kernel_name", [_I_, _I_, _I_], ctypes.c_char_p)
_lib.register("hfa_layernorm_split", [_I_, _I_, _P_, _LL_, _P_, _LL_, _P_, _P_, _F_, _I_, _P_, _LL_, _I_, _P_, _P_, _LL_,
                                      _LL_, _P_, _P_])
_lib.register("hfa_layernorm_f32",[_I_, _I_, _P_, _LL_, _P_, _LL_, _P_, _P_, _F_, _I_, _P_, _LL_, _I_, _P_, _P_])
_lib.register("hfa_groupnorm_f32", [_I_, _I_, _I_, _I_, _P_, _LL_, _I_, _P_, _P_, _F_, _I_, _P_, _LL_, _I_, _P_,
                                    _P_, _P_])
_lib.register("hfa_groupnorm_workspace_bytes", [_I_, _I_, _I_, _I_], ctypes.c_longlong)
_lib.register("hfa_groupnorm_split", [_I_, _I_, _I_, _I_, _P_, _LL_, _I_, _P_, _P_, _F_, _I_, _P_, _LL_, _I_, _P_, _P_,
                                      _LL_, _I_, _LL_, _P_, _P_, _P_])
_lib.register("hfa_conv0_workspace_bytes", [_I_, _I_], ctypes.c_longlong)
_lib.register("hfa_conv0_f32", [_I_, _I_, _P_, _LL_, _P_, _P_, _I_, _P_, _P_, _F_, _P_, _P_, _LL_, _P_, _P_])
_lib.register("hfa_conv0_split", [_I_, _I_, _P_, _LL_, _P_, _P_, _I_, _P_, _P_, _F_, _P_, _P_, _LL_, _LL_, _P_, _P_,
                                   _P_])
_lib.register("hfa_units_gather_f32", [_I_, _I_, _I_, _P_, _LL_, _I_, _I_, _I_, _F_, _P_, _LL_, _I_, _P_, _P_, _P_])
_lib.register("hfa_mask_rows_f32", [_I_, _I_, _I_, _P_, _LL_, _I_, _P_, _P_])
_lib.register("hfa_wav_normalize_f32", [_I_, _I_, _P_, _LL_, _F_, _P_, _LL_, _P_, _P_, _P_])
_lib.register("hfa_wav_normalize_workspace_bytes", [_I_], ctypes.c_longlong)
_lib.register("hfa_pad_rows_f32", [_I_, _I_, _P_, _LL_, _I_, _I_, _P_, _LL_, _P_])
_lib.register("hfa_add_f32", [_LL_, _P_, _P_, _P_, _P_])
_lib.register("hfa_selftest_erf", [_LL_, _P_, _P_, _P_, _P_])
_lib.register("hfa_selftest_gelu", [_LL_, _P_, _P_, _P_])
_lib.register("hfa_resample_workspace_bytes", [_I_, _I_, _I_, _I_], ctypes.c_longlong)
_lib.register("hfa_resample_f32", [_I_, _I_, _P_, _LL_, _I_, _I_, _P_, _I_, _I_, _P_, _P_, _LL_, _P_])


class KernelProbe:
    """Times every launch of the watched kernels with HIP events on the launching stream (bench.py).

    ``name`` is the rocprof kernel symbol stem of the dominant kernel, e.g. ``gemm_f32_kernel<1, true, ...>``;
    ``extra`` names further kernels to time (the DP, conv0, attention).  Per launch the algorithmic work (FLOPs
    for MFMA kernels, bytes for HBM/latency-bound ones) is recorded next to the event pair, so
    achieved = sum(work) / sum(durations).  Census mode (name None) times nothing and tallies FLOPs per
    MFMA instantiation so bench.py can pick the dominant one."""

    def __init__(self, name: str | None, extra=()):
        self.name = name
        self.watch = set(extra) | ({name} if name else set())
        self.records = {}
        self.census = {}
        self.active = True           # False: launches pass through untimed (bench.py samples the timed steps)

    def dominant(self) -> str:
        return max(self.census, key=self.census.get)

    def __call__(self, name: str, work: float, launch, kind: str = "flops", shape=None, units=None, label=None):
        if self.name is None:
            if kind == "flops":
                self.census[name] = self.census.get(name, 0.0) + work
            return launch()
        if name not in self.watch or not self.active:
            return launch()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.records.setdefault(name, []).append((s, e, work, units))

    def summary(self, name: str | None = None):
        """launches, total / average ms, work; ``units`` = the launches' own units (the DP's time steps) when
        every launch reported them, else None."""
        torch.cuda.synchronize()
        recs = self.records.get(name or self.name, [])
        n = len(recs)
        ms = sum(s.elapsed_time(e) for s, e, _, _ in recs)
        w = sum(f for _, _, f, _ in recs)
        u = sum(x for *_, x in recs) if recs and all(x is not None for *_, x in recs) else None
        return {"launches": n, "total_ms": ms, "avg_ms": ms / max(n, 1), "work": w, "avg_work": w / max(n, 1),
                "flops": w, "avg_flops": w / max(n, 1), "units": u}


PROBE = None


def _gemm_name(*args) -> str:
    """rocprof symbol stem of the instantiation hfa_conv_gemm_f32 dispatches to for these arguments (the
    library answers from the same plan it launches)."""
    return _lib.lib().hfa_gemm_kernel_name(*args).decode()


def conv_gemm(A, W, C, *, M, N, K, Zb=1, G=1, sAb=0, sAg=0, ldx, stride=1, pad=0, Cg=None, Tin=None, sWg=0,
              ldw=None, bias=None, sBg=0, R=None, sRb=0, sRg=0, ldr=0, sCb=0, sCg=0, ldc, epilogue=EPI_NONE):
    """Implicit-GEMM conv / Linear on MFMA (see gemm.hip for the exact A/W/C addressing)."""
    for t, n in ((A, "A"), (W, "W"), (C, "C")):
        _need(t, torch.float32, n, contiguous=False)

    args = (M, N, K, Zb, G, _ptr(A), sAb, sAg, ldx, stride, pad, Cg or K, Tin if Tin is not None else M, _ptr(W),
            sWg, ldw if ldw is not None else K, _ptr(bias), sBg, _ptr(R), sRb, sRg, ldr, _ptr(C), sCb, sCg, ldc,
            epilogue)

    def launch():
        _lib.call("hfa_conv_gemm_f32", *args, _stream(C.device))
    if PROBE is None:
        return launch()
    PROBE(_gemm_name(*args), 2.0 * M * N * K * Zb * G, launch)


def linear(x, W, bias=None, residual=None, out=None, epilogue=EPI_NONE):
    """y = epi(x @ W^T + bias) (+ residual); x [..., K] rows contiguous, W [N, K] contiguous."""
    K = x.shape[-1]
    N = W.shape[0]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if out is None:
        out = torch.empty((*x.shape[:-1], N), dtype=torch.float32, device=x.device)
    o2 = out.view(-1, N)
    r2 = residual.reshape(-1, N) if residual is not None else None
    _need(W, torch.float32, "W")

    args = (M, N, K, _ptr(x2), x2.stride(0), _ptr(W), W.stride(0), _ptr(bias), _ptr(r2),
            r2.stride(0) if r2 is not None else 0, _ptr(o2), o2.stride(0), epilogue)

    def launch():
        _lib.call("hfa_gemm_f32", *args, _stream(x.device))
    if PROBE is None:
        launch()
    else:                       # hfa_gemm_f32 is hfa_conv_gemm_f32 with Zb = G = 1, stride 1, Cg = K, Tin = M
        PROBE(_gemm_name(M, N, K, 1, 1, _ptr(x2), 0, 0, x2.stride(0), 1, 0, K, M, _ptr(W), 0, W.stride(0), _ptr(bias),
                         0, _ptr(r2), 0, 0, r2.stride(0) if r2 is not None else 0, _ptr(o2), 0, 0, o2.stride(0),
                         epilogue), 2.0 * M * N * K, launch)
    return out


# ---- split-f16 operands (gemm.hip gemm_split_kernel) ----------------------------------------------------------
# A split tensor is a float16 tensor [2, *shape]: plane 0 = f16(x), plane 1 = f16((x - plane0) * 2^11).
_OFLOW = {}


def split_flag(device) -> torch.Tensor:
    """Device int32 flag the split producers raise when a value leaves f16 range (|x| >= 65504 / non-finite);
    the caller re-runs that batch on the f32 path (see task.ForcedAlignmentTask)."""
    key = torch.device(device)
    if key.type == "cuda" and key.index is None:
        key = torch.device("cuda", torch.cuda.current_device())
    if key not in _OFLOW:
        _OFLOW[key] = torch.zeros(1, dtype=torch.int32, device=key)
    return _OFLOW[key]


def split(x, out=None, flag=None):
    """f32 [..., C] (row-strided) -> split planes [2, ..., C]; out-of-range values raise ``flag`` (default: the
    device's split_flag)."""
    _need(x, torch.float32, "x", contiguous=False)
    C = x.shape[-1]
    x2 = x.reshape(-1, C) if x.dim() != 2 else x
    if x2.stride(-1) != 1:
        raise ValueError("split: last dim must be contiguous")
    rows = x2.shape[0]
    if out is None:
        out = torch.empty((2, *x.shape), dtype=torch.float16, device=x.device)
    o2 = out.view(2, rows, C)
    _lib.call("hfa_split_f16", rows, C, _ptr(x2), x2.stride(0), _ptr(o2), o2.stride(1), o2.stride(0),
              _ptr(split_flag(x.device) if flag is None else flag), _stream(x.device))
    return out


def _split_name(M, N, K, Z, out_split, epilogue, Cg) -> str:
    return _lib.lib().hfa_gemm_split_kernel_name(M, N, K, Z, int(out_split), epilogue, Cg).decode()


def conv_gemm_split(As, Ws, C=None, Cs=None, *, M, N, K, Zb=1, G=1, sAb=0, sAg=0, ldx, stride=1, pad=0, Cg=None,
                    Tin=None, sWg=0, ldw=None, bias=None, sBg=0, R=None, sRb=0, sRg=0, ldr=0, sCb=0, sCg=0, ldc,
                    epilogue=EPI_NONE, flag=None, f16=False):
    """conv_gemm on split operands (As, Ws: [2, ...] f16 planes; strides in elements of one plane).  Output to f32
    C (+R), to split planes Cs [2, ...] (bias/GELU epilogue only), or both (dual: the planes of the final C).
    R may be f32 or split planes [2, ...] f16 (f32 C alone; its strides in halves of one plane).
    ``f16``: the opt-in fast mode (high planes only, one f16 product per MAC: f16-class accuracy)."""
    Rs = None
    if R is not None and R.dtype == torch.float16:
        R, Rs = None, R
    if f16:
        epilogue |= GEMM_F16
    _need(As, torch.float16, "As", contiguous=False)
    _need(Ws, torch.float16, "Ws", contiguous=False)
    if C is None and Cs is None:
        raise ValueError("conv_gemm_split: C and / or Cs")
    dev = (C if C is not None else Cs).device
    args = (M, N, K, Zb, G, _ptr(As), As.stride(0), sAb, sAg, ldx, stride, pad, Cg or K, Tin if Tin is not None else M,
            _ptr(Ws), Ws.stride(0), sWg, ldw if ldw is not None else K, _ptr(bias), sBg, _ptr(R), sRb, sRg, ldr,
            _ptr(Rs), Rs.stride(0) if Rs is not None else 0,
            _ptr(C), _ptr(Cs), Cs.stride(0) if Cs is not None else 0, sCb, sCg, ldc, epilogue,
            _ptr(split_flag(dev) if flag is None else flag))

    def launch():
        _lib.call("hfa_conv_gemm_split", *args, _stream(dev))
    if PROBE is None:
        return launch()
    PROBE(_split_name(M, N, K, Zb * G, Cs is not None and C is None, epilogue, Cg or K), 2.0 * M * N * K * Zb * G, launch,
          shape=(M, N, K, Zb * G))


def linear_split(xs, Ws, bias=None, residual=None, out=None, epilogue=EPI_NONE, out_split=False, flag=None,
                 f16=False):
    """y = epi(x @ W^T + bias) (+ residual) with x, W given as split planes [2, ..., K] / [2, N, K]; y f32, or split
    planes [2, ..., N] when out_split (no residual), or both as (y, planes) when out_split == "dual"."""
    K = xs.shape[-1]
    N = Ws.shape[1]
    lead = xs.shape[1:-1]
    M = 1
    for d in lead:
        M *= d
    dual = out_split == "dual"
    planes = out_split and not dual
    if out is None:
        out = torch.empty(((2,) if planes else ()) + (*lead, N), dtype=torch.float16 if planes else torch.float32,
                          device=xs.device)
    hs = torch.empty((2, *lead, N), dtype=torch.float16, device=xs.device) if dual else None
    if residual is None:
        r2 = None
    elif residual.dtype == torch.float16:                  # split planes [2, ..., N] (a LayerNorm's plane output)
        r2 = residual.reshape(2, -1, N)
    else:
        r2 = residual.reshape(-1, N)
    conv_gemm_split(xs, Ws, C=None if planes else out, Cs=out if planes else hs, M=M, N=N, K=K,
                    ldx=xs.stride(-2) if xs.dim() > 2 else K, bias=bias, R=r2, ldr=r2.stride(-2) if r2 is not None else 0,
                    ldc=N, epilogue=epilogue, flag=flag, f16=f16)
    return (out, hs) if dual else out


def _lens(lens):
    """Optional per-row lengths of a variable-length batch: None or an int32 device tensor [B]."""
    if lens is None:
        return None
    _need(lens, torch.int32, "lengths")
    return lens


def attention(q, k, v, out, *, B, H, L, head_dim, scale, q_bs, q_ld, k_bs, k_ld, v_bs, v_ld, o_bs, o_ld,
              key_len=None):
    """Flash attention; ``key_len`` [B] int32 (optional): per-row lengths (keys and queries beyond are padding)."""
    kl = _lens(key_len)

    def launch():
        _lib.call("hfa_attention_f32", B, H, L, head_dim, float(scale), _ptr(q), q_bs, q_ld, _ptr(k), k_bs, k_ld,
                  _ptr(v), v_bs, v_ld, _ptr(out), o_bs, o_ld, _ptr(kl), _stream(out.device))
    if PROBE is None:
        launch()
    else:                       # QK^T and PV: 2 * 2 * L * L * head_dim per (batch, head)
        PROBE("attn_fwd_f32_kernel", 4.0 * B * H * L * L * head_dim, launch, kind="flops_aux")
    return out


def attention_split(qkv_s, out_s, *, B, H, L, head_dim, scale, key_len=None):
    """Flash attention on split planes (attention.hip attn_fwd_split16_kernel / attn_fwd_split_kernel): ``qkv_s``
    [2, B, L, 3*H*head_dim] f16 planes of the fused QKV projection (Q | K | V column blocks), ``out_s``
    [2, B, L, H*head_dim] planes."""
    _need(qkv_s, torch.float16, "qkv_s")
    _need(out_s, torch.float16, "out_s")
    D = H * head_dim
    if qkv_s.shape != (2, B, L, 3 * D) or out_s.shape != (2, B, L, D):
        raise ValueError(f"attention_split: qkv_s {tuple(qkv_s.shape)} / out_s {tuple(out_s.shape)} do not match "
                         f"B={B} L={L} H={H} head_dim={head_dim}")
    kl = _lens(key_len)
    sp, bs, ld = qkv_s.stride(0), qkv_s.stride(1), qkv_s.stride(2)
    base = qkv_s.data_ptr()

    def launch():
        _lib.call("hfa_attention_split", B, H, L, head_dim, float(scale), _P(base), sp, bs, ld, _P(base + 2 * D),
                  sp, bs, ld, _P(base + 4 * D), sp, bs, ld, _ptr(out_s), out_s.stride(0), out_s.stride(1),
                  out_s.stride(2), _ptr(kl), _stream(out_s.device))
    if PROBE is None:
        launch()
    else:
        PROBE(attention_split_probe_name(), 4.0 * B * H * L * L * head_dim, launch, kind="flops_aux",
              shape=(B, H, L, head_dim))
    return out_s


def attention_split_probe_name() -> str:
    """rocprof symbol stem of the split attention the library launches under the current MFMA form
    (hfa_attention_split_form): "attn_fwd_split16_kernel" (16x16x32, the default) or "attn_fwd_split_kernel"."""
    return _lib.lib().hfa_attention_split_kernel_name(1, 1, 1).decode().split("<")[0]


def layernorm(x, gamma, beta, eps=1e-5, act=ACT_NONE, out=None, residual=None, t_len=None, out_split=None,
              flag=None):
    """Row LayerNorm (+act) over the last dim; with ``t_len`` [B] (x is [B, T, C]) rows t >= t_len[b] -> 0.
    ``out_split`` ([2, ..., C] f16, or True to allocate): the output also as split planes (returned second)."""
    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    if out is False:                                      # split planes only (out_split required)
        if out_split is None or out_split is False:
            raise ValueError("layernorm: out=False needs out_split")
        o2 = None
    else:
        if out is None:
            out = torch.empty_like(x)
        o2 = out.view(-1, C)
    r2 = residual.reshape(-1, C) if residual is not None else None
    tl = _lens(t_len)
    T = x.shape[-2] if (tl is not None and x.dim() == 3) else 0
    if out_split is None or out_split is False:
        _lib.call("hfa_layernorm_f32", x2.shape[0], C, _ptr(x2), x2.stride(0), _ptr(r2),
                  r2.stride(0) if r2 is not None else 0, _ptr(gamma), _ptr(beta), float(eps), act, _ptr(o2),
                  o2.stride(0), T, _ptr(tl), _stream(x.device))
        return out
    if out_split is True:
        out_split = torch.empty((2, *x.shape), dtype=torch.float16, device=x.device)
    _need(out_split, torch.float16, "out_split")
    s2 = out_split.view(2, -1, C)
    _lib.call("hfa_layernorm_split", x2.shape[0], C, _ptr(x2), x2.stride(0), _ptr(r2),
              r2.stride(0) if r2 is not None else 0, _ptr(gamma), _ptr(beta), float(eps), act, _ptr(o2),
              o2.stride(0) if o2 is not None else 0, T, _ptr(tl), _ptr(s2), s2.stride(1), s2.stride(0),
              _ptr(split_flag(x.device) if flag is None else flag), _stream(x.device))
    return (None if o2 is None else out), out_split


def groupnorm(x, G, gamma, beta, eps=1e-5, act=ACT_NONE, out=None, t_len=None, out_split=None, flag=None):
    """GroupNorm over channels-last x [B, T, C] (stats over T x C/G per group; over t_len[b] rows if given,
    padding rows -> 0).  ``out_split`` ([2, B, T, C] f16, or True to allocate): write split planes; with
    ``out=False`` the planes only (no f32 output).  Returns the f32 output, the planes, or (f32, planes)."""
    B, T, C = x.shape
    tl = _lens(t_len)
    ws = torch.empty(max(1, int(_lib.lib().hfa_groupnorm_workspace_bytes(B, T, C, G))), dtype=torch.uint8,
                     device=x.device)
    if out_split is None or out_split is False:
        if out is None:
            out = torch.empty_like(x)
        _lib.call("hfa_groupnorm_f32", B, T, C, G, _ptr(x), x.stride(0), x.stride(1), _ptr(gamma), _ptr(beta),
                  float(eps), act, _ptr(out), out.stride(0), out.stride(1), _ptr(tl), _ptr(ws), _stream(x.device))
        return out
    if out_split is True:
        out_split = torch.empty((2, B, T, C), dtype=torch.float16, device=x.device)
    _need(out_split, torch.float16, "out_split", contiguous=False)
    if out is None:
        out = torch.empty_like(x)
    y = None if out is False else out
    _lib.call("hfa_groupnorm_split", B, T, C, G, _ptr(x), x.stride(0), x.stride(1), _ptr(gamma), _ptr(beta),
              float(eps), act, _ptr(y), y.stride(0) if y is not None else 0, y.stride(1) if y is not None else 0,
              _ptr(tl), _ptr(out_split), out_split.stride(1), out_split.stride(2), out_split.stride(0),
              _ptr(split_flag(x.device) if flag is None else flag), _ptr(ws), _stream(x.device))
    return out_split if y is None else (y, out_split)


def conv0(x, w0, *, bias=None, gamma=None, beta=None, eps=1e-5, out=None, workspace=None, t0_len=None,
          out_split=False):
    """First extractor conv (1->512, k10, s5) -> [B, T0, 512]; GroupNorm+GELU when gamma/beta are given
    (statistics over t0_len[b] frames if given).  out_split: the output as split-f16 planes [2, B, T0, 512]."""
    B, N = x.shape
    T0 = (N - 10) // 5 + 1
    if out is None:
        out = torch.empty(((2,) if out_split else ()) + (B, T0, 512),
                          dtype=torch.float16 if out_split else torch.float32, device=x.device)
    norm = gamma is not None
    if norm and workspace is None:
        nbytes = _lib.lib().hfa_conv0_workspace_bytes(B, N)
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    tl = _lens(t0_len)

    def launch():
        if out_split:
            _lib.call("hfa_conv0_split", B, N, _ptr(x), x.stride(0), _ptr(w0), _ptr(bias), 1 if norm else 0,
                      _ptr(gamma), _ptr(beta), float(eps), _ptr(workspace), _ptr(out), out.stride(1), out.stride(0),
                      _ptr(split_flag(x.device)), _ptr(tl), _stream(x.device))
        else:
            _lib.call("hfa_conv0_f32", B, N, _ptr(x), x.stride(0), _ptr(w0), _ptr(bias), 1 if norm else 0,
                      _ptr(gamma), _ptr(beta), float(eps), _ptr(workspace), _ptr(out), out.stride(0), _ptr(tl),
                      _stream(x.device))
    if PROBE is None:
        launch()
    else:                       # wave in (4 B/sample) + activations out (4 B x 512 x T0)
        PROBE("hfa_conv0_split" if out_split else "hfa_conv0_f32", B * (4.0 * N + 4.0 * 512 * T0), launch,
              kind="bytes")
    return out


def units_gather(units, n_frames, T_pad, ratio, out=None, n_frames_b=None, U_b=None):
    B, U, C = units.shape
    if out is None:
        out = torch.empty((B, T_pad, C), dtype=torch.float32, device=units.device)
    nf, ub = _lens(n_frames_b), _lens(U_b)
    _lib.call("hfa_units_gather_f32", B, U, C, _ptr(units), units.stride(0), units.stride(1), n_frames, T_pad,
              float(ratio), _ptr(out), out.stride(0), out.stride(1), _ptr(nf), _ptr(ub), _stream(units.device))
    return out


def mask_rows(x, lens):
    """Zero rows t >= lens[b] of x [B, T, C] (or [B, N] as C = 1), in place."""
    ln = _lens(lens)
    if x.dim() == 2:
        B, T = x.shape
        C, ld = 1, 1
    else:
        B, T, C = x.shape
        ld = x.stride(1)
    _lib.call("hfa_mask_rows_f32", B, T, C, _ptr(x), x.stride(0), ld, _ptr(ln), _stream(x.device))
    return x


def wav_normalize(x, eps=1e-7, out=None, lens=None):
    B, N = x.shape
    if out is None:
        out = torch.empty_like(x)
    ln = _lens(lens)
    ws = torch.empty(max(1, int(_lib.lib().hfa_wav_normalize_workspace_bytes(B))), dtype=torch.uint8,
                     device=x.device)
    _lib.call("hfa_wav_normalize_f32", B, N, _ptr(x), x.stride(0), float(eps), _ptr(out), out.stride(0), _ptr(ln),
              _ptr(ws), _stream(x.device))
    return out


def pad_rows(x, left, n_out, out=None):
    B, N = x.shape
    if out is None:
        out = torch.empty((B, n_out), dtype=torch.float32, device=x.device)
    _lib.call("hfa_pad_rows_f32", B, N, _ptr(x), x.stride(0), left, n_out, _ptr(out), out.stride(0),
              _stream(x.device))
    return out


_lib.register("hfa_flag_take", [_I_, _P_, _P_, _P_])


def flag_take(flag: torch.Tensor) -> torch.Tensor:
    """Snapshot of a device int32 flag tensor, which is cleared (stream-ordered, one launch)."""
    _need(flag, torch.int32, "flag")
    snap = torch.empty_like(flag)
    _lib.call("hfa_flag_take", flag.numel(), _ptr(flag), _ptr(snap), _stream(flag.device))
    return snap


_lib.register("hfa_set_grid_cap", [_I_])


@contextlib.contextmanager
def grid_cap(wgs: int):
    """Launches of the row-streaming kernels (split_f16, LayerNorm, lattice prologue) made by this thread inside the
    block use at most ``wgs`` workgroups (hfa_set_grid_cap; results identical)."""
    _lib.call("hfa_set_grid_cap", int(wgs))
    try:
        yield
    finally:
        _lib.call("hfa_set_grid_cap", 0)


def add(a, b, out=None):
    if out is None:
        out = torch.empty_like(a)
    _lib.call("hfa_add_f32", a.numel(), _ptr(a), _ptr(b), _ptr(out), _stream(a.device))
    return out


_lib.register("hfa_resample_split_workspace_bytes", [_I_, _I_, _I_, _I_, _I_], ctypes.c_longlong)
_lib.register("hfa_resample_split", [_I_, _I_, _P_, _LL_, _I_, _I_, _P_, _I_, _I_, _I_, _P_, _P_, _LL_, _P_, _P_])


def resample_split(x, orig, new, w_planes, G, width, out=None, workspace=None, flag=None, n_out=None):
    """Sinc resample rows of x [B, N] (row stride free, unit element stride) on the split-f16 GEMM; w_planes
    [2, G, new, Kg] (resample.Resampler builds them).  Returns the [B, ceil(new*N/orig)] view of the output (``n_out``
    columns instead: resample.ChainResampler, whose composite filter's length is the two stages')."""
    _need(x, torch.float32, "x", contiguous=False)
    if x.stride(-1) != 1:
        raise ValueError("resample_split: rows must have unit stride")
    B, N = x.shape
    Kg = w_planes.shape[-1]
    F = N // orig + 1
    cols = F * new if G == 1 else -(-F // 8) * 8 * new
    if out is None:
        out = torch.empty((B, cols), dtype=torch.float32, device=x.device)
    if workspace is None:
        nbytes = _lib.lib().hfa_resample_split_workspace_bytes(B, N, orig, Kg, G)
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    def launch():
        _lib.call("hfa_resample_split", B, N, _ptr(x), x.stride(0), orig, new, _ptr(w_planes), Kg, G, width,
                  _ptr(workspace), _ptr(out), out.stride(0), _ptr(split_flag(x.device) if flag is None else flag),
                  _stream(x.device))
    if PROBE is None:
        launch()
    else:      # (its GEMM shares an instantiation with the encoder's: reported outside the dominant-kernel census)
        rows = F if G == 1 else -(-F // 8)
        PROBE(_split_name(rows, new, Kg, B * G, False, 0, Kg), 2.0 * rows * new * Kg * B * G, launch,
              kind="flops_aux", shape=(rows, new, Kg, B * G),
              label="resampler chain (one pass)" if orig == new else f"resampler {orig} -> {new} (reduced rates)")
    from .resample import target_length
    return out[:, : target_length(N, orig, new) if n_out is None else n_out]


_lib.register("hfa_resample_chain_edges_workspace_bytes", [_I_, _I_, _I_, _I_], restype=_LL_)
_lib.register("hfa_resample_chain_edges", [_I_, _I_, _P_, _P_, _LL_, _I_, _I_, _P_, _I_, _I_, _P_, _I_, _I_, _P_, _P_,
                                            _LL_, _I_, _P_])


def resample_chain_edges(x, lens, P, Q, wu_t, wu_width, wd_t, wd_width, y):
    """Overwrite the edge frames of a composite two-stage resample y [B, >= cols] (hfa_resample_chain_edges): x
    [B, N] the input rows, ``lens`` an int32 device tensor of per-row input lengths or None (all N)."""
    _need(x, torch.float32, "x", contiguous=False)
    _need(y, torch.float32, "y", contiguous=False)
    if x.stride(-1) != 1 or y.stride(-1) != 1:
        raise ValueError("resample_chain_edges: rows must have unit stride")
    B, N = x.shape
    nbytes = _lib.lib().hfa_resample_chain_edges_workspace_bytes(B, Q, wd_t.shape[0], wd_width)
    ws = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=x.device)
    _lib.call("hfa_resample_chain_edges", B, N, _ptr(lens) if lens is not None else None, _ptr(x), x.stride(0), P, Q,
              _ptr(wu_t), wu_t.shape[0], wu_width, _ptr(wd_t), wd_t.shape[0], wd_width, _ptr(ws), _ptr(y), y.stride(0),
              y.shape[1], _stream(x.device))


def resample(x, orig, new, kernel, width, out=None, workspace=None):
    """Sinc resample rows of x [B, N] (gcd-reduced orig/new rates); returns [B, ceil(new*N/orig)] view."""
    B, N = x.shape
    Kpad = kernel.shape[1]
    F = N // orig + 1
    if out is None:
        out = torch.empty((B, F * new), dtype=torch.float32, device=x.device)
    if workspace is None:
        nbytes = _lib.lib().hfa_resample_workspace_bytes(B, N, orig, Kpad)
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    _lib.call("hfa_resample_f32", B, N, _ptr(x), x.stride(0), orig, new, _ptr(kernel), Kpad, width,
              _ptr(workspace), _ptr(out), out.stride(0), _stream(x.device))
    from .resample import target_length
    return out[:, : target_length(N, orig, new)]
