"""Sinc resampler (torchaudio Resample semantics) on the GPU: host-side tap table + HIP pad/GEMM kernel.

Replaces ``torchaudio.transforms.Resample`` at tools/load_wav.py:7 (sr -> 44100, lowpass_filter_width 6) and
tools/encoder.py:46-48 (44100 -> 16000, lowpass_filter_width 128).  Taps follow torchaudio's published
``sinc_interp_hann`` construction (rolloff 0.99, dtype flow of ``dtype=None``, cast to float32) and are zero-padded to a
multiple of 16 so the MFMA implicit GEMM consumes them directly.  torchaudio is absent from this environment,
so its parity is unpinned (see oracle/resample.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import ops


def target_length(n: int, orig_freq: int, new_freq: int) -> int:
    """Output samples of torchaudio's ``_apply_sinc_resample_kernel`` for an n-sample row:
    ``ceil(torch.as_tensor(new * n / orig))`` over the gcd-reduced rates.  The quotient is a Python float that
    ``as_tensor`` stores as float32 (the default dtype) before the ceil, so a quotient just above an integer can
    round down onto it (e.g. 44100 -> 16000 at n = 441 k + 3): the exact-integer ceil would be one sample more."""
    if int(orig_freq) == int(new_freq):
        return int(n)
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    return int(np.ceil(np.float32(new * int(n) / orig)))


def sinc_taps(orig_freq: int, new_freq: int, lowpass_filter_width: int, rolloff: float = 0.99):
    """Tap table [new, 2*width + orig] f32 following torchaudio's ``_get_sinc_resample_kernel`` with
    ``dtype=None`` (what ``transforms.Resample`` passes), operation for operation on torch CPU: positions in
    float64, the output-phase term ``arange(0, -new, -1) / new`` in float32 (int64 / int -> the default dtype)
    promoted to float64 by the add, ``kernels *= window * scale``, then the cast to float32."""
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    with torch.no_grad():
        pos = torch.arange(-width, width + orig, dtype=torch.float64)[None, :] / orig
        phase = torch.arange(0, -new, -1)[:, None] / new                    # float32
        t = (phase + pos) * base
        t = t.clamp(-lowpass_filter_width, lowpass_filter_width)
        window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
        t = t * math.pi
        sinc = torch.where(t == 0, torch.tensor(1.0, dtype=torch.float64), t.sin() / t)
        taps = (sinc * (window * (base / orig))).to(torch.float32)
    return taps.numpy(), width, orig, new


class Resampler:
    """GPU resampler for one (orig, new, width) triple; taps are uploaded once.

    ``split=True`` (the encoder's split precision) runs it on the split-f16 GEMM (ops.resample_split, f32-class)
    when the gcd-reduced orig is 0 or 1 mod 8 (16 k -> 44.1 k: 160; 44.1 k -> 16 k: 441): 16-B aligned A rows, with
    frames 8m + g as eight groups whose taps are shifted right by g for orig % 8 == 1; else, and for ``split=False``
    (the range guard's f32 re-run), the f32-MFMA GEMM (ops.resample)."""

    def __init__(self, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, device=None):
        self.identity = int(orig_freq) == int(new_freq)
        if self.identity:
            return
        taps, self.width, self.orig, self.new = sinc_taps(orig_freq, new_freq, lowpass_filter_width)
        dev = torch.device(device or "cuda")
        kw = taps.shape[1]
        kpad = (kw + 15) // 16 * 16
        padded = np.zeros((self.new, kpad), np.float32)
        padded[:, :kw] = taps
        self.kernel = torch.from_numpy(padded).to(dev)
        self.G = 1 if self.orig % 8 == 0 else (8 if self.orig % 8 == 1 else 0)
        self.w_planes = None
        if self.G and dev.type == "cuda":
            kg = (kw + self.G - 1 + 31) // 32 * 32
            wg = np.zeros((self.G, self.new, kg), np.float32)
            for g in range(self.G):
                wg[g, :, g:g + kw] = taps
            self.w_planes = ops.split(torch.from_numpy(wg).to(dev))

    def __call__(self, x: torch.Tensor, split: bool = False) -> torch.Tensor:
        if self.identity:
            return x
        squeeze = x.dim() == 1
        x2 = x.reshape(1, -1) if squeeze else x.reshape(-1, x.shape[-1])
        x2 = x2.float()
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        if split and self.w_planes is not None:
            y = ops.resample_split(x2, self.orig, self.new, self.w_planes, self.G, self.width)
        else:
            y = ops.resample(x2, self.orig, self.new, self.kernel, self.width)
        return y[0] if squeeze else y.reshape(*x.shape[:-1], y.shape[-1])


def chain_taps(tu, wu: int, td, wd: int, P: int, Q: int):
    """Composed taps of two sinc stages rate -> mid -> rate (ChainResampler): tu [Q, kwu] / td [P, kwd] the stages'
    float32 tap tables (sinc_taps), wu / wd their widths, P / Q the first stage's reduced orig / new.  Returns (C
    [P, Kg] float64, W): y[P i + q] = sum_m C[q][m] x[P i + m - W] wherever the second stage's window lies inside the
    intermediate row; Kg a multiple of 32 with Kg >= 2 W + P (hfa_resample_split's bound).  Second-stage tap l of
    output frame i reads r = Q i - wd + l, i.e. first-stage frame i + fl (fl = floor((l - wd) / Q)) at phase
    l - wd - Q fl, whose tap k reads input P (i + fl) - wu + k: column P fl - wu + k + W."""
    kwu, kwd = tu.shape[1], td.shape[1]
    fl_lo, fl_hi = (-wd) // Q, (kwd - 1 - wd) // Q
    W = -P * fl_lo + wu                                   # the lowest composed tap lands on column 0
    K = P * fl_hi + kwu - wu + W
    Kg = max(-(-K // 32) * 32, -(-(2 * W + P) // 32) * 32)
    comp = np.zeros((P, Kg), np.float64)
    tu64, td64 = tu.astype(np.float64), td.astype(np.float64)
    for fl in range(fl_lo, fl_hi + 1):
        l0, l1 = max(0, wd + Q * fl), min(kwd, wd + Q * (fl + 1))
        if l0 < l1:
            c0 = P * fl - wu + W
            comp[:, c0:c0 + kwu] += td64[:, l0:l1] @ tu64[np.arange(l0, l1) - wd - Q * fl, :]
    return comp, W


class ChainResampler:
    """Two sinc stages that return to the input rate as ONE pass: ``rate -> mid`` (width ``up_width``) then ``mid ->
    rate`` (width ``down_width``) -- HubertFA's 16 kHz input path, load_wav's resample to the melspec rate
    (tools/load_wav.py:7, width 6) followed by the encoder's resample back to 16 kHz (tools/encoder.py:46-48,
    width 128), whose 44.1 kHz wave nothing else reads (only its length: the frame grid).

    With P / Q the first stage's gcd-reduced orig / new (160 / 441), output frame i (outputs P i .. P i + P - 1) of
    the second stage reads the intermediate samples r = Q i - wd_width + l, and each of those reads input samples
    P (r div Q) - wu_width + k, so the chain is one polyphase filter of stride P over the input: y[P i + q] =
    sum_m C[q][m] x[P i + m - W], the composed taps C (P x ~494, against the 174 x 441 / 160 + 1155 = 1635 MACs per
    output of the two stages) summed in float64 from the stages' float32 taps, on the split-f16 GEMM
    (ops.resample_split, orig = new = P).  That form holds wherever the second stage's window lies inside the
    intermediate row; at the row's two ends each stage zero-pads its own input, which the composite cannot
    express, so those few frames (the first ceil(wd_width / Q), the last ~3 of each row) are recomputed exactly as the
    two stages compute them by ops.resample_chain_edges.  Results agree with the two-stage restatement
    (oracle/resample.py) within the split path's own tolerance (tests/test_kernels_gpu.py); torchaudio itself is
    absent, so, like the stages, parity is unpinned."""

    def __init__(self, rate: int, mid: int, up_width: int, down_width: int, device=None):
        tu, self.wu_width, self.P, self.Q = sinc_taps(rate, mid, up_width)          # [Q, kwu]
        td, self.wd_width, q2, p2 = sinc_taps(mid, rate, down_width)                # [P, kwd]
        if (q2, p2) != (self.Q, self.P) or self.P % 8 or td.shape[1] + 512 > 16384:
            raise ValueError("ChainResampler: the stages must return to the input rate with P % 8 == 0 and a second "
                             "stage of at most 15 872 taps (hfa_resample_chain_edges' window)")
        comp, self.W = chain_taps(tu, self.wu_width, td, self.wd_width, self.P, self.Q)
        self.Kg = comp.shape[1]
        dev = torch.device(device or "cuda")
        self.taps = comp                                  # float64, for tests
        self.w_planes = ops.split(torch.from_numpy(comp.astype(np.float32))[None].to(dev))
        self.wu_t = torch.from_numpy(np.ascontiguousarray(tu.T)).to(dev)            # [kwu, Q]
        self.wd_t = torch.from_numpy(np.ascontiguousarray(td.T)).to(dev)            # [kwd, P]

    def out_length(self, n: int) -> int:
        """The two stages' output length for an n-sample row (each stage's float32-quotient ceil)."""
        return target_length(target_length(int(n), self.P, self.Q), self.Q, self.P)

    def __call__(self, x: torch.Tensor, lens: torch.Tensor | None = None) -> torch.Tensor:
        """x [B, N] f32 (unit element stride) -> [B, out_length(N)]; ``lens`` (int32 device [B]): per-row input
        lengths of a zero-padded batch (each row then resamples as it would alone, up to its own output length;
        the columns past it are not defined: mask them)."""
        B, N = x.shape
        P = self.P
        out = torch.empty((B, (N // P + 1) * P), dtype=torch.float32, device=x.device)
        y = ops.resample_split(x, P, P, self.w_planes, 1, self.W, out=out, n_out=self.out_length(N))
        ops.resample_chain_edges(x, lens, P, self.Q, self.wu_t, self.wu_width, self.wd_t, self.wd_width, out)
        return y
