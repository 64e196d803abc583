"""Sinc resampler (torchaudio Resample semantics) on the GPU: host-side tap table + HIP pad/GEMM kernel.

Replaces ``torchaudio.transforms.Resample`` at tools/load_wav.py:7 (sr -> 44100, lowpass_filter_width 6) and
tools/encoder.py:46-48 (44100 -> 16000, lowpass_filter_width 128).  Taps follow torchaudio's published
``sinc_interp_hann`` construction (rolloff 0.99, computed in float64, cast to float32) and are zero-padded to a
multiple of 16 so the MFMA implicit GEMM consumes them directly.  torchaudio is absent from this environment,
so its parity is unpinned (see oracle/resample.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import ops


def sinc_taps(orig_freq: int, new_freq: int, lowpass_filter_width: int, rolloff: float = 0.99):
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    pos = np.arange(-width, width + orig, dtype=np.float64) / orig          # tap positions (input grid)
    phase = -np.arange(new, dtype=np.float64)[:, None] / new                 # output phase offsets
    t = np.clip((phase + pos[None, :]) * base, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    arg = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        sinc = np.where(arg == 0, 1.0, np.sin(arg) / arg)
    taps = (sinc * window * (base / orig)).astype(np.float32)               # [new, 2*width + orig]
    return taps, width, orig, new


class Resampler:
    """GPU resampler for one (orig, new, width) triple; taps are uploaded once."""

    def __init__(self, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, device=None):
        self.identity = int(orig_freq) == int(new_freq)
        if self.identity:
            return
        taps, self.width, self.orig, self.new = sinc_taps(orig_freq, new_freq, lowpass_filter_width)
        kw = taps.shape[1]
        kpad = (kw + 15) // 16 * 16
        padded = np.zeros((self.new, kpad), np.float32)
        padded[:, :kw] = taps
        self.kernel = torch.from_numpy(padded).to(device or "cuda")

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if self.identity:
            return x
        squeeze = x.dim() == 1
        x2 = x.reshape(1, -1) if squeeze else x.reshape(-1, x.shape[-1])
        y = ops.resample(x2.contiguous().float(), self.orig, self.new, self.kernel, self.width)
        return y[0] if squeeze else y.reshape(*x.shape[:-1], y.shape[-1])
