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
