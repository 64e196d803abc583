"""TEST INFRASTRUCTURE ONLY — restatement of torchaudio's sinc resampler (torchaudio.functional.functional
``_get_sinc_resample_kernel`` / ``_apply_sinc_resample_kernel``; transforms.Resample with the default
``resampling_method="sinc_interp_hann"``, ``rolloff=0.99``) as called by the reference:

  * tools/load_wav.py:7      Resample(sr, 44100)                        (lowpass_filter_width = 6)
  * tools/encoder.py:46-48   Resample(44100, 16000, lowpass_filter_width=128)

torchaudio is NOT installed in this container and is not pinned by the reference (requirements.txt: "install
manually"), so this restatement is PARITY UNPINNED: no reference output exists here to check it against.
It follows torchaudio's published algorithm with Resample's ``dtype=None``: positions in float64, the output
phase term in float32 promoted to float64, kernels *= window * scale, cast to float32; input padded by
(width, width + orig), conv1d with stride orig, output truncated to ceil(as_tensor(new * N / orig)) — a float32
quotient.
"""
from __future__ import annotations

import math

import torch


def sinc_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """_get_sinc_resample_kernel(..., dtype=None): idx in float64; the phase arange is int64 and its division by
    new_freq yields float32 (default dtype), promoted to float64 by the add; kernels *= window * scale; cast to
    float32 because dtype is None."""
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1)[:, None, None] / new + idx
    t *= base
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base / orig
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels *= window * scale
    return kernels.to(torch.float32), width, orig, new


def resample(x: torch.Tensor, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6) -> torch.Tensor:
    """x [..., N] float32 (CPU) -> [..., ceil(as_tensor(new*N/orig))] (_apply_sinc_resample_kernel)."""
    if orig_freq == new_freq:
        return x
    kernel, width, orig, new = sinc_kernel(orig_freq, new_freq, lowpass_filter_width)
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    n = x2.shape[-1]
    xp = torch.nn.functional.pad(x2, (width, width + orig))
    y = torch.nn.functional.conv1d(xp[:, None], kernel, stride=orig)
    y = y.transpose(1, 2).reshape(x2.shape[0], -1)
    target = int(torch.ceil(torch.as_tensor(new * n / orig)).long())       # float32 quotient, as torchaudio
    return y[..., :target].reshape(*shape[:-1], -1)
