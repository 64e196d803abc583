"""WAV reading (torchaudio.load replacement) + ``load_wav`` (reference: tools/load_wav.py:4-8).

The RIFF/WAVE decoder is native (libhfa ``hfa_wav_info`` / ``hfa_wav_read``, hubertfa_amd/csrc/wav.cpp): PCM
8/16/24/32-bit integer and IEEE float 32/64 (incl. WAVE_FORMAT_EXTENSIBLE), scaled like torchaudio's default
``normalize=True`` (int16 / 2^15, int32 / 2^31, 24-bit / 2^23, uint8 (x-128)/128), decoded straight into the
caller's array (``read_wav_into``: a row of infer.py's pinned batch buffer).  ``load_wav`` then resamples
sr -> sample_rate with the width-6 sinc on the GPU and returns channel 0.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np
import torch

from . import _lib

def _path(path) -> bytes:
    return os.fsencode(os.fspath(path))


def _err(path, e: Exception) -> ValueError:
    return ValueError(f"{path}: {e}")


def wav_info(path) -> tuple[int, int, int]:
    """-> (samples per channel, sample_rate, channels) from the RIFF headers only (the data chunk is not read):
    the batch plan and the multi-GPU shard costs need every file's length before any is decoded."""
    n, ch, sr = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
    try:
        _lib.call("hfa_wav_info", _path(path), ctypes.byref(n), ctypes.byref(ch), ctypes.byref(sr))
    except _lib.HFAArgumentError as e:      # an unreadable file (a missing library or a HIP error propagates)
        raise _err(path, e) from None
    return n.value, sr.value, ch.value


def read_wav_into(path, dst: np.ndarray, channel: int = 0) -> tuple[int, int]:
    """Decode ``channel`` of ``path`` into the front of the contiguous float32 array ``dst`` -> (frames,
    sample_rate).  ValueError if the file is unreadable or does not fit."""
    if dst.dtype != np.float32 or not dst.flags.c_contiguous:
        raise ValueError("read_wav_into: dst must be a contiguous float32 array")
    n, sr = ctypes.c_int64(), ctypes.c_int32()
    try:
        _lib.call("hfa_wav_read", _path(path), channel, dst.ctypes.data, dst.size, ctypes.byref(n),
                  ctypes.byref(sr))
    except _lib.HFAArgumentError as e:      # an unreadable file (a missing library or a HIP error propagates)
        raise _err(path, e) from None
    return n.value, sr.value


def read_wav(path) -> tuple[np.ndarray, int]:
    """-> (float32 [channels, N], sample_rate)."""
    n, _, ch = wav_info(path)
    x = np.empty((ch, n), np.float32)
    m, sr = read_wav_into(path, x.reshape(-1), channel=-1)
    if m != n:
        raise ValueError(f"{path}: changed while being read")
    return x, sr


def write_wav(path, x: np.ndarray, sr: int) -> None:
    """16-bit PCM mono writer (synthetic test/bench inputs)."""
    q = np.clip(np.round(np.asarray(x, np.float64) * 32768.0), -32768, 32767).astype("<i2")
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + q.nbytes) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sr, sr * 2, 2, 16))
        f.write(b"data" + struct.pack("<I", q.nbytes) + q.tobytes())


_RESAMPLERS = {}


def load_wav(path, device, sample_rate=None) -> torch.Tensor:
    """Channel 0 of ``path`` at ``sample_rate`` as a device tensor (tools/load_wav.py:4-8)."""
    from .resample import Resampler
    x, sr = read_wav(str(path))
    wave = torch.from_numpy(x[0]).to(device)
    if sample_rate is not None and sample_rate != sr:
        key = (sr, sample_rate, str(device))
        if key not in _RESAMPLERS:
            _RESAMPLERS[key] = Resampler(sr, sample_rate, 6, device)
        wave = _RESAMPLERS[key](wave)
    return wave
