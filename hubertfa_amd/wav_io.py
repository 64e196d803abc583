"""WAV reading (torchaudio.load replacement) + ``load_wav`` (reference: tools/load_wav.py:4-8).

RIFF/WAVE parser for PCM 8/16/24/32-bit integer and IEEE float 32/64 (incl. WAVE_FORMAT_EXTENSIBLE), scaled
like torchaudio's default ``normalize=True`` (int16 / 2^15, int32 / 2^31, 24-bit / 2^23, uint8 (x-128)/128).
``load_wav`` then resamples sr -> sample_rate with the width-6 sinc on the GPU and returns channel 0.
"""
from __future__ import annotations

import struct

import numpy as np
import torch


def read_wav(path) -> tuple[np.ndarray, int]:
    """-> (float32 [channels, N], sample_rate)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, bits = fmt
    if tag == 3:
        x = np.frombuffer(pcm, dtype="<f4" if bits == 32 else "<f8").astype(np.float32)
    elif tag == 1:
        if bits == 8:
            x = (np.frombuffer(pcm, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(pcm, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(pcm[: len(pcm) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = (np.frombuffer(pcm, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
        else:
            raise ValueError(f"{path}: unsupported PCM width {bits}")
    else:
        raise ValueError(f"{path}: unsupported WAVE format tag {tag}")
    n = len(x) // ch
    return x[: n * ch].reshape(n, ch).T.copy(), sr


def wav_info(path) -> tuple[int, int, int]:
    """-> (samples per channel, sample_rate, channels) from the RIFF headers only (the data chunk is skipped,
    not read): the sharding cost estimate of a multi-GPU run needs every file's length before any is loaded."""
    with open(path, "rb") as f:
        head = f.read(12)
        if head[:4] != b"RIFF" or head[8:12] != b"WAVE":
            raise ValueError(f"{path}: not a RIFF/WAVE file")
        fmt, n_bytes = None, None
        while True:
            hdr = f.read(8)
            if len(hdr) < 8:
                break
            cid, size = hdr[:4], struct.unpack("<I", hdr[4:])[0]
            if cid == b"fmt ":
                body = f.read(size)
                _, ch, sr, _, block, _ = struct.unpack("<HHIIHH", body[:16])
                fmt = (ch, sr, block)
                if size & 1:
                    f.seek(1, 1)
            else:
                if cid == b"data":
                    n_bytes = size
                f.seek(size + (size & 1), 1)
            if fmt is not None and n_bytes is not None:
                break
    if fmt is None or n_bytes is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    ch, sr, block = fmt
    return n_bytes // max(block, 1), sr, ch


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
