"""TEST INFRASTRUCTURE ONLY — numpy restatement of torchaudio.load (default ``normalize=True``) on RIFF/WAVE, the
reader behind tools/load_wav.py:5, used by tests/ to check libhfa's native reader (hfa_wav_info / hfa_wav_read,
hubertfa_amd/csrc/wav.cpp).  PCM 8/16/24/32-bit integer and IEEE float 32/64 (incl. WAVE_FORMAT_EXTENSIBLE),
scaled as torchaudio's documented normalisation: uint8 (x-128)/128, int16 / 2^15, 24-bit / 2^23, int32 / 2^31.
torchaudio is absent here, so the scaling is pinned by its documentation and by the reference's own 16-bit
files being read identically (tests/test_api_gpu.py), not by torchaudio output.
"""
from __future__ import annotations

import struct

import numpy as np


def read_wav_np(path) -> tuple[np.ndarray, int]:
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


def wav_info_np(path) -> tuple[int, int, int]:
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
