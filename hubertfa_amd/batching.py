"""Host-side batching plans for the drop-in CLI (pure functions, CPU-tested).

The reference aligns one file per predict_step (networks/task/forced_alignment.py:154-186).  Here files of one
sample rate are sorted by length and aligned ``batch_size`` at a time as zero-padded variable-length batches
(every row then equals its one-utterance run: tests/test_varlen_gpu.py).  Files whose encoder input is shorter than
the 400-sample window take the reference's short-input quirk (tools/encoder.py:51-52, which pads the ORIGINAL
audio) and are aligned alone.
"""
from __future__ import annotations



def resampled_length(n: int, orig: int, new: int) -> int:
    """torchaudio Resample output length (hubertfa_amd.resample.target_length: a float32 ceil)."""
    from .resample import target_length
    return target_length(n, orig, new)


def encoder_length(n: int, file_sr: int, sr: int = 44100, enc_sr: int = 16000) -> int:
    """Samples the encoder sees for an n-sample file: load_wav resamples to ``sr`` (tools/load_wav.py:7), the
    encoder resamples that to ``enc_sr`` (tools/encoder.py:46-48)."""
    return resampled_length(resampled_length(n, file_sr, sr), sr, enc_sr)


def plan_batches(items, batch_size: int, sr: int = 44100, enc_sr: int = 16000, min_enc: int = 400):
    """items: iterable of (key, n_samples, file_sr) -> list of (file_sr, [keys]) batches.

    Per sample rate: short files (encoder input < ``min_enc``) one per batch, then the rest sorted by length in
    batches of at most ``batch_size`` (adjacent lengths, little padding)."""
    by_sr = {}
    for key, n, fsr in items:
        by_sr.setdefault(int(fsr), []).append((int(n), key))
    plan = []
    for fsr, group in by_sr.items():
        group.sort(key=lambda t: t[0])
        short = [k for n, k in group if encoder_length(n, fsr, sr, enc_sr) < min_enc]
        rest = [k for n, k in group if encoder_length(n, fsr, sr, enc_sr) >= min_enc]
        plan += [(fsr, [k]) for k in short]
        plan += [(fsr, rest[i:i + batch_size]) for i in range(0, len(rest), max(1, int(batch_size)))]
    return plan
