"""The 16 k -> 44.1 k -> 16 k chain as one composite filter (hubertfa_amd/resample.py chain_taps, ChainResampler):
the composed taps against the two stages evaluated in float64 (CPU), and the edge-frame rule the GPU edge pass
(hfa_resample_chain_edges) follows.  The GPU path itself: tests/test_kernels_gpu.py::test_chain_resampler_*."""
import numpy as np
import pytest

from hubertfa_amd.resample import chain_taps, sinc_taps, target_length


def _stage(x, taps, width, orig, new):
    """torchaudio's _apply_sinc_resample_kernel in float64: pad (width, width + orig), stride-orig frames, each
    frame's new outputs, truncated to the float32-quotient ceil."""
    n = x.shape[-1]
    kw = taps.shape[1]
    xp = np.concatenate([np.zeros(width), x, np.zeros(width + orig)])
    F = (len(xp) - kw) // orig + 1
    idx = np.arange(F)[:, None] * orig + np.arange(kw)[None, :]
    y = (xp[idx] @ taps.astype(np.float64).T).reshape(-1)
    return y[:target_length(n, orig, new)]


def _chain64(x):
    tu, wu, P, Q = sinc_taps(16000, 44100, 6)
    td, wd, _, _ = sinc_taps(44100, 16000, 128)
    return _stage(_stage(x, tu, wu, P, Q), td, wd, Q, P)


def _composite64(x, comp, W, P):
    n = len(x)
    xp = np.concatenate([np.zeros(W), x, np.zeros(comp.shape[1] + P)])
    F = n // P + 1
    idx = np.arange(F)[:, None] * P + np.arange(comp.shape[1])[None, :]
    return (xp[idx] @ comp.T).reshape(-1)


def _edge_frames(n, P, Q, kwd, wd):
    """Frames hfa_resample_chain_edges recomputes for an n-sample row (its rule, restated)."""
    len_u = target_length(n, P, Q)
    len_y = target_length(len_u, Q, P)
    left = set(range(-(-wd // Q)))
    num = len_u - (kwd - 1 - wd)
    i0 = 0 if num <= 0 else -(-num // Q)
    right = set(range(i0, (len_y - 1) // P + 1))
    return left | right, len_y


@pytest.mark.parametrize("n", [160000, 4000, 12345, 441 * 3 + 7, 160 * 25 + 159])
def test_chain_taps_match_two_stages_in_float64(n):
    """Inside the row (every frame the edge pass does not recompute) the composed filter IS the two stages: equal
    in float64 to 1e-12 of the signal, and the edge frames are exactly those where it is not."""
    tu, wu, P, Q = sinc_taps(16000, 44100, 6)
    td, wd, _, _ = sinc_taps(44100, 16000, 128)
    comp, W = chain_taps(tu, wu, td, wd, P, Q)
    assert comp.shape[1] % 32 == 0 and comp.shape[1] >= 2 * W + P
    x = np.random.default_rng(n).standard_normal(n) * 0.3
    ref = _chain64(x)
    got = _composite64(x, comp, W, P)
    edges, len_y = _edge_frames(n, P, Q, td.shape[1], wd)
    assert len(ref) == len_y
    scale = np.abs(ref).max()
    inner = np.array([i for i in range(-(-len_y // P)) if i not in edges])
    for i in inner:
        lo, hi = P * i, min(P * (i + 1), len_y)
        assert np.abs(got[lo:hi] - ref[lo:hi]).max() <= 1e-12 * scale, i
    # and the composite is NOT the chain on the edge frames (the rule recomputes what it must)
    assert max(np.abs(got[P * i:min(P * (i + 1), len_y)] - ref[P * i:min(P * (i + 1), len_y)]).max()
               for i in edges if P * i < len_y) > 1e-6 * scale
    assert len(edges) <= -(-wd // Q) + (td.shape[1] - 1 - wd) // Q + 3
