"""Resampler split-GEMM tiles (run on the GPU box): the two resamples of config 2's path (16 k -> 44.1 k, 44.1 k ->
16 k; B = 32 x 10 s) and the one-pass chain that replaces them (resample.ChainResampler: composite GEMM + edge
frames) under each forced split tile (hfa_gemm_split_tuning) against the automatic choice, us per call (median of
5 x 20 calls, pad + GEMM [+ edges]) and a bit-for-bit check of the output; then the chain's parts alone."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import _lib  # noqa: E402
from hubertfa_amd import ops  # noqa: E402
from hubertfa_amd.resample import ChainResampler, Resampler  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return sorted(ts)[2]


def main():
    d = torch.device("cuda")
    up, down = Resampler(16000, 44100, 6, d), Resampler(44100, 16000, 128, d)
    x16 = torch.randn(32, 160000, device=d) * 0.1
    x44 = up(x16, split=True)
    chain = ChainResampler(16000, 44100, 6, 128, d)
    print(f"two stages: {timeit(lambda: down(up(x16, split=True), split=True)):7.1f} us", flush=True)
    for name, fn, x in (("16k->44.1k", lambda x: up(x, split=True), x16),
                        ("44.1k->16k", lambda x: down(x, split=True), x44), ("chain", chain, x16)):
        ref = fn(x).clone()
        for cfg in (0, 17, 18, 19, 20, 23, 24, 25):
            _lib.lib().hfa_gemm_split_tuning(cfg)
            same = torch.equal(fn(x), ref)
            us = timeit(lambda: fn(x))
            _lib.lib().hfa_gemm_split_tuning(0)
            print(f"{name:11s} cfg {cfg:2d}: {us:7.1f} us {'' if same else 'MISMATCH'}", flush=True)
    out = torch.empty((32, (160000 // 160 + 1) * 160), device=d)
    print(f"chain edges alone: {timeit(lambda: ops.resample_chain_edges(x16, None, 160, 441, chain.wu_t, chain.wu_width, chain.wd_t, chain.wd_width, out)):7.1f} us")
    print(f"chain body alone: {timeit(lambda: ops.resample_split(x16, 160, 160, chain.w_planes, 1, chain.W, out=out, n_out=160000)):7.1f} us")


if __name__ == "__main__":
    main()
