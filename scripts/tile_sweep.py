"""Split-GEMM tile sweep on the side stream's shapes (run on the GPU box): the UNet's convs / linears at config 2
(B = 32; 864 / 432 / 216 / 108 frames per utterance) and the resampler's 44.1 k -> 16 k GEMM, each under every
forced split tile (hfa_gemm_split_tuning) against the automatic choice: us per launch (median of 5 x 20) and a
bit-for-bit check against the automatic tile's output."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import _lib, ops  # noqa: E402

# name, T (frames per utterance), Cin, N (Cout), taps k (1: linear over B*T rows), stride
SHAPES = [("unet k3 864 192->192", 864, 192, 192, 3, 1), ("unet k3 432 192->192", 432, 192, 192, 3, 1),
          ("unet k3 216 192->192", 216, 192, 192, 3, 1), ("unet k3 108 384->384", 108, 384, 384, 3, 1),
          ("unet k3 864 768->192", 864, 768, 192, 3, 1), ("unet lin 432 192->384", 432, 192, 384, 1, 1),
          ("unet k2s2 864 192->192", 864, 192, 192, 2, 2), ("head lin 864 192->68", 864, 192, 68, 1, 1)]
# --encoder: the encoder's smaller main-stream shapes (feature projection; extractor conv6 = k2 s2 over 999 frames,
# and two off-path probes: k2 s2 over 499 frames, k3 s2 over 1999 frames)
ENC_SHAPES = [("feature proj 512->768", 15968, 512, 768, 1, 1), ("conv6 k2s2 Tin=999", 999, 512, 512, 2, 2),
              ("k2s2 Tin=499", 499, 512, 512, 2, 2), ("k3s2 Tin=1999", 1999, 512, 512, 3, 2)]
CFGS = (0, 17, 18, 19, 20, 23, 24, 25)


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
    enc = "--encoder" in sys.argv
    for name, T, Cin, N, k, s in (ENC_SHAPES if enc else SHAPES):
        B = 1 if (enc and k == 1) else 32
        K = k * Cin
        W = ops.split(torch.randn(N, K, device=d) * K ** -0.5)
        bias = torch.randn(N, device=d)
        A = ops.split(torch.randn(B, T, Cin, device=d))
        pad = k // 2 if (k == 3 and not enc) else 0     # the UNet's k3 convs pad 1; the extractor's do not
        M = (T + 2 * pad - k) // s + 1
        C = torch.empty(B, M, N, device=d)

        def go():
            ops.conv_gemm_split(A, W, C=C, M=M, N=N, K=K, Zb=B, sAb=T * Cin, ldx=Cin, stride=s, pad=pad, Cg=Cin,
                                Tin=T, bias=bias, sCb=M * N, ldc=N)
            return C
        ref = go().clone()
        for cfg in CFGS:
            _lib.lib().hfa_gemm_split_tuning(cfg)
            same = torch.equal(go(), ref)
            us = timeit(go)
            _lib.lib().hfa_gemm_split_tuning(0)
            print(f"{name:24s} M={M:4d} K={K:5d} cfg {cfg:2d}: {us:7.1f} us {'' if same else 'MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
