"""Guard bands around every device buffer the pipeline allocates, to rule out stores past a buffer's bounds.

DESIGN.md §3.2a records an intermittent wrong value in conv0's split-plane output that showed up only while the
next batch's encoder ran beside the previous batch's UNet head (two streams).  One explanation the round-1 review
raised: a co-resident kernel (a split GEMM epilogue, pad_rows / mask_rows, ...) storing past ITS output into a
neighbouring buffer such as conv0's.  These tests put every allocation made by the product code during a pipelined
run (torch.empty / empty_like / zeros, i.e. every activation, plane, lattice and workspace buffer) inside a 4 KiB
canary band on both sides, run the two-stream pipeline (uniform and variable-length batches), and check every band
byte; a second test does the same per kernel with ragged shapes and strided outputs (canaries in the row padding).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CANARY = 0xA5
BAND = 4096


class GuardedAlloc:
    """Patches torch.empty / empty_like / zeros so CUDA tensors live inside canary bands; check() verifies them."""

    def __init__(self):
        self.bufs = []
        self.orig = {}

    def _guarded(self, shape, dtype, device, fill=None):
        dtype = dtype or torch.get_default_dtype()
        n = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        raw = self.orig["full"]((n + 2 * BAND,), CANARY, dtype=torch.uint8, device=device)
        self.bufs.append((raw, n))
        t = raw[BAND:BAND + n].view(dtype).view(shape)
        if fill is not None:
            t.fill_(fill)
        return t

    @staticmethod
    def _shape(size):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = size[0]
        return tuple(int(s) for s in size)

    def __enter__(self):
        self.orig = {k: getattr(torch, k) for k in ("empty", "empty_like", "zeros", "full")}
        o = self.orig

        def empty(*size, dtype=None, device=None, **kw):
            dev = torch.device(device) if device is not None else None
            if dev is None or dev.type != "cuda" or kw.get("pin_memory") or kw.get("out") is not None:
                return o["empty"](*size, dtype=dtype, device=device, **kw)
            return self._guarded(self._shape(size), dtype, dev)

        def empty_like(x, dtype=None, device=None, **kw):
            dev = torch.device(device) if device is not None else x.device
            if dev.type != "cuda" or not x.is_contiguous() or kw:
                return o["empty_like"](x, dtype=dtype, device=device, **kw)
            return self._guarded(tuple(x.shape), dtype or x.dtype, dev)

        def zeros(*size, dtype=None, device=None, **kw):
            dev = torch.device(device) if device is not None else None
            if dev is None or dev.type != "cuda" or kw:
                return o["zeros"](*size, dtype=dtype, device=device, **kw)
            return self._guarded(self._shape(size), dtype, dev, fill=0)

        torch.empty, torch.empty_like, torch.zeros = empty, empty_like, zeros
        return self

    def __exit__(self, *exc):
        torch.empty, torch.empty_like, torch.zeros = self.orig["empty"], self.orig["empty_like"], self.orig["zeros"]

    def check(self):
        torch.cuda.synchronize()
        bad = []
        for i, (raw, n) in enumerate(self.bufs):
            head, tail = raw[:BAND], raw[BAND + n:]
            if not bool((head == CANARY).all()) or not bool((tail == CANARY).all()):
                hb = int((head != CANARY).sum())
                tb = int((tail != CANARY).sum())
                bad.append((i, n, hb, tb))
        return bad


def _folder(tmp_path, secs_rates):
    from hubertfa_amd import synth
    from hubertfa_amd.task import synth_checkpoint
    from hubertfa_amd.wav_io import write_wav
    d = synth.synth_dictionary(n_words=40)
    dpath = tmp_path / "dict.txt"
    dpath.write_text("".join(f"{w}\t{' '.join(p)}\n" for w, p in d.items()))
    seg = tmp_path / "segments"
    seg.mkdir()
    for i, (secs, sr) in enumerate(secs_rates):
        write_wav(seg / f"g{i}.wav", synth.synth_audio(int(secs * sr), sr, seed=70 + i), sr)
        (seg / f"g{i}.lab").write_text(synth.synth_lab(4 + i % 3, d, seed=70 + i))
    ck = tmp_path / "m.ckpt"
    synth_checkpoint(str(ck))
    return seg, dpath, ck


@pytest.mark.parametrize("kind", ["uniform", "ragged"])
def test_pipeline_guard_bands(tmp_path, kind):
    """The CLI's two-stream pipeline (encoder of batch i+1 beside the UNet head, lattice and DP of batch i), every
    product allocation banded: no kernel stores outside its own buffer.  Uniform batches run the dual-output and
    planes-only paths, ragged ones the masking paths (mask_rows, per-row GroupNorm / LayerNorm lengths)."""
    import infer
    import hubertfa_amd.g2p as g2p_mod
    from hubertfa_amd.task import ForcedAlignmentTask
    files = [(2.0, 16000)] * 6 if kind == "uniform" else [(2.0, 16000), (3.1, 16000), (1.2, 22050), (2.6, 22050),
                                                            (0.9, 16000), (3.3, 16000), (1.7, 16000)]
    seg, dpath, ck = _folder(tmp_path, files)
    g = g2p_mod.DictionaryG2P(dictionary=str(dpath))
    g.set_in_format("lab")
    rows = list(g.get_dataset(sorted(seg.rglob("*.wav"))))
    torch.set_grad_enabled(False)
    task = ForcedAlignmentTask.load_from_checkpoint(str(ck), device=torch.device("cuda"), hubert_model_path="synth:0")
    keys = list(range(len(rows)))
    ref = infer._predict(task, rows, keys, 2, [])
    with GuardedAlloc() as ga:
        got = infer._predict(task, rows, keys, 2, [])
        bad = ga.check()
        n_bufs = len(ga.bufs)
    assert n_bufs > 50, f"only {n_bufs} guarded allocations: the patch did not reach the pipeline"
    assert not bad, f"stores past buffer bounds (index, bytes, head bytes hit, tail bytes hit): {bad[:10]}"
    for k in keys:                                  # and the banded run computed exactly the normal results
        for f in ("ph_time_int", "ph_idx_seq", "frame_confidence", "edge_diff"):
            assert np.array_equal(np.asarray(got[k][f]), np.asarray(ref[k][f])), (k, f)


def _banded_rows(rows, cols, ld, dtype, planes=1):
    """A [planes, rows, ld] canary-filled buffer inside guard bands; returns (raw, view [planes, rows, cols])."""
    es = torch.empty((), dtype=dtype).element_size()
    n = planes * rows * ld * es
    raw = torch.full((n + 2 * BAND,), CANARY, dtype=torch.uint8, device="cuda")
    full = raw[BAND:BAND + n].view(dtype).view(planes, rows, ld)
    return raw, full, full[:, :, :cols]


def _untouched(raw, full, cols):
    torch.cuda.synchronize()
    pad = full[:, :, cols:].contiguous().view(torch.uint8)
    return (bool((raw[:BAND] == CANARY).all()) and bool((raw[-BAND:] == CANARY).all())
            and bool((pad == CANARY).all()))


@pytest.mark.parametrize("cfg", [0, 17, 18, 19, 20, 23, 24, 25])
@pytest.mark.parametrize("M,N,K", [(1, 68, 64), (257, 200, 96), (300, 516, 512), (1000, 772, 768)])
def test_split_gemm_epilogue_bounds(cfg, M, N, K):
    """Split GEMM epilogues (f32 + residual, planes-only, dual) on ragged M / N into strided outputs whose row
    padding holds canaries: nothing lands past column N, past row M, or outside the buffer."""
    from hubertfa_amd import ops, _lib
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).cuda()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).cuda()
    b = torch.randn(N, generator=g).cuda()
    r = torch.randn(M, N, generator=g).cuda()
    xs, ws = ops.split(x), ops.split(w)
    ld = N + 20
    _lib.lib().hfa_gemm_split_tuning(cfg)
    try:
        rawc, fullc, c = _banded_rows(M, N, ld, torch.float32)
        ops.conv_gemm_split(xs, ws, C=c[0], M=M, N=N, K=K, ldx=K, bias=b, R=r, ldr=N, ldc=ld)
        assert _untouched(rawc, fullc, N), "f32 + residual epilogue"
        rawp, fullp, p = _banded_rows(M, N, ld, torch.float16, planes=2)
        ops.conv_gemm_split(xs, ws, Cs=p, M=M, N=N, K=K, ldx=K, bias=b, ldc=ld, epilogue=ops.EPI_GELU)
        assert _untouched(rawp, fullp, N), "planes epilogue"
        rawc2, fullc2, c2 = _banded_rows(M, N, ld, torch.float32)
        rawp2, fullp2, p2 = _banded_rows(M, N, ld, torch.float16, planes=2)
        ops.conv_gemm_split(xs, ws, C=c2[0], Cs=p2, M=M, N=N, K=K, ldx=K, bias=b, R=r, ldr=N, ldc=ld)
        assert _untouched(rawc2, fullc2, N) and _untouched(rawp2, fullp2, N), "dual epilogue"
        assert torch.equal(c2[0], c[0])
    finally:
        _lib.lib().hfa_gemm_split_tuning(0)


def test_row_kernels_bounds():
    """conv0 (split planes), pad_rows, mask_rows, LayerNorm (planes), GroupNorm (planes), units gather and the split
    attention write only their own rows and columns."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    B, N = 3, 16000 + 37
    x = torch.randn(B, N, device=d) * 0.1
    T0 = (N - 10) // 5 + 1
    w0 = torch.randn(512, 10, device=d) * 0.3
    gm, bt = torch.ones(512, device=d), torch.zeros(512, device=d)
    raw, full, ys = _banded_rows(B * T0, 512, 512, torch.float16, planes=2)
    ops.conv0(x, w0, gamma=gm, beta=bt, out=ys.view(2, B, T0, 512), out_split=True)
    assert _untouched(raw, full, 512), "conv0 split"
    raw, full, y = _banded_rows(B, N + 80, N + 96, torch.float32)
    ops.pad_rows(x, 40, N + 80, out=y[0])
    assert _untouched(raw, full, N + 80), "pad_rows"
    raw, full, y = _banded_rows(B * 50, 192, 200, torch.float32)
    y3 = full[0].view(B, 50, 200)[:, :, :192]
    y3.copy_(torch.randn(B, 50, 192, device=d))
    ops.mask_rows(y3, torch.tensor([50, 17, 1], dtype=torch.int32, device=d))
    assert _untouched(raw, full, 192), "mask_rows"
    h = torch.randn(B, 64, 192, device=d)
    lens = torch.tensor([64, 30, 5], dtype=torch.int32, device=d)
    raw, full, ps = _banded_rows(B * 64, 192, 192, torch.float16, planes=2)
    ops.groupnorm(h, 16, torch.ones(192, device=d), torch.zeros(192, device=d), out=False, t_len=lens,
                  out_split=ps.view(2, B, 64, 192))
    assert _untouched(raw, full, 192), "groupnorm planes"
    raw, full, ps = _banded_rows(B * 64, 192, 192, torch.float16, planes=2)
    ops.layernorm(h, torch.ones(192, device=d), torch.zeros(192, device=d), t_len=lens,
                  out_split=ps.view(2, B, 64, 192))
    assert _untouched(raw, full, 192), "layernorm planes"
    L, H = 77, 768
    qkv = ops.split(torch.randn(B, L, 3 * H, device=d) * 0.5)
    raw, full, o = _banded_rows(B * L, H, H, torch.float16, planes=2)
    ops.attention_split(qkv, o.view(2, B, L, H), B=B, H=12, L=L, head_dim=64, scale=0.125,
                        key_len=torch.tensor([77, 40, 3], dtype=torch.int32, device=d))
    assert _untouched(raw, full, H), "attention split"
