"""Split-f16 GEMM path (gemm.hip gemm_split_kernel, hfa_split_f16, conv0 split output) against fp64 CPU references.

The split operand x = x1 + 2^-11 x2 keeps 22 significand bits; the product adds three exact f16 x f16 partial
products in f32.  Bars: the same tolerances as the f32 MFMA GEMM tests (2e-5 relative + 2e-5 absolute on unit-scale
data) — the split path is measured at or below the f32 path's own error (scripts/split_gemm_bench.py).
"""
import contextlib

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F = torch.nn.functional


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def _close(got, ref, rtol, atol):
    got = got.detach().cpu().double()
    ref = ref.detach().cpu().double()
    err = (got - ref).abs()
    assert bool((err <= atol + rtol * ref.abs()).all()), f"max err {float(err.max()):.3e}"


def test_split_planes_and_flag():
    from hubertfa_amd import ops
    d = torch.device("cuda")
    x = torch.cat([_r(1000, seed=1) * 100, _r(1000, seed=2) * 1e-3, torch.tensor([0.0, 1e-9, -65000.0, 3.0e-5])])
    x = x.reshape(1, -1)[:, :2000].contiguous()
    flag = ops.split_flag(d)
    flag.zero_()
    s = ops.split(x.to(d)).cpu().float()
    back = s[0] + s[1] / 2048.0
    err = (back.double() - x.double()).abs()
    assert bool((err <= 2.0 ** -22 * x.abs().double() + 2.0 ** -36).all())
    assert int(flag.item()) == 0
    for bad in (70000.0, float("inf"), float("nan")):
        flag.zero_()
        ops.split(torch.tensor([[1.0, bad, 2.0, 3.0, 4.0]], device=d))
        assert int(flag.item()) == 1, bad
    flag.zero_()


@pytest.mark.parametrize("cfg", [0, 15, 17, 18, 19, 20, 23, 24, 25])
@pytest.mark.parametrize("M,N,K,epi,res,outs", [(300, 200, 128, 0, False, False), (1000, 768, 768, 1, False, False),
                                                (257, 72, 192, 0, True, False), (4096, 3072, 768, 1, False, True),
                                                (130, 2304, 768, 0, False, True), (64, 768, 3072, 0, True, False)])
def test_split_linear(cfg, M, N, K, epi, res, outs):
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    x, w, b = _r(M, K, seed=1), _r(N, K, seed=2, scale=K ** -0.5), _r(N, seed=3)
    r = _r(M, N, seed=4) if res else None
    ref = x.double() @ w.double().T + b.double()
    if epi:
        ref = F.gelu(ref)
    if res:
        ref = ref + r.double()
    _lib.lib().hfa_gemm_split_tuning(cfg)
    try:
        got = ops.linear_split(ops.split(x.to(d)), ops.split(w.to(d)), b.to(d), residual=r.to(d) if res else None,
                               epilogue=epi, out_split=outs)
    finally:
        _lib.lib().hfa_gemm_split_tuning(0)
    if outs:
        got = got[0].float() + got[1].float() / 2048.0
        _close(got, ref, 2e-5 + 2.0 ** -21, 2e-5)
    else:
        _close(got, ref, 2e-5, 2e-5)


@pytest.mark.parametrize("cfg", [0, 17, 18, 19, 20])
@pytest.mark.parametrize("Cin,Cout,k,s,pad,T", [(512, 512, 3, 2, 0, 301), (512, 512, 2, 2, 0, 100),
                                                (192, 192, 3, 1, 1, 64), (192, 384, 2, 2, 0, 40),
                                                (512, 512, 3, 2, 0, 1301)])
def test_split_conv_vs_conv1d(Cin, Cout, k, s, pad, T, cfg):
    from hubertfa_amd import ops, _lib
    _lib.lib().hfa_gemm_split_tuning(cfg)
    B = 3
    d = torch.device("cuda")
    x = _r(B, T, Cin, seed=5)
    w = _r(Cout, Cin, k, seed=6, scale=(Cin * k) ** -0.5)
    b = _r(Cout, seed=7)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=s, padding=pad).transpose(1, 2)
    Tout = ref.shape[1]
    wi = w.permute(0, 2, 1).reshape(Cout, k * Cin).contiguous()
    y = torch.empty(B, Tout, Cout, device=d)
    try:
        ops.conv_gemm_split(ops.split(x.to(d)), ops.split(wi.to(d)), C=y, M=Tout, N=Cout, K=k * Cin, Zb=B,
                            sAb=T * Cin, ldx=Cin, stride=s, pad=pad, Cg=Cin, Tin=T, bias=b.to(d), sCb=Tout * Cout,
                            ldc=Cout)
    finally:
        _lib.lib().hfa_gemm_split_tuning(0)
    _close(y, ref, 2e-5, 2e-5)


@pytest.mark.parametrize("H,G,k,L,cfg", [(768, 16, 128, 499, 0), (768, 16, 128, 77, 18), (96, 2, 8, 40, 0),
                                         (640, 16, 16, 130, 0), (768, 16, 128, 300, 20), (1024, 16, 32, 260, 20),
                                         (1024, 16, 128, 499, 0), (768, 16, 128, 499, 15), (768, 16, 64, 1000, 15),
                                         (768, 16, 128, 5, 15), (96, 2, 8, 40, 15), (1024, 16, 32, 100, 15),
                                         (768, 16, 128, 499, 16), (768, 16, 128, 300, 16), (768, 16, 128, 3, 16),
                                         (768, 16, 128, 600, 16), (96, 2, 8, 40, 16), (512, 16, 64, 257, 16),
                                         (1024, 16, 128, 499, 16), (768, 16, 128, 499, 15)])
def test_split_grouped_posconv_general_taps(H, G, k, L, cfg):
    """Grouped positional conv with Cg = H/G not a multiple of 32 (48 at Hubert-base: per-lane tap tracking; the
    automatic choice and cfg 15 run the 16x16x32 N = 48 kernel), GELU + residual epilogue, pad k/2 and the last
    frame dropped, against f64 conv1d (model.py:132-147)."""
    from hubertfa_amd import ops, _lib
    B = 2
    Cg = H // G
    d = torch.device("cuda")
    x = _r(B, L, H, seed=12)
    w = _r(H, Cg, k, seed=13, scale=(Cg * k) ** -0.5)
    b = _r(H, seed=14) * 0.1
    conv = F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), padding=k // 2, groups=G)[..., :L]
    ref = x.double() + F.gelu(conv.transpose(1, 2))
    wi = w.permute(0, 2, 1).reshape(H, k * Cg).contiguous()
    xd = x.to(d)
    out = torch.empty(B, L, H, device=d)
    _lib.lib().hfa_gemm_split_tuning(cfg)
    try:
        ops.conv_gemm_split(ops.split(xd), ops.split(wi.to(d)), C=out, M=L, N=Cg, K=k * Cg, Zb=B, G=G, sAb=L * H,
                            sAg=Cg, ldx=H, stride=1, pad=k // 2, Cg=Cg, Tin=L, sWg=Cg * k * Cg, bias=b.to(d), sBg=Cg,
                            R=xd, sRb=L * H, sRg=Cg, ldr=H, sCb=L * H, sCg=Cg, ldc=H, epilogue=ops.EPI_GELU)
    finally:
        _lib.lib().hfa_gemm_split_tuning(0)
    _close(out, ref, 2e-5, 2e-5)


def test_posconv_window_tiles_bit_identical():
    """The window positional conv's 512-row tiles (M > 256, Cg = 48) and 256-row tiles run every output row through
    the same MFMA chain: rows whose 128-tap window lies inside the first 256 frames come out bit-identical from a
    499-frame call (512-row tile) and a 256-frame call (256-row tile)."""
    from hubertfa_amd import ops
    B, H, G, k = 2, 768, 16, 128
    Cg = H // G
    d = torch.device("cuda")
    x = _r(B, 499, H, seed=21).to(d)
    w = ops.split((_r(H, Cg, k, seed=22, scale=(Cg * k) ** -0.5)).permute(0, 2, 1).reshape(H, k * Cg).contiguous().to(d))
    b = (_r(H, seed=23) * 0.1).to(d)

    def run(L):
        xl = x[:, :L].contiguous()
        out = torch.empty(B, L, H, device=d)
        ops.conv_gemm_split(ops.split(xl), w, C=out, M=L, N=Cg, K=k * Cg, Zb=B, G=G, sAb=L * H, sAg=Cg, ldx=H,
                            stride=1, pad=k // 2, Cg=Cg, Tin=L, sWg=Cg * k * Cg, bias=b, sBg=Cg, R=xl, sRb=L * H,
                            sRg=Cg, ldr=H, sCb=L * H, sCg=Cg, ldc=H, epilogue=ops.EPI_GELU)
        return out
    assert ops._split_name(499, Cg, k * Cg, B * G, False, 1, Cg).endswith(", 4>")
    assert ops._split_name(256, Cg, k * Cg, B * G, False, 1, Cg).endswith(", 2>")
    assert torch.equal(run(499)[:, :192], run(256)[:, :192])


@pytest.mark.parametrize("outs", [False, True])
@pytest.mark.parametrize("cfgs", [(0, 17, 18, 19, 20, 23, 24, 25)])
def test_split_single_acc_tiles_bit_identical(outs, cfgs):
    """Every built tile (17 = 256x256, 18 = 128x128, 19 = 128x64, 20 = 256x64, 23 = 256x192, 24 = 192x256,
    25 = 128x192: single-accumulator 16x16x32 tiles) gives the same bits, so a row's result does not depend on the
    batch (and so the grid) it runs in."""
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    M, N, K = 700, 768, 1536
    xs, ws = ops.split(_r(M, K, seed=1).to(d)), ops.split(_r(N, K, seed=2, scale=K ** -0.5).to(d))
    b = _r(N, seed=3).to(d)
    outs_ = []
    for cfg in cfgs:
        _lib.lib().hfa_gemm_split_tuning(cfg)
        try:
            outs_.append(ops.linear_split(xs, ws, b, epilogue=ops.EPI_GELU, out_split=outs))
        finally:
            _lib.lib().hfa_gemm_split_tuning(0)
    for o in outs_[1:]:
        assert torch.equal(o, outs_[0])


@pytest.mark.parametrize("cfg,outs", [(17, False), (17, True), (18, True), (19, False), (20, True), (23, True),
                                      (24, False), (25, True), (25, False)])
def test_split_single_acc_weight_range_flag(cfg, outs):
    """Single-accumulator tiles form 2^11 * hi(w) in f16: a weight with |w| >= 32 overflows there, and the
    non-finite result raises the split flag (the caller re-runs on the f32 GEMM) instead of passing silently."""
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    M, N, K = 512, 512, 256
    x, w = _r(M, K, seed=1), _r(N, K, seed=2, scale=K ** -0.5)
    w[3, 7] = 40.0
    flag = ops.split_flag(d)
    flag.zero_()
    _lib.lib().hfa_gemm_split_tuning(cfg)
    try:
        ops.linear_split(ops.split(x.to(d)), ops.split(w.to(d)), None, out_split=outs)
    finally:
        _lib.lib().hfa_gemm_split_tuning(0)
    assert int(flag.item()) == 1
    flag.zero_()


@pytest.mark.parametrize("C,act,varlen", [(768, 0, False), (1024, 1, True), (192, 2, True), (512, 0, False)])
def test_layernorm_split_output(C, act, varlen):
    """LayerNorm's fused split-plane output equals split(LayerNorm(x)) bit for bit (padding rows zero)."""
    from hubertfa_amd import ops
    from hubertfa_amd.hubert import dev_lengths
    d = torch.device("cuda")
    B, T = 3, 50
    x = (_r(B, T, C, seed=20, scale=3.0) + 0.5).to(d)
    r = _r(B, T, C, seed=21).to(d)
    g, b = (_r(C, seed=22) * 0.1 + 1).to(d), (_r(C, seed=23) * 0.1).to(d)
    tl = dev_lengths([50, 17, 3], d) if varlen else None
    flag = ops.split_flag(d)
    flag.zero_()
    y, ys = ops.layernorm(x, g, b, 1e-5, act=act, residual=r, t_len=tl, out_split=True)
    y_ref = ops.layernorm(x, g, b, 1e-5, act=act, residual=r, t_len=tl)
    assert torch.equal(y, y_ref)
    assert torch.equal(ys, ops.split(y_ref))
    assert int(flag.item()) == 0
    big = torch.full((4, C), 1.0, device=d)
    big[:, 0] = 1e9                           # normalised output stays small: no flag
    ops.layernorm(big, g, b * 0 + 7e4, 1e-5, out_split=True)          # beta 7e4: every output >= 65504
    assert int(flag.item()) == 1
    flag.zero_()


def test_conv0_split_output_matches_f32():
    from hubertfa_amd import ops
    d = torch.device("cuda")
    B, N = 2, 16000
    x = _r(B, N, seed=8).to(d)
    w0 = _r(512, 10, seed=9, scale=0.3).to(d)
    g, bb = (1 + 0.1 * _r(512, seed=10)).to(d), (0.1 * _r(512, seed=11)).to(d)
    y32 = ops.conv0(x, w0, gamma=g, beta=bb)
    ys = ops.conv0(x, w0, gamma=g, beta=bb, out_split=True)
    back = ys[0].double() + ys[1].double() / 2048.0
    # the split output's conv runs on the f16 MFMA (3 exact split products, 2^-22 per operand), the f32 output's on
    # the VALU fmaf chain; GroupNorm scales the conv's rounding by rstd * gamma
    assert float((back - y32.double()).abs().max()) <= 2e-6 * float(y32.abs().max()) + 1e-9


@pytest.mark.parametrize("N,lens", [(16000, None), (12345, None), (16000, [16000, 5003]), (97, None)])
def test_conv0_packed_vs_f64(N, lens):
    """The packed f16-MFMA apply pass (three split products in one K step, stores through a per-wave LDS tile) and
    the f32 VALU pass against an f64 evaluation of conv -> GroupNorm -> GELU (and of the raw conv + bias planes of the
    LN-conv variant); ragged chunk tails and per-row frame counts (statistics over each row's own frames) included."""
    import torch.nn.functional as F
    from hubertfa_amd import ops
    from hubertfa_amd.hubert import dev_lengths
    d = torch.device("cuda")
    B = 2
    x = _r(B, N, seed=31, scale=0.3)
    w0 = _r(512, 10, seed=32, scale=0.3)
    g, bb = 1 + 0.1 * _r(512, seed=33), 0.1 * _r(512, seed=34)
    t0 = [(n - 10) // 5 + 1 for n in (lens or [N] * B)]
    tl = None if lens is None else dev_lengths(t0, d)
    ys = ops.conv0(x.to(d), w0.to(d), gamma=g.to(d), beta=bb.to(d), out_split=True, t0_len=tl)
    y32 = ops.conv0(x.to(d), w0.to(d), gamma=g.to(d), beta=bb.to(d), t0_len=tl)
    yb = ops.conv0(x.to(d), w0.to(d), bias=bb.to(d), out_split=True)
    torch.cuda.synchronize()
    c = F.conv1d(x.double()[:, None], w0.double()[:, None], stride=5)               # [B, 512, T0]
    for b in range(B):
        cb = c[b:b + 1, :, :t0[b]]
        ref = F.gelu(F.group_norm(cb, 512, g.double(), bb.double(), 1e-5))[0].T
        split = (ys[0, b, :t0[b]].double() + ys[1, b, :t0[b]].double() / 2048).cpu()
        scale = max(1.0, float(ref.abs().max()))
        assert float((split - ref).abs().max()) <= 4e-6 * scale, b
        assert float((y32[b, :t0[b]].double().cpu() - ref).abs().max()) <= 4e-6 * scale, b
    raw = (c[:, :, :].transpose(1, 2) + bb.double()).cpu()
    back = (yb[0].double() + yb[1].double() / 2048).cpu()
    assert float((back - raw).abs().max()) <= 2e-6 * max(1.0, float(raw.abs().max()))


def test_conv0_lag_product_stats_dc_heavy():
    """GroupNorm statistics from lag products on a wave with a large DC offset (mean >> std per channel: the
    variance is a small difference of large sums) against an f64 evaluation of conv -> GroupNorm -> GELU."""
    import torch.nn.functional as F
    from hubertfa_amd import ops
    d = torch.device("cuda")
    B, N = 2, 48000
    x = 0.8 + 0.01 * _r(B, N, seed=35)
    w0 = _r(512, 10, seed=36, scale=0.3)
    g, bb = 1 + 0.1 * _r(512, seed=37), 0.1 * _r(512, seed=38)
    c = F.conv1d(x.double()[:, None], w0.double()[:, None], stride=5)
    ref = F.gelu(F.group_norm(c, 512, g.double(), bb.double(), 1e-5)).transpose(1, 2)
    got = ops.conv0(x.to(d), w0.to(d), gamma=g.to(d), beta=bb.to(d))
    err = float((got.double().cpu() - ref).abs().max())
    assert err < 2e-4, err


def test_encoder_split_vs_f32_precision():
    """The whole Hubert-base encoder, split vs f32 GEMMs: units agree to f32-path accuracy."""
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    d = torch.device("cuda")
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    wav = _r(2, 32000, seed=12).to(d) * 0.1
    u32 = HubertEncoder(arch, sd, d, precision="f32")(wav)
    us = HubertEncoder(arch, sd, d, precision="split")(wav)
    assert float((us - u32).abs().max()) < 2e-4 * max(1.0, float(u32.abs().max()))


def test_range_guard_reruns_batch_on_f32():
    """An activation outside f16 range raises the split flag; assemble returns the f32-GEMM re-run of the batch,
    identical to running the batch with precision f32."""
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=d)
    task.on_predict_start()
    enc = task.unitsEncoder.model
    enc.conv_ln[0][1][5] = 1.0e5            # GroupNorm beta of one conv0 channel: that channel's output ~1e5
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(2, 2.0, 6, 5)
    w = torch.from_numpy(wav).to(d)
    calls = []
    redo = task._align_f32
    task._align_f32 = lambda *a: calls.append(1) or redo(*a)
    got = task.align_batch(w, ph_seqs, word_seqs, p2ws, wav_sr=16000)
    assert calls == [1]
    assert enc.precision == "split" and task.head.precision == "split"
    enc.precision = task.head.precision = "f32"
    ref = task.align_batch(w, ph_seqs, word_seqs, p2ws, wav_sr=16000)
    enc.precision = task.head.precision = "split"
    for a, b in zip(got, ref):
        assert list(a["ph_seq"]) == list(b["ph_seq"])
        assert (a["ph_intervals"] == b["ph_intervals"]).all()
    import hubertfa_amd.ops as ops
    assert int(ops.split_flag(d).item()) == 0


def test_range_guard_head_flag_reruns_batch():
    """A UNet activation outside f16 range raises the head's own flag (snapshot on the stream that ran the head,
    also through the two-stream submit path); the batch is re-run with f32 GEMMs in the encoder and the head."""
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=d)
    task.on_predict_start()
    blk = task.head.encoders[0][0]
    blk.gn[1][3] = 1.0e5                    # GroupNorm beta of one hidden channel: its conv2 input ~1e5
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(2, 2.0, 6, 5)
    w = torch.from_numpy(wav).to(d)
    calls = []
    redo = task._align_f32
    task._align_f32 = lambda *a: calls.append(1) or redo(*a)
    got = task.decoder.assemble(task.submit(w, ph_seqs, word_seqs, p2ws, wav_sr=16000), ph_seqs, word_seqs, p2ws)
    torch.cuda.synchronize()
    assert calls == [1]
    assert task.head.precision == "split" and int(task.head.flag.item()) == 0
    task.unitsEncoder.model.precision = task.head.precision = "f32"
    ref = task.align_batch(w, ph_seqs, word_seqs, p2ws, wav_sr=16000)
    task.unitsEncoder.model.precision = task.head.precision = "split"
    for a, b in zip(got, ref):
        assert list(a["ph_seq"]) == list(b["ph_seq"])
        assert (a["ph_intervals"] == b["ph_intervals"]).all()


def _attn_ref(qkv, B, L, H, D, lens=None):
    """f64 softmax(QK^T / sqrt(D)) V per (batch, head); with lens, keys >= lens[b] masked (rows past: don't care)."""
    q, k, v = qkv.double().split(H * D, dim=-1)
    q, k, v = (t.view(B, L, H, D).transpose(1, 2) for t in (q, k, v))
    s = (q @ k.transpose(-1, -2)) * D ** -0.5
    if lens is not None:
        mask = torch.arange(L)[None, :] >= torch.tensor(lens)[:, None]          # [B, L] keys
        s = s.masked_fill(mask[:, None, None, :], float("-inf"))
    return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, H * D)


@contextlib.contextmanager
def _attn_form(form):
    """hfa_attention_split's MFMA form for the block: 16 (16x16x32, the default), 32 (32x32x16)."""
    from hubertfa_amd import _lib
    _lib.call("hfa_attention_split_form", form)
    try:
        yield
    finally:
        _lib.call("hfa_attention_split_form", 0)


ATTN_FORMS = [16, 32]


@pytest.mark.parametrize("form", ATTN_FORMS)
@pytest.mark.parametrize("B,H,L", [(2, 12, 499), (1, 3, 64), (3, 2, 1), (1, 16, 200), (1, 1, 1500)])
def test_attention_split(B, H, L, form):
    """Split attention vs f64, at the f32 kernel's own tolerance (tests/test_kernels_gpu.py::test_attention), in
    both MFMA forms."""
    from hubertfa_amd import ops
    D = 64
    qkv = _r(B, L, 3 * H * D, seed=8, scale=1.5)
    ref = _attn_ref(qkv, B, L, H, D)
    d = torch.device("cuda")
    qs = ops.split(qkv.to(d))
    out = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)
    with _attn_form(form):
        ops.attention_split(qs, out, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5)
    got = out[0].float() + out[1].float() / 2048.0
    _close(got, ref, 1e-4, 2e-5)


@pytest.mark.parametrize("L", [499, 4999])
def test_attention_split_forms_agree(L):
    """The 16x16x32 and 32x32x16 forms compute the same products in the same K/V tile order and differ only in the
    MFMA's internal summation: against f64, the 16x16x32 form's largest error is within 1.25x the 32x32x16 form's
    (and both meet the split tolerance), at config 2's length and a long row; and the launched instantiation's name
    follows the form."""
    from hubertfa_amd import ops, _lib
    B, H, D = (4, 12, 64) if L < 1000 else (1, 2, 64)
    qkv = _r(B, L, 3 * H * D, seed=21, scale=2.0)
    ref = _attn_ref(qkv, B, L, H, D)
    d = torch.device("cuda")
    qs = ops.split(qkv.to(d))
    errs = []
    for form in (16, 32):
        with _attn_form(form):
            o = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)
            ops.attention_split(qs, o, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5)
            got = (o[0].double() + o[1].double() / 2048.0).cpu()
            name = _lib.lib().hfa_attention_split_kernel_name(B, H, L).decode()
            assert name.startswith("attn_fwd_split16_kernel<" if form == 16 else "attn_fwd_split_kernel<"), name
        _close(got.float(), ref, 1e-4, 2e-5)
        errs.append(float((got - ref).abs().max()))
    assert errs[0] <= 1.25 * errs[1] + 1e-7, errs


@pytest.mark.parametrize("form", ATTN_FORMS)
def test_attention_split_varlen(form):
    """Per-row key lengths: each row equals its own un-padded attention (rows past the length untouched)."""
    from hubertfa_amd import ops
    from hubertfa_amd.hubert import dev_lengths
    B, H, L, D = 3, 4, 300, 64
    lens = [300, 129, 65]
    qkv = _r(B, L, 3 * H * D, seed=9, scale=2.0)
    ref = _attn_ref(qkv, B, L, H, D, lens)
    d = torch.device("cuda")
    qs = ops.split(qkv.to(d))
    out = torch.full((2, B, L, H * D), float("nan"), dtype=torch.float16, device=d)   # padding rows must be written
    with _attn_form(form):
        ops.attention_split(qs, out, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5, key_len=dev_lengths(lens, d))
    got = (out[0].float() + out[1].float() / 2048.0).cpu()
    for b, n in enumerate(lens):
        _close(got[b, :n], ref[b, :n], 1e-4, 2e-5)
        assert bool((got[b, n:] == 0).all())


def test_attention_split_repeatable():
    """The pipelined K/V rings: 30 launches over a many-tile, many-workgroup batch are bit-identical, and a
    varlen batch equals each row run alone (an LDS stage overwritten while another wave still reads it shows
    up here as run-to-run differences)."""
    from hubertfa_amd import ops
    from hubertfa_amd.hubert import dev_lengths
    B, H, L, D = 16, 12, 499, 64
    d = torch.device("cuda")
    qs = ops.split(_r(B, L, 3 * H * D, seed=11, scale=2.0).to(d))
    lens = [L - 37 * (b % 9) for b in range(B)]
    kl = dev_lengths(lens, d)
    first = None
    side = torch.cuda.Stream(d)                      # a concurrent GEMM stream skews the waves of a workgroup
    a = torch.randn(4096, 4096, device=d)
    outs = []
    for i in range(40):
        if i % 4 == 0:
            with torch.cuda.stream(side):
                for _ in range(4):
                    a = torch.tanh(a @ a)
        out = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)
        ops.attention_split(qs, out, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5, key_len=kl)
        outs.append(out)
    torch.cuda.synchronize()
    first = outs[0]
    for i, out in enumerate(outs[1:]):
        assert torch.equal(out, first), f"launch {i + 1} differs from launch 0"
    for b in (0, 4, 8):
        n = lens[b]
        one = torch.empty(2, 1, n, H * D, dtype=torch.float16, device=d)
        ops.attention_split(qs[:, b:b + 1, :n].contiguous(), one, B=1, H=H, L=n, head_dim=D, scale=D ** -0.5)
        assert torch.equal(one[:, 0], first[:, b, :n])


@pytest.mark.parametrize("form", ATTN_FORMS)
@pytest.mark.parametrize("L", [499, 700])
def test_attention_split_waves_bit_identical(L, form):
    """4- and 8-wave workgroups give bit-identical planes (each query row sees the same key tiles in the same
    order), with and without per-row key lengths, in both MFMA forms."""
    from hubertfa_amd import ops, _lib
    from hubertfa_amd.hubert import dev_lengths
    B, H, D = 3, 4, 64
    d = torch.device("cuda")
    qs = ops.split(_r(B, L, 3 * H * D, seed=13, scale=2.0).to(d))
    for kl in (None, dev_lengths([L, L - 200, 65], d)):
        outs = []
        for nw in (4, 8):
            _lib.call("hfa_attention_split_tuning", nw)
            try:
                with _attn_form(form):
                    o = torch.full((2, B, L, H * D), float("nan"), dtype=torch.float16, device=d)
                    ops.attention_split(qs, o, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5, key_len=kl)
                outs.append(o)
            finally:
                _lib.call("hfa_attention_split_tuning", 0)
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("form", ATTN_FORMS)
def test_attention_split_large_scores(form):
    """Peaked softmax (scores ~ +-60): the score's own f32-level rounding dominates both kernels' error; the split
    kernel stays within 2x the f32 MFMA kernel's error against f64."""
    from hubertfa_amd import ops
    B, H, L, D = 1, 2, 777, 64
    qkv = _r(B, L, 3 * H * D, seed=10, scale=4.0)
    qkv[..., : H * D] *= 2.5
    ref = _attn_ref(qkv, B, L, H, D)
    d = torch.device("cuda")
    out = torch.empty(2, B, L, H * D, dtype=torch.float16, device=d)
    with _attn_form(form):
        ops.attention_split(ops.split(qkv.to(d)), out, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5)
    qd = qkv.to(d)
    o32 = torch.empty(B, L, H * D, device=d)
    ld = 3 * H * D
    ops.attention(qd, qd[..., H * D:], qd[..., 2 * H * D:], o32, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5,
                  q_bs=L * ld, q_ld=ld, k_bs=L * ld, k_ld=ld, v_bs=L * ld, v_ld=ld, o_bs=L * H * D, o_ld=H * D)
    e_split = float(((out[0].double() + out[1].double() / 2048.0).cpu() - ref).abs().max())
    e_f32 = float((o32.double().cpu() - ref).abs().max())
    assert e_split <= max(2.0 * e_f32, 2e-5), (e_split, e_f32)


@pytest.mark.parametrize("cap", [1, 7, 256])
def test_grid_cap_bit_identical(cap):
    """hfa_set_grid_cap (ops.grid_cap): the row-streaming kernels in a grid-stride loop over at most `cap`
    workgroups give the uncapped launches' outputs bit for bit -- split_f16 (and its range flag), LayerNorm at several
    row widths with residual, activation, split planes and varlen padding rows, and the lattice prologue; and the
    whole UNet head (its LayerNorms and conversions capped) on a variable-length batch."""
    from hubertfa_amd import ops
    from hubertfa_amd.hubert import dev_lengths
    d = torch.device("cuda")
    g = torch.Generator().manual_seed(cap)

    def both(fn):
        a = fn()
        with ops.grid_cap(cap):
            b = fn()
        torch.cuda.synchronize()
        return a, b
    x = torch.randn(3000, 768, generator=g).to(d)
    x[17, 5] = 70000.0                                          # out of f16 range: raises the flag
    for xa in (x, x[:, :700]):
        (pa, fa), (pb, fb) = both(lambda: (lambda f: (ops.split(xa, flag=f), f))(torch.zeros(1, dtype=torch.int32,
                                                                                             device=d)))
        assert torch.equal(pa, pb) and int(fa.item()) == int(fb.item()) == 1
    for C in (192, 384, 768, 1024):
        xb = torch.randn(4, 300, C, generator=g).to(d)
        res = torch.randn(4, 300, C, generator=g).to(d)
        gam, bet = torch.randn(C, generator=g).to(d), torch.randn(C, generator=g).to(d)
        tl = dev_lengths([300, 211, 5, 160], d)
        (oa, sa), (ob, sb) = both(lambda: ops.layernorm(xb, gam, bet, act=ops.ACT_GELU, residual=res, t_len=tl,
                                                        out_split=True))
        assert torch.equal(oa, ob) and torch.equal(sa, sb), C
    B, Tl, V, Smax = 5, 861, 65, 96
    fl = torch.randn(B, Tl, V, generator=g).to(d)
    el = torch.randn(B, Tl, generator=g).to(d)
    ids = torch.randint(0, V, (B, Smax), generator=g, dtype=torch.int32).to(d)
    Tv = torch.tensor([861, 430, 1, 0, 700], dtype=torch.int32, device=d)
    Sv = torch.tensor([91, 46, 3, 2, 96], dtype=torch.int32, device=d)
    from hubertfa_amd import synth
    from hubertfa_amd.unet import LatticeHead
    ua = synth.UNetArch(input_dims=768, vocab_size=63)
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_unet_state_dict(ua, seed=3).items()}
    head = LatticeHead(ua, sd, d)
    feats = torch.randn(6, 864, 768, generator=g).to(d)
    for t_pad in (None, [864, 432, 96, 864, 800, 8]):
        ha, hb = both(lambda: head.logits(feats, t_pad) if t_pad else head.logits(feats))
        assert torch.equal(ha, hb), t_pad
    la, lb = both(lambda: ops.lattice_prologue(fl, el, ids, Tv, Sv, want_frame_probs=True, init_dp=True))
    for b, (T, S) in enumerate(zip(Tv.tolist(), Sv.tolist())):      # what the prologue writes (the rest is empty())
        for k in ("edge_log", "not_edge_log", "edge_diff", "edge_prob", "ph_prob_log", "ph_frame_pred"):
            assert torch.equal(la[k][b, :T], lb[k][b, :T]), (k, b)
        assert torch.equal(la["prob_log"][b, :T, :S], lb["prob_log"][b, :T, :S]), b
        assert torch.equal(la["dp"][b, 0], lb["dp"][b, 0]) and torch.equal(la["curr"][b], lb["curr"][b]), b
