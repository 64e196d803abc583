"""Layer-level numerics of every encoder HIP kernel against a plain PyTorch fp32/fp64 CPU reference.

Tolerances are written per test; the f32 MFMA path is an exact fmaf chain, so differences are summation-order
only (~1e-6 relative at K <= 6144).
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F = torch.nn.functional
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def _close(got, ref, rtol, atol):
    got = got.detach().cpu().double()
    ref = ref.detach().cpu().double()
    err = (got - ref).abs()
    bound = atol + rtol * ref.abs()
    assert bool((err <= bound).all()), f"max err {float(err.max()):.3e}, max rel {float((err / (ref.abs() + 1e-30)).max()):.3e}"


@pytest.mark.parametrize("M,N,K,epi,res", [(300, 200, 128, 0, False), (1000, 768, 768, 1, False),
                                           (257, 65, 192, 0, True), (4096, 3072, 768, 1, False),
                                           (130, 2304, 768, 0, False), (64, 768, 3072, 0, True)])
def test_gemm_linear(M, N, K, epi, res):
    from hubertfa_amd import ops
    x, w, b = _r(M, K, seed=1), _r(N, K, seed=2, scale=K ** -0.5), _r(N, seed=3)
    r = _r(M, N, seed=4) if res else None
    ref = x.double() @ w.double().T + b.double()
    if epi:
        ref = F.gelu(ref)
    if res:
        ref = ref + r.double()
    d = torch.device("cuda")
    got = ops.linear(x.to(d), w.to(d), b.to(d), residual=r.to(d) if res else None, epilogue=epi)
    _close(got, ref, 2e-5, 2e-5)


@pytest.mark.parametrize("Cin,Cout,k,s,pad,T,G", [(512, 512, 3, 2, 0, 301, 1), (512, 512, 2, 2, 0, 100, 1),
                                                  (192, 192, 3, 1, 1, 64, 1), (768, 768, 128, 1, 64, 49, 16),
                                                  (192, 384, 2, 2, 0, 40, 1)])
def test_conv_gemm_vs_conv1d(Cin, Cout, k, s, pad, T, G):
    """Implicit-GEMM conv on channels-last activations == torch conv1d (channels-first)."""
    from hubertfa_amd import ops
    B = 2
    x = _r(B, T, Cin, seed=5)
    w = _r(Cout, Cin // G, k, seed=6, scale=(Cin // G * k) ** -0.5)
    b = _r(Cout, seed=7)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=s, padding=pad, groups=G)
    ref = ref.transpose(1, 2)
    Tout = ref.shape[1]
    d = torch.device("cuda")
    Cg, Ng = Cin // G, Cout // G
    # im2col weight order [Cout][k][Cin/G]
    wk = w.permute(0, 2, 1).contiguous().to(d)
    out = torch.empty(B, Tout, Cout, device=d)
    xd = x.to(d)
    ops.conv_gemm(xd, wk, out, M=Tout, N=Ng, K=k * Cg, Zb=B, G=G, sAb=T * Cin, sAg=Cg, ldx=Cin, stride=s, pad=pad,
                  Cg=Cg, Tin=T, sWg=Ng * k * Cg, bias=b.to(d), sBg=Ng, sCb=Tout * Cout, sCg=Ng, ldc=Cout)
    _close(out, ref, 5e-5, 5e-5)


@pytest.mark.parametrize("bk,bn", [(16, c) for c in range(1, 8)] + [(32, 1), (32, 3)] +
                         [(p, c) for p in (102, 103) for c in (1, 2, 4)] + [(102, 9)])
def test_gemm_tile_variants(bk, bn):
    """Every tile instantiation (register-staged BK 16/32, LDS-DMA 2/3 stages) is exact on a conv and a Linear
    shape with tails in M and N."""
    from hubertfa_amd import ops, _lib
    _lib.lib().hfa_gemm_tuning(bk, bn)
    try:
        d = torch.device("cuda")
        x, w, b = _r(2, 301, 512, seed=21), _r(200, 512, 3, seed=22, scale=(3 * 512) ** -0.5), _r(200, seed=23)
        ref = F.gelu(F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=2)).transpose(1, 2)
        Tout = ref.shape[1]
        out = torch.empty(2, Tout, 200, device=d)
        ops.conv_gemm(x.to(d), w.permute(0, 2, 1).contiguous().view(200, -1).to(d), out, M=Tout, N=200, K=1536,
                      Zb=2, sAb=301 * 512, ldx=512, stride=2, Cg=512, Tin=301, bias=b.to(d), sCb=Tout * 200, ldc=200,
                      epilogue=ops.EPI_GELU)
        _close(out, ref, 5e-5, 5e-5)
        x2, w2 = _r(77, 96, seed=24), _r(50, 96, seed=25)
        _close(ops.linear(x2.to(d), w2.to(d)), x2.double() @ w2.double().T, 2e-5, 2e-5)
    finally:
        _lib.lib().hfa_gemm_tuning(0, 0)


@pytest.mark.parametrize("Cg,Ng,k,pad,T,G,epi", [(48, 48, 7, 3, 150, 4, 1), (48, 48, 128, 64, 499, 2, 1),
                                                  (64, 40, 3, 1, 77, 3, 0), (96, 33, 1, 0, 300, 1, 1)])
def test_gemm_n48_tile(Cg, Ng, k, pad, T, G, epi):
    """The 48-wide 16x16x4-MFMA tile (32 < N <= 48): grouped padded convs with M tails, GELU and residual."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    B = 2
    Cin, Cout = Cg * G, Ng * G
    x = _r(B, T, Cin, seed=51)
    w = _r(Cout, Cg, k, seed=52, scale=(Cg * k) ** -0.5)
    b = _r(Cout, seed=53)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), b.double(), padding=pad, groups=G)[..., :T]
    if epi:
        ref = F.gelu(ref)
    ref = ref.transpose(1, 2)
    r = _r(B, T, Cout, seed=54)
    ref = ref + r.double()
    out = torch.empty(B, T, Cout, device=d)
    wk = w.permute(0, 2, 1).contiguous().to(d)
    args = dict(M=T, N=Ng, K=k * Cg, Zb=B, G=G, sAb=T * Cin, sAg=Cg, ldx=Cin, stride=1, pad=pad, Cg=Cg, Tin=T,
                sWg=Ng * k * Cg, bias=b.to(d), sBg=Ng, R=r.to(d), sRb=T * Cout, sRg=Ng, ldr=Cout, sCb=T * Cout,
                sCg=Ng, ldc=Cout, epilogue=epi)
    xd = x.to(d)
    name = ops._gemm_name(T, Ng, k * Cg, B, G, ops._ptr(xd), T * Cin, Cg, Cin, 1, pad, Cg, T, ops._ptr(wk),
                          Ng * k * Cg, k * Cg, ops._ptr(b), Ng, ops._ptr(r), T * Cout, Ng, Cout, ops._ptr(out),
                          T * Cout, Ng, Cout, epi)
    assert name.startswith("gemm_dma_n48_kernel"), name
    ops.conv_gemm(xd, wk, out, **args)
    _close(out, ref, 5e-5, 5e-5)


@pytest.mark.parametrize("N,ldc,res", [(198, 200, True), (198, 200, False), (61, 64, True), (130, 131, True)])
def test_gemm_epilogue_tails(N, ldc, res):
    """Vector (dwordx4 through LDS) and scalar epilogues: N tails inside an aligned row, unaligned rows, residual."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    M, K = 333, 256
    x, w, b = _r(M, K, seed=41), _r(N, K, seed=42, scale=K ** -0.5), _r(N, seed=43)
    r = _r(M, ldc, seed=44)
    out = torch.full((M, ldc), 7.0, device=d)
    rd = r.to(d)
    ops.conv_gemm(x.to(d), w.to(d), out, M=M, N=N, K=K, ldx=K, bias=b.to(d), R=rd if res else None, ldr=ldc,
                  ldc=ldc, epilogue=ops.EPI_GELU)
    ref = F.gelu(x.double() @ w.double().T + b.double())
    if res:
        ref = ref + r.double()[:, :N]
    _close(out[:, :N], ref, 2e-5, 2e-5)
    assert bool((out[:, N:] == 7.0).all()), "wrote past N"


def test_branch_free_erf_bit_identical():
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    x = torch.cat([torch.linspace(-12, 12, 1 << 20), _r(1 << 18, seed=30) * 3,
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 0.99999994, 1.0000001, float("inf"), -float("inf")])]).to(d)
    y_nb, y_ref = torch.empty_like(x), torch.empty_like(x)
    _lib.call("hfa_selftest_erf", x.numel(), ops._ptr(x), ops._ptr(y_nb), ops._ptr(y_ref), ops._stream(d))
    assert torch.equal(y_nb.view(torch.int32), y_ref.view(torch.int32))


def test_epilogue_gelu_accuracy():
    """hfa::gelu_fast vs fp64 GELU: within 4 |x| 2^-24 + 1e-37 everywhere (the f32 formula 0.5x(1+erf)'s own
    cancellation floor is 2 |x| 2^-24; scripts/fit_gelu_erf.py), and within 12 ulp where 1+erf is not small."""
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    x = torch.cat([torch.linspace(-12, 12, 1 << 21), _r(1 << 20, seed=31) * 3,
                   torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.95 * 2 ** 0.5, 1e6, -1e6])]).to(d)
    y = torch.empty_like(x)
    _lib.call("hfa_selftest_gelu", x.numel(), ops._ptr(x), ops._ptr(y), ops._stream(d))
    xd, yd = x.cpu().double(), y.cpu().double()
    ref = 0.5 * xd * (1 + torch.erf(xd / math.sqrt(2)))
    err = (yd - ref).abs()
    assert bool((err <= 4 * xd.abs() * 2.0 ** -24 + 1e-37).all()), float((err / (xd.abs() * 2.0 ** -24 + 1e-37)).max())
    m = xd > -1.5
    ulp = torch.from_numpy(np.spacing(ref[m].abs().float().numpy())).double()
    assert float((err[m] / ulp).max()) <= 12


@pytest.mark.parametrize("B,H,L", [(2, 12, 499), (1, 16, 49), (3, 12, 64), (1, 12, 1)])
def test_attention(B, H, L):
    from hubertfa_amd import ops
    D = 64
    qkv = _r(B, L, 3 * H * D, seed=8, scale=1.5)
    q, k, v = qkv.double().split(H * D, dim=-1)
    q = q.view(B, L, H, D).transpose(1, 2)
    k = k.view(B, L, H, D).transpose(1, 2)
    v = v.view(B, L, H, D).transpose(1, 2)
    att = torch.softmax((q @ k.transpose(-1, -2)) * D ** -0.5, -1) @ v
    ref = att.transpose(1, 2).reshape(B, L, H * D)
    d = torch.device("cuda")
    qd = qkv.to(d)
    out = torch.empty(B, L, H * D, device=d)
    ops.attention(qd, qd[..., H * D:], qd[..., 2 * H * D:], out, B=B, H=H, L=L, head_dim=D, scale=D ** -0.5,
                  q_bs=L * 3 * H * D, q_ld=3 * H * D, k_bs=L * 3 * H * D, k_ld=3 * H * D, v_bs=L * 3 * H * D,
                  v_ld=3 * H * D, o_bs=L * H * D, o_ld=H * D)
    _close(out, ref, 1e-4, 2e-5)


@pytest.mark.parametrize("C,act", [(768, 0), (512, 1), (192, 2), (1024, 0), (384, 2)])
def test_layernorm(C, act):
    from hubertfa_amd import ops
    x = _r(333, C, seed=9, scale=3.0) + 0.5
    g, b = _r(C, seed=10) * 0.1 + 1, _r(C, seed=11) * 0.1
    ref = F.layer_norm(x.double(), (C,), g.double(), b.double(), 1e-5)
    ref = [lambda t: t, F.gelu, F.hardswish][act](ref)
    d = torch.device("cuda")
    got = ops.layernorm(x.to(d), g.to(d), b.to(d), 1e-5, act=act)
    _close(got, ref, 1e-5, 2e-5)


@pytest.mark.parametrize("B,T,C", [(3, 864, 192), (1, 30000, 192), (2, 9000, 384)])
def test_groupnorm_hardswish(B, T, C):
    """Single-pass and split-T (long rows, few (batch, group) pairs) GroupNorm + Hardswish."""
    from hubertfa_amd import ops
    x = _r(B, T, C, seed=12, scale=2.0) + 0.3
    g, b = _r(C, seed=13) * 0.1 + 1, _r(C, seed=14) * 0.1
    ref = F.hardswish(F.group_norm(x.double().transpose(1, 2), 16, g.double(), b.double(), 1e-5)).transpose(1, 2)
    d = torch.device("cuda")
    got = ops.groupnorm(x.to(d), 16, g.to(d), b.to(d), 1e-5, act=ops.ACT_HARDSWISH)
    _close(got, ref, 1e-5, 2e-5)
    lens = torch.tensor([T // 2 + 7 * i for i in range(B)], dtype=torch.int32)
    got = ops.groupnorm(x.to(d), 16, g.to(d), b.to(d), 1e-5, act=ops.ACT_HARDSWISH, t_len=lens.to(d))
    for i in range(B):
        n = int(lens[i])
        ref_i = F.hardswish(F.group_norm(x[i:i + 1, :n].double().transpose(1, 2), 16, g.double(), b.double(),
                                         1e-5)).transpose(1, 2)
        _close(got[i:i + 1, :n], ref_i, 1e-5, 2e-5)
        assert bool((got[i, n:] == 0).all())


@pytest.mark.parametrize("B,T,C", [(3, 864, 192), (2, 216, 384), (1, 30000, 192)])
def test_groupnorm_split_planes(B, T, C):
    """GroupNorm's split-plane output (the UNet block's second-conv operand) equals split(GroupNorm f32) bit for bit,
    planes-only and dual; a row of a variable-length batch gives the same bits as that row alone."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    x = (_r(B, T, C, seed=15, scale=2.0) + 0.3).to(d)
    g, b = (_r(C, seed=16) * 0.1 + 1).to(d), (_r(C, seed=17) * 0.1).to(d)
    y = ops.groupnorm(x, 16, g, b, 1e-5, act=ops.ACT_HARDSWISH)
    ps = ops.groupnorm(x, 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, out=False, out_split=True)
    assert torch.equal(ps, ops.split(y))
    y2, ps2 = ops.groupnorm(x, 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, out_split=True)
    assert torch.equal(y2, y) and torch.equal(ps2, ps)
    lens = torch.tensor([T - 5 * i for i in range(B)], dtype=torch.int32, device=d)
    yl, pl = ops.groupnorm(x, 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, t_len=lens, out_split=True)
    for i in range(B):
        n = int(lens[i])
        alone = ops.groupnorm(x[i:i + 1, :n].contiguous(), 16, g, b, 1e-5, act=ops.ACT_HARDSWISH)
        assert torch.equal(yl[i, :n], alone[0]), i
        assert bool((yl[i, n:] == 0).all()) and bool((pl[:, i, n:] == 0).all())
    assert torch.equal(pl, ops.split(yl))


def test_groupnorm_long_row_stats_pass_bits():
    """Rows of more than 64 parts (2 048 frames) get their statistics from gn_rows_stats_kernel, which sums the parts in
    the order the apply pass uses in-block for shorter rows: a 1 500-frame row inside a batch padded to 3 000 frames
    (stats pass) gives the bits it gets alone (in-block sums), and a 30 000-frame row matches f64 GroupNorm."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    C = 192
    x = (_r(2, 3000, C, seed=18, scale=2.0) + 0.3).to(d)
    g, b = (_r(C, seed=19) * 0.1 + 1).to(d), (_r(C, seed=20) * 0.1).to(d)
    lens = torch.tensor([3000, 1500], dtype=torch.int32, device=d)
    yl, pl = ops.groupnorm(x, 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, t_len=lens, out_split=True)
    alone, pa = ops.groupnorm(x[1:2, :1500].contiguous(), 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, out_split=True)
    assert torch.equal(yl[1, :1500], alone[0]) and torch.equal(pl[:, 1, :1500], pa[:, 0])
    xl = (_r(1, 30000, C, seed=21, scale=2.0) + 0.3)
    ref = F.hardswish(F.group_norm(xl.double().transpose(1, 2), 16, g.cpu().double(), b.cpu().double(),
                                   1e-5)).transpose(1, 2)
    y, _ = ops.groupnorm(xl.to(d), 16, g, b, 1e-5, act=ops.ACT_HARDSWISH, out_split=True)
    _close(y, ref, 1e-5, 2e-5)


def test_split_gemm_dual_output():
    """Dual epilogue: the f32 output (+bias, +residual) and the planes of that same value in one launch."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    M, N, K = 1000, 768, 512
    x, w = _r(M, K, seed=21).to(d), (_r(N, K, seed=22) * K ** -0.5).to(d)
    bias, res = _r(N, seed=23).to(d), _r(M, N, seed=24).to(d)
    xs, ws = ops.split(x), ops.split(w)
    y = ops.linear_split(xs, ws, bias, residual=res)
    y2, ys = ops.linear_split(xs, ws, bias, residual=res, out_split="dual")
    assert torch.equal(y2, y)
    assert torch.equal(ys, ops.split(y))


@pytest.mark.parametrize("M,N,K,epi", [(1000, 768, 512, 0), (997, 764, 768, 1), (15968 // 4, 768, 3072, 0)])
def test_split_gemm_residual_planes(M, N, K, epi):
    """Residual given as split planes (the post-LN residual stream): the same result as adding the f32 value the
    planes encode (hi + 2^-11 lo, exact in f32), within one f32 rounding of adding the original f32 residual; N not a
    multiple of the tile takes the column tail.  A plane residual with planes output is rejected."""
    from hubertfa_amd import ops, _lib
    d = torch.device("cuda")
    x, w = _r(M, K, seed=41).to(d), (_r(N, K, seed=42) * K ** -0.5).to(d)
    bias, res = _r(N, seed=43).to(d), (3 * _r(M, N, seed=44)).to(d)
    xs, ws, rs = ops.split(x), ops.split(w), ops.split(res)
    r22 = rs[0].float() + rs[1].float() / 2048.0               # the value the planes carry
    y_pl = ops.linear_split(xs, ws, bias, residual=rs, epilogue=epi)
    y_f22 = ops.linear_split(xs, ws, bias, residual=r22.contiguous(), epilogue=epi)
    y_f32 = ops.linear_split(xs, ws, bias, residual=res, epilogue=epi)
    assert torch.equal(y_pl, y_f22)
    assert float((y_pl - y_f32).abs().max()) <= 2.0 ** -21 * float(res.abs().max()) + 1e-6
    with pytest.raises(_lib.HFALibraryError):
        ops.conv_gemm_split(xs, ws, Cs=torch.empty(2, M, N, dtype=torch.float16, device=d), M=M, N=N, K=K, ldx=K,
                            R=rs, ldr=N, ldc=N)


def test_conv0_groupnorm_gelu():
    from hubertfa_amd import ops
    B, N = 2, 16000
    x = _r(B, N, seed=15, scale=0.3)
    w = _r(512, 1, 10, seed=16, scale=0.3)
    g, b = _r(512, seed=17) * 0.1 + 1, _r(512, seed=18) * 0.1
    c = F.conv1d(x.double()[:, None], w.double(), stride=5)
    ref = F.gelu(F.group_norm(c, 512, g.double(), b.double(), 1e-5)).transpose(1, 2)
    d = torch.device("cuda")
    got = ops.conv0(x.to(d), w.view(512, 10).contiguous().to(d), gamma=g.to(d), beta=b.to(d))
    _close(got, ref, 1e-4, 1e-5)
    raw = ops.conv0(x.to(d), w.view(512, 10).contiguous().to(d), bias=b.to(d))
    _close(raw, (c + b.double()[None, :, None]).transpose(1, 2), 1e-5, 1e-6)


def test_units_gather_matches_reference_index():
    from hubertfa_amd import ops
    z = np.load(os.path.join(GOLDEN, "gather_index.npz"))
    d = torch.device("cuda")
    for key in z.files:
        n44 = int(key.split("_")[0][1:])
        U = int(key.split("units")[1])
        idx = z[key]
        n_frames = n44 // 512 + 1
        C = 8
        units = torch.arange(U, dtype=torch.float32).repeat_interleave(C).view(1, U, C).to(d)
        ratio = (512 / 44100) / (320 / 16000)
        out = ops.units_gather(units, n_frames, n_frames + 3, ratio).cpu().numpy()
        assert np.array_equal(out[0, :n_frames, 0].astype(np.int32), idx), key
        assert np.all(out[0, n_frames:] == 0)


def test_resample_vs_restated_torchaudio():
    from hubertfa_amd.resample import Resampler
    from oracle.resample import resample as ref_resample
    x = _r(2, 16000, seed=19, scale=0.2)
    for o, n, w in ((16000, 44100, 6), (44100, 16000, 128)):
        xx = x if o == 16000 else ref_resample(x, 16000, 44100, 6)
        ref = ref_resample(xx.double(), o, n, w) if False else ref_resample(xx, o, n, w)
        got = Resampler(o, n, w)(xx.cuda())
        assert got.shape == ref.shape
        _close(got, ref, 1e-4, 2e-6)


@pytest.mark.parametrize("o,n,w,N", [(16000, 44100, 6, 160000), (44100, 16000, 128, 441000), (44100, 16000, 128, 4413),
                                     (16000, 44100, 6, 4097), (8000, 44100, 6, 12345), (22050, 44100, 6, 9999),
                                     (48000, 44100, 6, 48000), (24000, 16000, 128, 24001)])
def test_resample_split_vs_f32_and_restatement(o, n, w, N):
    """The resampler on the split-f16 GEMM (G = 1 for orig % 8 == 0, 8 shifted-tap groups for orig % 8 == 1, the
    f32 GEMM otherwise): same length as the f32 path and the restated torchaudio kernel, within the f32 path's own
    tolerance of the restatement, from a row-pitched (non-contiguous) input."""
    from hubertfa_amd.resample import Resampler
    from oracle.resample import resample as ref_resample
    x = _r(2, N + 40, seed=21, scale=0.2)[:, 7:N + 7]            # rows with a pitch
    ref = ref_resample(x.contiguous(), o, n, w)
    rs = Resampler(o, n, w)
    xd = x.cuda()
    got = rs(xd, split=True)
    f32 = rs(xd, split=False)
    assert got.shape == ref.shape == f32.shape
    _close(got, ref, 1e-4, 2e-6)
    _close(f32, ref, 1e-4, 2e-6)
    assert float((got.double() - f32.double()).abs().max()) < 2e-6


@pytest.mark.parametrize("N", [160000, 4097, 12345, 441 * 3 + 7, 160 * 25 + 159, 4_800_000, 37, 161])
def test_chain_resampler_vs_two_stages(N):
    """16 k -> 44.1 k -> 16 k as one composite pass + the exact edge frames (resample.ChainResampler) against the
    restated two stages (oracle/resample.py, f32 as torchaudio) within the stages' own split-path tolerance, and
    against the GPU's two-stage split path (which it replaces on the product path) to 2e-6; same length, from
    row-pitched input; N = 4.8 M is config 5's 300 s row."""
    from hubertfa_amd.resample import ChainResampler, Resampler
    from oracle.resample import resample as ref_resample
    B = 2 if N < 1_000_000 else 1
    x = _r(B, N + 40, seed=N % 1000, scale=0.2)[:, 5:N + 5]
    chain = ChainResampler(16000, 44100, 6, 128)
    xd = x.cuda()
    got = chain(xd)
    two = Resampler(44100, 16000, 128)(Resampler(16000, 44100, 6)(xd, split=True).contiguous(), split=True)
    assert got.shape == two.shape == (B, chain.out_length(N))
    assert float((got.double() - two.double()).abs().max()) < 2e-6
    if N <= 200_000:
        ref = ref_resample(ref_resample(x.contiguous(), 16000, 44100, 6), 44100, 16000, 128)
        assert got.shape == ref.shape
        _close(got, ref, 1e-4, 2e-6)


def test_chain_resampler_ragged_rows_as_alone():
    """A zero-padded batch with per-row lengths: every row's first out_length(n) samples are what the row gives
    alone -- interior frames through the same composite GEMM arithmetic, the last frames recomputed against that
    row's own end (its intermediate length's float32-quotient ceil)."""
    from hubertfa_amd.resample import ChainResampler
    chain = ChainResampler(16000, 44100, 6, 128)
    lens = [48000, 47999, 30001, 4000, 44100 + 3]
    N = max(lens)
    x = torch.zeros(len(lens), N)
    for b, n in enumerate(lens):
        x[b, :n] = _r(n, seed=50 + b, scale=0.3)
    xd = x.cuda()
    got = chain(xd, torch.tensor(lens, dtype=torch.int32).cuda())
    for b, n in enumerate(lens):
        alone = chain(xd[b:b + 1, :n].contiguous())[0]
        m = chain.out_length(n)
        assert alone.shape[0] == m
        assert float((got[b, :m].double() - alone.double()).abs().max()) <= 1e-7, b


@pytest.mark.parametrize("N", [16000, 160000, 4097])
def test_wav_normalize(N):
    from hubertfa_amd import ops
    x = _r(3, N, seed=20, scale=0.3) + 0.01
    ref = (x.double() - x.double().mean(-1, keepdim=True)) / torch.sqrt(x.double().var(-1, unbiased=False, keepdim=True) + 1e-7)
    got = ops.wav_normalize(x.cuda())
    _close(got, ref, 1e-5, 1e-5)
    # per-row lengths: statistics over each row's own samples, zeros past it, and the same bits as the row alone
    lens = torch.tensor([N, N - 1000, N // 3], dtype=torch.int32)
    got = ops.wav_normalize(x.cuda(), lens=lens.cuda())
    for i in range(3):
        n = int(lens[i])
        alone = ops.wav_normalize(x[i:i + 1, :n].contiguous().cuda())
        assert torch.equal(got[i, :n], alone[0]), i
        assert bool((got[i, n:] == 0).all())
