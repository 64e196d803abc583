"""The split GEMM + residual + LayerNorm in one launch (gemm.hip hfa_linear_split_ln, ops.linear_split_ln): the
last workgroup of every row block normalises that block's rows after an agent-scope counter hand-off.  It must give
exactly the bits of the two launches it replaces (linear_split, then layernorm), on every tile the shape picks,
every time (a stale read across XCDs would show up as a difference in some repeat), and leave its counters zero."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


@pytest.mark.parametrize("M,N,K,res", [(15968, 768, 768, "planes"), (15968, 768, 3072, "planes"),
                                       (1000, 768, 768, "f32"), (1, 768, 768, "planes"), (257, 512, 256, "f32"),
                                       (15968, 1024, 1024, "f32"), (130, 1024, 4096, "planes"), (64, 256, 64, None)])
def test_linear_split_ln_bits_equal_two_launches(M, N, K, res):
    from hubertfa_amd import ops
    d = torch.device("cuda")
    xs = ops.split(_r(M, K, seed=1).to(d))
    ws = ops.split(_r(N, K, seed=2, scale=K ** -0.5).to(d))
    b = _r(N, seed=3).to(d)
    g, be = (_r(N, seed=4) * 0.1 + 1).to(d), (_r(N, seed=5) * 0.1).to(d)
    r = _r(M, N, seed=6).to(d) if res else None
    rr = ops.split(r) if res == "planes" else r
    ref = ops.linear_split(xs, ws, b, residual=rr)
    ref_y, ref_s = ops.layernorm(ref, g, be, 1e-5, out=torch.empty_like(ref), out_split=True)
    cnt = ops._ln_counters(d, M)
    for rep in range(20):
        y, s = ops.linear_split_ln(xs, ws, b, rr, g, be, 1e-5, out_f32=True, out_split=True)
        assert torch.equal(y, ref_y) and torch.equal(s, ref_s), f"rep {rep}: fused LayerNorm differs"
    y2, s2 = ops.linear_split_ln(xs, ws, b, rr, g, be, 1e-5, out_f32=False, out_split=True)
    assert y2 is None and torch.equal(s2, ref_s)
    y3, s3 = ops.linear_split_ln(xs, ws, b, rr, g, be, 1e-5, out_f32=True, out_split=False)
    assert s3 is None and torch.equal(y3, ref_y)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0, "row-block counters left non-zero"


def test_linear_split_ln_range_flag():
    """An LN output outside f16 range raises the split flag, as the separate LayerNorm's plane output does."""
    from hubertfa_amd import ops
    d = torch.device("cuda")
    M, N, K = 300, 768, 256
    xs = ops.split(_r(M, K, seed=1).to(d))
    ws = ops.split(_r(N, K, seed=2, scale=K ** -0.5).to(d))
    g = torch.full((N,), 1e5, device=d)                  # |y| ~ 1e5 > 65504 for typical rows
    flag = ops.split_flag(d)
    flag.zero_()
    ops.linear_split_ln(xs, ws, None, None, g, torch.zeros(N, device=d), 1e-5)
    assert int(flag.item()) == 1
    flag.zero_()


@pytest.mark.parametrize("varlen", [False, True])
def test_encoder_fused_ln_bit_identical(varlen):
    """The post-LN encoder (cnhubert base, 12 layers) with the out-projection / FFN2 LayerNorms fused gives the units
    of the two-launch form bit for bit (uniform and variable-length batches)."""
    from hubertfa_amd import synth
    from hubertfa_amd.hubert import HubertEncoder
    d = torch.device("cuda")
    arch = synth.arch_cnhubert_base()
    enc = HubertEncoder(arch, synth.synth_hubert_state_dict(arch, seed=0), d)
    wav = torch.stack([torch.from_numpy(synth.synth_audio(48000, 16000, seed=s)) for s in range(3)]).to(d)
    lengths = [48000, 30000, 41000] if varlen else None
    enc.fuse_ln = False
    ref = enc(wav, lengths=lengths)
    enc.fuse_ln = True
    for _ in range(3):
        assert torch.equal(enc(wav, lengths=lengths), ref)
