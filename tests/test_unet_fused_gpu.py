"""The fused lattice producer (unet.hip hfa_unet_head: UNet + head, one workgroup per utterance).

Checked against the chip-wide launches of the same layers (unet.py LatticeHead._chipwide, itself pinned by
tests/golden/unet_head.npz), against the reference modules' golden logits, for batch invariance (a row's bits do
not depend on the batch it runs in, as the reference's one-utterance runs require), for batches that mix rows above
and below FusedPlan.MAX_T, and for its range flag."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _head(input_dims=768, seed=21):
    from hubertfa_amd import synth
    from hubertfa_amd.unet import LatticeHead
    ua = synth.UNetArch(input_dims=input_dims)
    return ua, LatticeHead(ua, synth.synth_unet_state_dict(ua, seed=seed))


def _feats(ua, tps, Tmax, seed=0):
    """Padded variable-length features: row b valid for its own t_pad (zeros beyond)."""
    from hubertfa_amd import synth
    x = np.zeros((len(tps), Tmax, ua.input_dims), np.float32)
    for b, t in enumerate(tps):
        x[b, :t] = synth.rng(seed + b).standard_normal((t, ua.input_dims)).astype(np.float32)
    return torch.from_numpy(x).cuda()


def test_fused_plan_builds_and_runs():
    ua, head = _head()
    assert head.fused is not None, "the default UNet must take the fused kernel"
    assert head.fused.nops == 21        # 7 blocks x 2 convs + 3 down + 3 up + the head
    x = _feats(ua, [864], 864)
    lg = head.logits(x)
    assert lg.shape == (1, 864, ua.vocab_size + 2) and bool(torch.isfinite(lg).all())


@pytest.mark.parametrize("tps", [[864], [864, 216, 8], [208, 432]])
def test_fused_matches_chipwide(tps):
    ua, head = _head()
    Tmax = max(tps)
    x = _feats(ua, tps, Tmax, seed=len(tps))
    fused = head.logits(x, t_pad=tps if len(set(tps)) > 1 else None)
    ref = head._chipwide(x, t_pad=tps if len(set(tps)) > 1 else None)
    for b, t in enumerate(tps):
        e = float((fused[b, :t] - ref[b, :t]).abs().max())
        print(f"T={t}: fused vs chip-wide max |diff| {e:.2e}")
        assert e < 2e-4


def test_fused_vs_reference_golden():
    """unet_head.npz (the reference UNetBackbone + head at T = 203, 862) through the fused kernel."""
    ua, head = _head()
    z = np.load(os.path.join(GOLDEN, "unet_head.npz"))
    from hubertfa_amd import synth
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        Tp = head.padded_len(T)
        xp = np.zeros((1, Tp, ua.input_dims), np.float32)
        xp[:, :T] = x
        lg = head.fused(torch.from_numpy(xp).cuda(), [Tp], head.ctx.flag)[0, :T].cpu().numpy()
        e = float(np.abs(lg - z[f"T{T}_logits"]).max())
        print(f"fused unet T={T}: max err vs the reference {e:.2e}")
        assert e < 2e-4


def test_fused_batch_invariance():
    ua, head = _head()
    tps = [432, 864, 120]
    x = _feats(ua, tps, 864, seed=7)
    batch = head.logits(x, t_pad=tps)
    for b, t in enumerate(tps):
        alone = head.logits(x[b:b + 1, :t].contiguous())
        assert torch.equal(batch[b, :t], alone[0]), f"row {b} differs from its one-utterance run"


def test_fused_mixed_with_long_rows():
    """Rows above FusedPlan.MAX_T take the chip-wide path inside the same call; every row equals its own run."""
    from hubertfa_amd.unet import FusedPlan
    ua, head = _head()
    long_t = FusedPlan.MAX_T + 256
    tps = [long_t, 512]
    x = _feats(ua, tps, long_t, seed=11)
    out = head.logits(x, t_pad=tps)
    for b, t in enumerate(tps):
        alone = head.logits(x[b:b + 1, :t].contiguous())
        assert torch.equal(out[b, :t], alone[0]), f"row {b} (T={t})"


def test_fused_range_flag():
    ua, head = _head()
    x = _feats(ua, [64], 64)
    x[0, 3, 5] = 1e6                       # outside f16 range: the split operand flags it
    head.ctx.flag.zero_()
    head.fused(x, [64], head.ctx.flag)
    torch.cuda.synchronize()
    assert int(head.ctx.flag.item()) == 1
    head.ctx.flag.zero_()


@pytest.mark.parametrize("input_dims", [256, 1024])
def test_fused_other_encoder_widths(input_dims):
    """hubertsoft (256) and Hubert-large (1024) feature widths."""
    ua, head = _head(input_dims=input_dims, seed=5)
    x = _feats(ua, [216], 216, seed=3)
    e = float((head.logits(x) - head._chipwide(x)).abs().max())
    assert e < 2e-4, e


# ---- the tiled form (hfa_unet_head_tiled: one launch per op, one workgroup per row block and utterance) ----------

def _tiled(head, x, tps):
    return head.fused(x, tps, head.ctx.flag, tiled=True)


@pytest.mark.parametrize("tps", [[864], [864, 216, 8], [208, 432], [2304, 512]])
def test_tiled_matches_chipwide(tps):
    ua, head = _head()
    Tmax = max(tps)
    x = _feats(ua, tps, Tmax, seed=len(tps) + 40)
    out = _tiled(head, x, tps)
    ref = head._chipwide(x, t_pad=tps if len(set(tps)) > 1 else None)
    for b, t in enumerate(tps):
        e = float((out[b, :t] - ref[b, :t]).abs().max())
        print(f"T={t}: tiled vs chip-wide max |diff| {e:.2e}")
        assert e < 2e-4


def test_tiled_vs_reference_golden():
    """unet_head.npz (the reference UNetBackbone + head at T = 203, 862) through the tiled launches."""
    ua, head = _head()
    z = np.load(os.path.join(GOLDEN, "unet_head.npz"))
    from hubertfa_amd import synth
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        Tp = head.padded_len(T)
        xp = np.zeros((1, Tp, ua.input_dims), np.float32)
        xp[:, :T] = x
        lg = _tiled(head, torch.from_numpy(xp).cuda(), [Tp])[0, :T].cpu().numpy()
        e = float(np.abs(lg - z[f"T{T}_logits"]).max())
        print(f"tiled unet T={T}: max err vs the reference {e:.2e}")
        assert e < 2e-4


def test_tiled_batch_invariance_and_determinism():
    """Each row equals its one-utterance run bit for bit (GroupNorm partials summed in row-block order), and two
    runs agree bit for bit."""
    ua, head = _head()
    tps = [432, 864, 120]
    x = _feats(ua, tps, 864, seed=9)
    batch = _tiled(head, x, tps)
    again = _tiled(head, x, tps)
    for b, t in enumerate(tps):                      # (rows past t_pad[b] are not written)
        assert torch.equal(batch[b, :t], again[b, :t])
    for b, t in enumerate(tps):
        alone = _tiled(head, x[b:b + 1, :t].contiguous(), [t])
        assert torch.equal(batch[b, :t], alone[0]), f"row {b} differs from its one-utterance run"


def test_tiled_through_logits_switch():
    """LatticeHead.logits routes to the tiled launches when use_tiled is set (the HFA_UNET_TILED switch)."""
    ua, head = _head()
    x = _feats(ua, [864, 432], 864, seed=5)
    ref = head._chipwide(x, t_pad=[864, 432])
    head.use_tiled = True
    try:
        out = head.logits(x, t_pad=[864, 432])
    finally:
        head.use_tiled = False
    assert float((out[0] - ref[0]).abs().max()) < 2e-4 and float((out[1, :432] - ref[1, :432]).abs().max()) < 2e-4


def test_tiled_range_flag():
    ua, head = _head()
    x = _feats(ua, [64], 64)
    x[0, 3, 5] = 1e6
    head.ctx.flag.zero_()
    _tiled(head, x, [64])
    torch.cuda.synchronize()
    assert int(head.ctx.flag.item()) == 1
    head.ctx.flag.zero_()
