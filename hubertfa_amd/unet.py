"""Lattice producer: ``UNetBackbone`` + ``head`` of LitForcedAlignmentTask on libhfa kernels.

Reference: networks/layer/backbone/unet.py:9-119 (UNetBackbone), networks/layer/block/resnet_block.py:4-50
(ResidualBasicBlock), networks/layer/scaling/stride_conv.py:6-47 (DownSampling / UpSampling),
networks/task/forced_alignment.py:53-55, 284-292 (head + logit split).

All tensors stay channels-last [B, T, C]: the k3 convs are implicit GEMMs with pad 1 (zero rows outside [0, T)),
the stride-2 down-sampling conv is an implicit GEMM with overlapping-free rows, the transposed up-sampling conv is
ONE GEMM whose [T, 2*Cout] output is bit-for-bit the [2T, Cout] layout, GroupNorm/LayerNorm fuse their
Hardswish, and the residual shortcut is the second conv's epilogue.

Precision "split" (default on the GPU): every GEMM runs on the split-f16 MFMA kernel (f32-class accuracy, see
gemm.hip gemm_split_kernel), each GEMM input converted once to plane pairs; a value outside f16 range raises the
head's own flag (``LatticeHead.flag``), and the task re-runs the batch on the f32 GEMMs.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .synth import UNetArch


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else x.detach().cpu()


class _Ctx:
    """Per-head GEMM dispatch: split-f16 when the head runs split and the weight has planes, else f32."""

    def __init__(self, dev, precision):
        self.dev = dev
        self.precision = precision
        self.flag = torch.zeros(1, dtype=torch.int32, device=dev) if dev.type == "cuda" else None

    def planes(self, w):
        """One-time split of a weight; |w| >= 16 (none in practice) stays f32 (gemm.hip ONE tiles need |w| < 32)."""
        if self.precision != "split" or self.dev.type != "cuda" or w.shape[-1] % 32 or not bool(w.abs().max() < 16):
            return None
        return ops.split(w, flag=self.flag)

    def use_split(self, ws):
        return self.precision == "split" and ws is not None

    def split(self, x):
        return ops.split(x, flag=self.flag)

    def conv(self, x, xs, w, ws, out, out_s=None, **kw):
        """Implicit-GEMM conv into f32 ``out``; on the split path ``out_s`` (optional [2, ...] f16) also receives
        the output's planes (dual epilogue).  Returns (out, planes or None)."""
        if self.use_split(ws):
            ops.conv_gemm_split(xs if xs is not None else self.split(x), ws, C=out, Cs=out_s, flag=self.flag, **kw)
            return out, out_s
        ops.conv_gemm(x, w, out, **kw)
        return out, None

    def linear(self, x, xs, w, ws, bias=None, residual=None, dual=False):
        """Linear (+residual); ``dual`` on the split path: also the output's planes.  Returns (y, planes or None)."""
        if self.use_split(ws):
            r = ops.linear_split(xs if xs is not None else self.split(x), ws, bias, residual=residual, flag=self.flag,
                                 out_split="dual" if dual else False)
            return r if dual else (r, None)
        return ops.linear(x, w, bias, residual=residual), None

    def planes_for(self, t):
        """[2, *t.shape] f16 planes buffer on the split path, else None."""
        if self.precision != "split":
            return None
        return torch.empty((2, *t.shape), dtype=torch.float16, device=t.device)


class _Block:
    def __init__(self, sd, pre, dev, ctx):
        P = lambda n: _t(sd[pre + n]).float().contiguous().to(dev)  # noqa: E731
        self.ctx = ctx
        w1 = _t(sd[pre + "block.0.weight"]).float()
        w2 = _t(sd[pre + "block.3.weight"]).float()
        self.cin, self.hid, self.cout = w1.shape[1], w1.shape[0], w2.shape[0]
        self.w1 = w1.permute(0, 2, 1).reshape(self.hid, -1).contiguous().to(dev)
        self.w2 = w2.permute(0, 2, 1).reshape(self.cout, -1).contiguous().to(dev)
        self.gn = (P("block.1.weight"), P("block.1.bias"))
        self.n_groups = 16
        self.sc = P("shortcut.0.weight") if pre + "shortcut.0.weight" in sd else None
        self.ln = (P("out.0.weight"), P("out.0.bias"))
        self.w1s, self.w2s = ctx.planes(self.w1), ctx.planes(self.w2)
        self.scs = ctx.planes(self.sc) if self.sc is not None else None

    def __call__(self, x, lens=None, xs=None, want_split=False):
        """lens [B] int32 (variable-length batch): rows >= lens[b] are padding — zeroed on the way in (the k3
        convs must read zeros there) and excluded from the GroupNorm statistics, zero on the way out.  ``xs``: x's
        split planes when its producer wrote them (only passed when they are valid for ``lens``).  GroupNorm writes
        the second conv's operand as planes directly, and with ``want_split`` the closing LayerNorm also writes the
        output's planes for the next split GEMM.  Returns (y, planes or None)."""
        B, T, _ = x.shape
        c = self.ctx
        if lens is not None and xs is None:
            ops.mask_rows(x, lens)
        if xs is None and (c.use_split(self.w1s) or c.use_split(self.scs)):
            xs = c.split(x)
        h = torch.empty((B, T, self.hid), dtype=torch.float32, device=x.device)
        c.conv(x, xs, self.w1, self.w1s, h, M=T, N=self.hid, K=3 * self.cin, Zb=B, sAb=T * self.cin, ldx=self.cin,
               stride=1, pad=1, Cg=self.cin, Tin=T, sCb=T * self.hid, ldc=self.hid)
        hs = None
        if c.use_split(self.w2s):        # GN(16) + Hardswish straight to the planes of the second conv's operand
            hs = ops.groupnorm(h, self.n_groups, self.gn[0], self.gn[1], 1e-5, act=ops.ACT_HARDSWISH, out=False,
                               t_len=lens, out_split=True, flag=c.flag)
        else:
            h = ops.groupnorm(h, self.n_groups, self.gn[0], self.gn[1], 1e-5, act=ops.ACT_HARDSWISH, out=h, t_len=lens)
        sc = x if self.sc is None else c.linear(x, xs, self.sc, self.scs)[0]
        y = torch.empty((B, T, self.cout), dtype=torch.float32, device=x.device)
        c.conv(h, hs, self.w2, self.w2s, y, M=T, N=self.cout, K=3 * self.hid, Zb=B, sAb=T * self.hid, ldx=self.hid,
               stride=1, pad=1, Cg=self.hid, Tin=T, R=sc, sRb=T * self.cout, ldr=self.cout, sCb=T * self.cout,
               ldc=self.cout)
        if want_split and c.precision == "split":
            return ops.layernorm(y, self.ln[0], self.ln[1], 1e-5, act=ops.ACT_HARDSWISH, out=y, t_len=lens,
                                 out_split=True, flag=c.flag)
        return ops.layernorm(y, self.ln[0], self.ln[1], 1e-5, act=ops.ACT_HARDSWISH, out=y, t_len=lens), None


class _Down:
    def __init__(self, sd, pre, dev, ctx):
        w = _t(sd[pre + "conv.weight"]).float()       # [Cout, Cin, f]
        self.cout, self.cin, self.f = w.shape
        self.w = w.permute(0, 2, 1).reshape(self.cout, -1).contiguous().to(dev)
        self.b = _t(sd[pre + "conv.bias"]).float().contiguous().to(dev)
        self.ctx = ctx
        self.ws = ctx.planes(self.w) if self.cin % 32 == 0 else None

    def __call__(self, x, lens=None, xs=None, want_split=False):
        """Stride-f conv (stride_conv.py:23-47).  Its output rows past a shorter row's length are not zero (the
        next block masks them), so output planes (dual epilogue) are written only for a uniform batch."""
        B, T, _ = x.shape
        assert T % self.f == 0, "T is pre-padded to a multiple of factor**times (unet.py:103-106)"
        To = T // self.f
        y = torch.empty((B, To, self.cout), dtype=torch.float32, device=x.device)
        ys = self.ctx.planes_for(y) if (want_split and lens is None and self.ctx.use_split(self.ws)) else None
        return self.ctx.conv(x, xs, self.w, self.ws, y, out_s=ys, M=To, N=self.cout, K=self.f * self.cin, Zb=B,
                             sAb=T * self.cin, ldx=self.cin, stride=self.f, Cg=self.cin, Tin=T, bias=self.b,
                             sCb=To * self.cout, ldc=self.cout)


class _Up:
    def __init__(self, sd, pre, dev, ctx):
        w = _t(sd[pre + "conv.weight"]).float()       # ConvTranspose1d: [Cin, Cout, f]
        self.cin, self.cout, self.f = w.shape
        # out[f*t + j, o] = sum_c x[t, c] w[c, o, j] + b[o]  ->  W'[(j, o), c]
        self.w = w.permute(2, 1, 0).reshape(self.f * self.cout, self.cin).contiguous().to(dev)
        b = _t(sd[pre + "conv.bias"]).float()
        self.b = b.repeat(self.f).contiguous().to(dev)
        self.ctx = ctx
        self.ws = ctx.planes(self.w)

    def __call__(self, x, lens=None, xs=None, want_split=False, skip=None):
        """Transposed conv as one GEMM; ``skip`` (the UNet's skip connection, [B, f T, Cout]) is added in the
        epilogue (the same f32 sum as a separate add), and for a uniform batch the sum's planes are written too."""
        B, T, _ = x.shape
        dual = want_split and lens is None and self.ctx.use_split(self.ws)
        r = skip.view(B, T, self.f * self.cout) if skip is not None else None
        y, ys = self.ctx.linear(x, xs, self.w, self.ws, self.b, residual=r, dual=dual)
        return y.view(B, T * self.f, self.cout), (ys.view(2, B, T * self.f, self.cout) if ys is not None else None)


class LatticeHead:
    """UNet backbone + linear head: features [B, T_pad, C_in] -> logits [B, T_pad, V+2]."""

    def __init__(self, arch: UNetArch, state_dict: dict, device="cuda", precision: str = "split"):
        if precision not in ("split", "f32"):
            raise ValueError(f"precision must be 'split' or 'f32', not {precision!r}")
        dev = torch.device(device)
        self.arch = arch
        self.ctx = c = _Ctx(dev, precision)
        sd = {k[len("backbone."):] if k.startswith("backbone.") else k: v for k, v in state_dict.items()}
        self.divisible = arch.factor ** arch.times
        self.encoders = [[_Block(sd, "encoders.0.", dev, c)]]
        for i in range(1, arch.times):
            self.encoders.append([_Down(sd, f"encoders.{i}.0.", dev, c), _Block(sd, f"encoders.{i}.1.", dev, c)])
        self.bottleneck = [_Down(sd, "bottle_neck.0.", dev, c), _Block(sd, "bottle_neck.1.", dev, c),
                           _Up(sd, "bottle_neck.2.", dev, c)]
        self.decoders = []
        for i in range(arch.times - 1):
            self.decoders.append([_Block(sd, f"decoders.{i}.0.", dev, c), _Up(sd, f"decoders.{i}.1.", dev, c)])
        self.decoders.append([_Block(sd, f"decoders.{arch.times - 1}.", dev, c)])
        self.head_w = _t(sd["head.weight"]).float().contiguous().to(dev)
        self.head_b = _t(sd["head.bias"]).float().contiguous().to(dev)
        # split path: the head's rows padded with zeros to a multiple of 4 (the split GEMM's f32 C rows are 16-B
        # aligned); its logits are the leading V+2 columns of the padded output (a strided view)
        n, n4 = self.head_w.shape[0], -(-self.head_w.shape[0] // 4) * 4
        self.head_wp = torch.zeros((n4, self.head_w.shape[1]), dtype=torch.float32, device=dev)
        self.head_wp[:n] = self.head_w
        self.head_bp = torch.zeros(n4, dtype=torch.float32, device=dev)
        self.head_bp[:n] = self.head_b
        self.head_ws = c.planes(self.head_wp)
        self.vocab_size = self.head_w.shape[0] - 2

    @property
    def precision(self) -> str:
        return self.ctx.precision

    @precision.setter
    def precision(self, value: str):
        self.ctx.precision = value

    @property
    def flag(self):
        """Device int32 [1]: raised when a split operand of this head left f16 range (see task._guard)."""
        return self.ctx.flag

    def padded_len(self, T: int) -> int:
        r = T % self.divisible
        return T if r == 0 else T + self.divisible - r

    @torch.no_grad()
    def backbone(self, x: torch.Tensor, t_pad=None, want_split=False):
        """x [B, T_pad, C_in] with T_pad % factor**times == 0 (zero rows beyond the real T).  ``t_pad`` (optional
        host ints [B]): each row's own padded length (a multiple of factor**times) in a variable-length batch; the
        reference runs each utterance alone at that length (unet.py:103-106), so every level masks beyond it.
        Split path: every producer whose consumer is a split GEMM writes that operand's planes (block GroupNorm and
        LayerNorm, down / up convs with the skip add in their epilogue), so no separate conversion runs beyond the
        input's.  Returns y, or (y, planes) with ``want_split``."""
        lv = None
        if t_pad is not None and any(int(t) != x.shape[1] for t in t_pad):
            from .hubert import dev_lengths
            lv = [dev_lengths([int(t) // self.arch.factor ** i for t in t_pad], x.device)
                  for i in range(self.arch.times + 1)]
        L = (lambda i: None) if lv is None else (lambda i: lv[i])
        n_enc = len(self.encoders)
        h = [(x, None)]
        for i, enc in enumerate(self.encoders):
            t = h[-1]
            for m in enc:
                t = m(t[0], L(i), xs=t[1], want_split=True)
            h.append(t)
        bd, bb, bu = self.bottleneck
        t = bd(h[-1][0], L(self.arch.times), xs=h[-1][1], want_split=True)
        t = bb(t[0], L(self.arch.times), xs=t[1], want_split=True)
        t = bu(t[0], L(self.arch.times), xs=t[1], want_split=True, skip=h[n_enc][0])
        for i, dec in enumerate(self.decoders):
            lev = self.arch.times - 1 - i
            last = i + 1 == len(self.decoders)
            t = dec[0](t[0], L(lev), xs=t[1], want_split=want_split if last else True)
            if len(dec) > 1:
                t = dec[1](t[0], L(lev), xs=t[1], want_split=True, skip=h[n_enc - 1 - i][0])
        return t if want_split else t[0]

    @torch.no_grad()
    def logits(self, x: torch.Tensor, t_pad=None) -> torch.Tensor:
        """x [B, T_pad, C_in] -> logits [B, T_pad, V+2] on the chip-wide launches (every GEMM spreads over the whole
        chip; a row's result depends on its own length only).  The one-kernel and per-op-engine forms of round 3
        were parity-green but slower in the pipeline; they are in git history."""
        if self.ctx.use_split(self.head_ws):
            y, ys = self.backbone(x, t_pad, want_split=True)
            return self.ctx.linear(y, ys, self.head_wp, self.head_ws, self.head_bp)[0][:, :, :self.head_w.shape[0]]
        y = self.backbone(x, t_pad)
        return self.ctx.linear(y, None, self.head_w, None, self.head_b)[0]

    @staticmethod
    def split(logits: torch.Tensor):
        """(ph_frame_logits, ph_edge_logits, ctc_logits) views, forced_alignment.py:287-292."""
        # (basic slicing only: a list index would upload an index tensor through a synchronising pageable copy)
        return logits[:, :, 2:], logits[:, :, 0], torch.cat([logits[:, :, 1:2], logits[:, :, 3:]], dim=-1)

    def flops(self, T_pad: int) -> float:
        a = self.arch
        f = 0.0

        def blk(T, ci, co):
            hid = max(16 * (co // 16), 16)
            return 2.0 * T * (3 * ci * hid + 3 * hid * co + (ci * co if ci != co else 0))
        T = T_pad
        f += blk(T, a.input_dims, a.hidden_dims)
        for i in range(1, a.times):
            T //= a.factor
            f += 2.0 * T * a.ch(i - 1) * a.ch(i) * a.factor + blk(T, a.ch(i), a.ch(i))
        Tb = T // a.factor
        f += 2.0 * Tb * a.ch(a.times - 1) * a.ch(a.times) * a.factor + blk(Tb, a.ch(a.times), a.ch(a.times))
        f += 2.0 * Tb * a.ch(a.times) * a.ch(a.times - 1) * a.factor
        for i in range(1, a.times):
            f += blk(T, a.ch(a.times - i), a.ch(a.times - i)) + 2.0 * T * a.ch(a.times - i) * a.ch(a.times - i - 1) * a.factor
            T *= a.factor
        f += blk(T, a.hidden_dims, a.output_dims)
        f += 2.0 * T * a.output_dims * (a.vocab_size + 2)
        return f
