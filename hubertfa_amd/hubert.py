"""Hubert encoders (HF ``HubertModel`` = cnhubert, bshall ``HubertSoft``) executed on libhfa's gfx950 kernels.

Reference arithmetic:
  * HF HubertModel.forward (transformers modeling_hubert.py): HubertFeatureEncoder -> HubertFeatureProjection ->
    HubertEncoder (pos-conv, +x, LN, post-LN layers) or HubertEncoderStableLayerNorm (pre-LN layers, final LN).
  * bshall Hubert.encode / HubertSoft.units (networks/hubert/model.py:45-54, 75-79, 95-172).
  * cnhubert input normalisation (tools/encoder.py:94-95 -> Wav2Vec2FeatureExtractor.zero_mean_unit_var_norm).

Layout: activations are channels-last [B, T, C] f32 in HBM from conv0 onward, so every conv is an implicit GEMM
with overlapping rows (no im2col buffer) and every Linear reads rows directly.  Weights are converted once at
load: conv weights to [Cout][k][Cin] im2col order, Q/K/V fused into one [3H, H] projection, the positional
conv's weight-norm folded (torch._weight_norm, dim=2).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .synth import HubertArch


def _t(x) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    return x.detach().cpu()


def _strip(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        for pre in ("module.", "hubert."):
            if k.startswith(pre):
                k = k[len(pre):]
        out[k] = v
    return out


def _conv_im2col(w: torch.Tensor) -> torch.Tensor:
    """torch conv weight [Cout, Cin, k] -> [Cout, k*Cin] with k-major (matches the GEMM's A addressing)."""
    return w.permute(0, 2, 1).reshape(w.shape[0], -1).contiguous()


def _weight_norm(sd: dict, prefix: str) -> torch.Tensor:
    if prefix + "weight" in sd:
        return _t(sd[prefix + "weight"]).float()
    if prefix + "weight_g" in sd:
        g, v = _t(sd[prefix + "weight_g"]).float(), _t(sd[prefix + "weight_v"]).float()
    else:
        g = _t(sd[prefix + "parametrizations.weight.original0"]).float()
        v = _t(sd[prefix + "parametrizations.weight.original1"]).float()
    return torch._weight_norm(v, g, 2)


class _Layer:
    __slots__ = ("wqkv", "bqkv", "wo", "bo", "ln1_w", "ln1_b", "w1", "b1", "w2", "b2", "ln2_w", "ln2_b",
                 "wqkv_s", "wo_s", "w1_s", "w2_s")


def frame_count(arch: HubertArch, n_samples: int) -> int:
    """Hubert frames of an n-sample input (after the layout's wave padding) through the CNN extractor's valid
    convs (receptive field 400 samples, hop 320 for every layout here)."""
    t = n_samples + 2 * arch.wav_pad
    for k, st in zip(arch.conv_kernel, arch.conv_stride):
        t = (t - k) // st + 1 if t >= k else 0
    return t


def dev_lengths(values, device) -> torch.Tensor:
    """Host ints -> int32 device tensor through pinned memory and a non-blocking copy (a pageable upload would
    synchronise the stream and stall the pipelined host)."""
    return torch.tensor([int(v) for v in values], dtype=torch.int32).pin_memory().to(device, non_blocking=True)


class HubertEncoder:
    """Hubert forward on HIP kernels.  ``forward(wav[B, N]) -> units[B, L, C_out]`` (f32, channels-last).

    ``precision``: "split" (default) evaluates every dense contraction whose channel count allows it (K, Cg
    multiples of 32) on the split-f16 MFMA GEMM (gemm.hip gemm_split_kernel: f32-class accuracy, 2-2.5x the f32
    MFMA rate), the operands carried as f16 plane pairs written directly by their producers; "f32" runs every
    GEMM on the f32 MFMA.  A split producer that meets a value outside f16 range raises ops.split_flag(), and
    the caller re-runs that batch with precision "f32" (task.ForcedAlignmentTask).  "f16" (opt-in fast mode, not
    f32-class): the split path with every split GEMM on the operands' high planes alone, one f16 product per MAC
    (ops.GEMM_F16); attention and the grouped positional conv keep the three products."""

    def __init__(self, arch: HubertArch, state_dict: dict, device: str | torch.device = "cuda",
                 precision: str = "split"):
        if precision not in ("split", "f32", "f16"):
            raise ValueError(f"precision must be 'split', 'f32' or 'f16', not {precision!r}")
        self.arch = arch
        self.f16 = precision == "f16"           # a flag beside precision: the f32 re-run of the range guard
        precision = "split" if self.f16 else precision      # switches precision only
        self.precision = precision
        self.device = torch.device(device)
        sd = _strip(state_dict)
        dev = self.device

        def P(name):
            return _t(sd[name]).float().contiguous().to(dev)

        hf = arch.layout == "hf"
        n_conv = len(arch.conv_dim)
        self.conv_w, self.conv_b, self.conv_ln = [], [], []
        for i in range(n_conv):
            pre = f"feature_extractor.conv_layers.{i}." if hf else f"feature_extractor.conv{i}."
            w = _t(sd[pre + "conv.weight" if hf else pre + "weight"]).float()
            self.conv_w.append((w.reshape(w.shape[0], -1) if i == 0 else _conv_im2col(w)).contiguous().to(dev))
            bkey = pre + ("conv.bias" if hf else "bias")
            self.conv_b.append(P(bkey) if bkey in sd else None)
            if hf and (arch.feat_extract_norm == "layer" or i == 0):
                self.conv_ln.append((P(pre + "layer_norm.weight"), P(pre + "layer_norm.bias")))
            elif not hf and i == 0:
                self.conv_ln.append((P("feature_extractor.norm0.weight"), P("feature_extractor.norm0.bias")))
            else:
                self.conv_ln.append(None)
        fp = "feature_projection."
        self.fp_ln = (P(fp + ("layer_norm" if hf else "norm") + ".weight"), P(fp + ("layer_norm" if hf else "norm") + ".bias"))
        self.fp_w, self.fp_b = P(fp + "projection.weight"), P(fp + "projection.bias")
        pc = "encoder.pos_conv_embed.conv." if hf else "positional_embedding.conv."
        self.pos_w = _conv_im2col(_weight_norm(sd, pc)).to(dev)          # [H, k*H/G] grouped im2col
        self.pos_b = P(pc + "bias")
        self.enc_ln = (P("encoder.layer_norm.weight"), P("encoder.layer_norm.bias")) if hf else \
            (P("norm.weight"), P("norm.bias"))
        self.layers = []
        for l in range(arch.layers):
            L = _Layer()
            p = f"encoder.layers.{l}."
            if hf:
                a = p + "attention."
                L.wqkv = torch.cat([_t(sd[a + f"{n}_proj.weight"]).float() for n in "qkv"], 0).contiguous().to(dev)
                L.bqkv = torch.cat([_t(sd[a + f"{n}_proj.bias"]).float() for n in "qkv"], 0).contiguous().to(dev)
                L.wo, L.bo = P(a + "out_proj.weight"), P(a + "out_proj.bias")
                L.ln1_w, L.ln1_b = P(p + "layer_norm.weight"), P(p + "layer_norm.bias")
                L.w1, L.b1 = P(p + "feed_forward.intermediate_dense.weight"), P(p + "feed_forward.intermediate_dense.bias")
                L.w2, L.b2 = P(p + "feed_forward.output_dense.weight"), P(p + "feed_forward.output_dense.bias")
                L.ln2_w, L.ln2_b = P(p + "final_layer_norm.weight"), P(p + "final_layer_norm.bias")
            else:
                L.wqkv, L.bqkv = P(p + "self_attn.in_proj_weight"), P(p + "self_attn.in_proj_bias")
                L.wo, L.bo = P(p + "self_attn.out_proj.weight"), P(p + "self_attn.out_proj.bias")
                L.ln1_w, L.ln1_b = P(p + "norm1.weight"), P(p + "norm1.bias")
                L.w1, L.b1 = P(p + "linear1.weight"), P(p + "linear1.bias")
                L.w2, L.b2 = P(p + "linear2.weight"), P(p + "linear2.bias")
                L.ln2_w, L.ln2_b = P(p + "norm2.weight"), P(p + "norm2.bias")
            self.layers.append(L)
        self.proj = (P("proj.weight"), P("proj.bias")) if (not hf and arch.proj_dim) else None
        self._ws = {}
        # split-f16 planes of every GEMM weight (one-time); conv weights only where Cin is a multiple of 32
        def sp(w):   # weights with |w| >= 16 (none in practice) stay on the f32 GEMM: the single-accumulator
            # split tile forms 2^11 * hi(w) in f16 (gemm.hip gemm_split_kernel ONE)
            if precision != "split" or self.device.type != "cuda" or not bool(w.abs().max() < 16):
                return None
            return ops.split(w)
        self.conv_ws = [None] + [sp(w) if arch.conv_dim[i - 1] % 32 == 0 else None
                                 for i, w in enumerate(self.conv_w) if i > 0]
        self.fp_ws = sp(self.fp_w) if self.fp_w.shape[1] % 32 == 0 else None
        cg = arch.hidden // arch.pos_groups                  # grouped pos conv: per-lane taps when Cg % 32 != 0
        self.pos_ws = sp(self.pos_w) if (cg % 32 == 0 or (cg % 8 == 0 and cg >= 32)) else None
        for L in self.layers:
            L.wqkv_s, L.wo_s, L.w1_s, L.w2_s = sp(L.wqkv), sp(L.wo), sp(L.w1), sp(L.w2)
        self.proj_s = sp(self.proj[0]) if self.proj is not None else None

    # ----------------------------------------------------------------------------------------------------------
    def _workspace(self, name, nbytes):
        buf = self._ws.get(name)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            self._ws[name] = buf
        return buf

    def frame_lengths(self, n_samples: int) -> int:
        """Hubert frames of an n-sample input (after wav_pad), through the CNN extractor's valid convs."""
        return frame_count(self.arch, n_samples)

    def _split_conv(self, i: int) -> bool:
        return self.precision == "split" and self.conv_ws[i] is not None

    def feature_extractor(self, x: torch.Tensor, t0_len: torch.Tensor | None = None) -> torch.Tensor:
        """[B, N] -> [B, L, 512] (channels-last); GELU applied after every conv.  ``t0_len`` [B] int32: conv0
        frames per row of a variable-length batch (GroupNorm statistics); later convs need no lengths (their
        valid rows only read valid rows).  In split precision a conv whose consumer is a split GEMM writes its
        output as split planes (conv0's apply pass, the GEMM epilogues)."""
        a = self.arch
        B, N = x.shape
        ln0 = self.conv_ln[0]
        n = len(a.conv_dim)
        if a.feat_extract_norm == "group":
            ws = self._workspace("conv0", ops._lib.lib().hfa_conv0_workspace_bytes(B, N))
            h = ops.conv0(x, self.conv_w[0], gamma=ln0[0], beta=ln0[1], eps=1e-5, workspace=ws, t0_len=t0_len,
                          out_split=n > 1 and self._split_conv(1))
        else:
            h = ops.conv0(x, self.conv_w[0], bias=self.conv_b[0])
            if n > 1 and self._split_conv(1):      # LayerNorm + GELU straight to the next conv's split planes
                h = ops.layernorm(h, ln0[0], ln0[1], a.layer_norm_eps, act=ops.ACT_GELU, out=False,
                                  out_split=True)[1]
            else:
                h = ops.layernorm(h, ln0[0], ln0[1], a.layer_norm_eps, act=ops.ACT_GELU, out=h)
        for i in range(1, n):
            k, s = a.conv_kernel[i], a.conv_stride[i]
            split_in = h.dtype == torch.float16
            Tin, Cin = h.shape[-2], h.shape[-1]
            Tout = (Tin - k) // s + 1
            Cout = a.conv_dim[i]
            layer_norm = self.conv_ln[i] is not None
            split_out = split_in and not layer_norm and i + 1 < n and self._split_conv(i + 1)
            out = torch.empty(((2,) if split_out else ()) + (B, Tout, Cout),
                              dtype=torch.float16 if split_out else torch.float32, device=x.device)
            kw = dict(M=Tout, N=Cout, K=k * Cin, Zb=B, sAb=Tin * Cin, ldx=Cin, stride=s, Cg=Cin, Tin=Tin,
                      bias=self.conv_b[i], sCb=Tout * Cout, ldc=Cout,
                      epilogue=ops.EPI_NONE if layer_norm else ops.EPI_GELU)
            if split_in:
                ops.conv_gemm_split(h, self.conv_ws[i], C=None if split_out else out, Cs=out if split_out else None,
                                    f16=self.f16, **kw)
            else:
                ops.conv_gemm(h, self.conv_w[i], out, **kw)
            if layer_norm:
                # (HubertLayerNormConvLayer, Hubert-large) the planes of LayerNorm + GELU written by the LayerNorm
                # itself when a split conv follows -- the same values as splitting its f32 output, without the f32
                # write and the conversion pass (2.1 GB each way at conv0's 32 x 32 000 frames)
                if i + 1 < n and self._split_conv(i + 1):
                    out = ops.layernorm(out, self.conv_ln[i][0], self.conv_ln[i][1], a.layer_norm_eps,
                                        act=ops.ACT_GELU, out=False, out_split=True)[1]
                else:
                    out = ops.layernorm(out, self.conv_ln[i][0], self.conv_ln[i][1], a.layer_norm_eps,
                                        act=ops.ACT_GELU, out=out)
            h = out
        return h

    def _linear(self, x, w, ws, bias=None, residual=None, epilogue=ops.EPI_NONE, out_split=False, xs=None):
        # (xs: x's split planes when its producer wrote them; only read on the split path)
        """Linear on the split GEMM when this encoder runs split and the weight has planes (x given as f32 and/or
        as planes xs), else on the f32 GEMM."""
        if self.precision == "split" and ws is not None:
            if xs is None:
                xs = ops.split(x)
            return ops.linear_split(xs, ws, bias, residual=residual, epilogue=epilogue, out_split=out_split,
                                    f16=self.f16)
        return ops.linear(x, w, bias, residual=residual, epilogue=epilogue)

    def positional(self, h: torch.Tensor, lens: torch.Tensor | None = None, hs: torch.Tensor | None = None
                   ) -> torch.Tensor:
        """h + GELU(grouped conv k128 pad64 (+bias), last frame dropped) — one GEMM launch over (batch, group).
        With ``lens`` the padding rows are zeroed first: the conv's padding must read zeros past each row's end.
        ``hs``: h's split planes when its producer wrote them (uniform batches only)."""
        a = self.arch
        B, L, H = h.shape
        G, k = a.pos_groups, a.pos_kernel
        Cg = H // G
        if lens is not None:
            ops.mask_rows(h, lens)
        out = torch.empty_like(h)
        kw = dict(M=L, N=Cg, K=k * Cg, Zb=B, G=G, sAb=L * H, sAg=Cg, ldx=H, stride=1, pad=k // 2, Cg=Cg, Tin=L,
                  sWg=Cg * k * Cg, bias=self.pos_b, sBg=Cg, R=h, sRb=L * H, sRg=Cg, ldr=H, sCb=L * H, sCg=Cg, ldc=H,
                  epilogue=ops.EPI_GELU)
        if self.precision == "split" and self.pos_ws is not None:
            ops.conv_gemm_split(hs if (hs is not None and lens is None) else ops.split(h), self.pos_ws, C=out,
                                f16=self.f16, **kw)
        else:
            ops.conv_gemm(h, self.pos_w, out, **kw)
        return out

    def attention_block(self, h_in: torch.Tensor, L_: _Layer, lens: torch.Tensor | None = None,
                        hs: torch.Tensor | None = None, gate=None) -> torch.Tensor:
        """softmax(QK^T/sqrt(dh))V over the fused QKV projection.  Split precision: QKV written as split planes,
        attention on the split kernel, O returned as split planes (the out-projection's A operand).  ``gate``
        (optional callable) is called right before the attention launch: its grid runs several rounds, so work
        another stream enqueues there (task.submit: a long lattice's DP range) costs it little, where beside a
        one-round GEMM grid a held CU delays the whole launch."""
        a = self.arch
        B, L, H = (h_in if h_in is not None else hs[0]).shape      # h_in None: the input lives in its planes
        nh = a.heads
        dh = H // nh
        if self.precision == "split" and L_.wqkv_s is not None and L_.wo_s is not None and dh == 64:
            qkv_s = self._linear(h_in, L_.wqkv, L_.wqkv_s, L_.bqkv, out_split=True, xs=hs)
            o_s = torch.empty((2, B, L, H), dtype=torch.float16, device=qkv_s.device)
            if gate is not None:
                gate()
            return ops.attention_split(qkv_s, o_s, B=B, H=nh, L=L, head_dim=dh, scale=dh ** -0.5, key_len=lens)
        qkv = self._linear(h_in, L_.wqkv, L_.wqkv_s, L_.bqkv)
        o = torch.empty((B, L, H), dtype=torch.float32, device=h_in.device)
        if gate is not None:
            gate()
        ops.attention(qkv, qkv[..., H:], qkv[..., 2 * H:], o, B=B, H=nh, L=L, head_dim=dh, scale=dh ** -0.5,
                      q_bs=L * 3 * H, q_ld=3 * H, k_bs=L * 3 * H, k_ld=3 * H, v_bs=L * 3 * H, v_ld=3 * H,
                      o_bs=L * H, o_ld=H, key_len=lens)
        return o

    def _out_proj(self, o: torch.Tensor, L_: _Layer, residual: torch.Tensor) -> torch.Tensor:
        if o.dtype == torch.float16:          # split planes from the split attention
            return self._linear(None, L_.wo, L_.wo_s, L_.bo, residual=residual, xs=o)
        return self._linear(o, L_.wo, L_.wo_s, L_.bo, residual=residual)

    def _ln(self, x, w, b, out=None, split=False, planes_only=False):
        """LayerNorm; with ``split`` (a split GEMM consumes the result) also the split planes, from the same
        kernel: returns (y, planes) — planes None when not requested.  ``planes_only`` (split path): no f32 output
        (y None) — every consumer, residual adds included, reads the planes."""
        eps = self.arch.layer_norm_eps
        if split and self.precision == "split":
            return ops.layernorm(x, w, b, eps, out=False if planes_only else out, out_split=True)
        return ops.layernorm(x, w, b, eps, out=out), None

    def layer(self, h: torch.Tensor, L_: _Layer, lens: torch.Tensor | None = None, hs: torch.Tensor | None = None,
              want_split: bool = False, gate=None):
        """One encoder layer: (h, hs) -> (h', hs').  ``hs``: h's split planes if its producer wrote them;
        ``want_split``: also return the output's planes (the next layer's QKV operand), else None.  ``gate``: see
        attention_block."""
        sp = self.precision == "split" and L_.w1_s is not None and L_.w2_s is not None
        if not self.arch.stable_layer_norm:   # post-LN (HubertEncoderLayer / nn.TransformerEncoderLayer)
            # split path: the residual stream rides in the LayerNorms' split planes (hi + 2^-11 lo, 22 significand
            # bits, the precision every split GEMM operand has): no f32 LayerNorm output is written or read back
            o = self.attention_block(h, L_, lens, hs, gate=gate)
            res = hs if (hs is not None and L_.wo_s is not None and self.precision == "split") else h
            h1 = self._out_proj(o, L_, res)
            h1, h1s = self._ln(h1, L_.ln1_w, L_.ln1_b, out=h1, split=sp, planes_only=sp)
            f = self._linear(h1, L_.w1, L_.w1_s, L_.b1, epilogue=ops.EPI_GELU, out_split=sp, xs=h1s)
            h2 = self._linear(None, L_.w2, L_.w2_s, L_.b2, residual=h1s, xs=f) if sp else \
                ops.linear(f, L_.w2, L_.b2, residual=h1)
            return self._ln(h2, L_.ln2_w, L_.ln2_b, out=h2, split=want_split, planes_only=want_split)
        # pre-LN (HubertEncoderLayerStableLayerNorm): the LayerNorm outputs feed only split GEMMs (planes only);
        # the residual stream is the raw f32 sum
        q_planes = (self.precision == "split" and L_.wqkv_s is not None and L_.wo_s is not None and
                    self.arch.hidden // self.arch.heads == 64)
        a_, a_s = self._ln(h, L_.ln1_w, L_.ln1_b, split=L_.wqkv_s is not None, planes_only=q_planes)
        o = self.attention_block(a_, L_, lens, a_s, gate=gate)
        h = self._out_proj(o, L_, h)
        a_, a_s = self._ln(h, L_.ln2_w, L_.ln2_b, split=sp, planes_only=sp)
        f = self._linear(a_, L_.w1, L_.w1_s, L_.b1, epilogue=ops.EPI_GELU, out_split=sp, xs=a_s)
        if sp:
            return self._linear(None, L_.w2, L_.w2_s, L_.b2, residual=h, xs=f), None
        return ops.linear(f, L_.w2, L_.b2, residual=h), None

    @torch.no_grad()
    def forward(self, wav: torch.Tensor, n_layers: int | None = None, lengths=None,
                normalized: bool = False, gate=None) -> torch.Tensor:
        """wav [B, N] -> units [B, L, C].  ``lengths`` (optional, host ints [B]): samples per row of a
        variable-length batch (rows zero-padded to N); row b's units are valid for frame_lengths(lengths[b])
        frames and equal what that utterance gives alone.  ``normalized``: the caller already applied the
        do_normalize wave statistics (long-form windows of one utterance)."""
        a = self.arch
        x = wav.float()
        if x.dim() == 1:
            x = x[None]
        if x.stride(-1) != 1:          # a row pitch is fine (every first consumer takes a row stride), a gap is not
            x = x.contiguous()
        B, N = x.shape
        if lengths is not None and all(int(n) == N for n in lengths):
            lengths = None
        ns = lens0 = lensL = None
        if lengths is not None:
            ns = dev_lengths(lengths, x.device)
            lens0 = dev_lengths([(int(n) + 2 * a.wav_pad - a.conv_kernel[0]) // a.conv_stride[0] + 1
                                 for n in lengths], x.device)
            lensL = dev_lengths([self.frame_lengths(int(n)) for n in lengths], x.device)
        if a.do_normalize and not normalized:
            x = ops.wav_normalize(x, 1e-7, lens=ns)
        if a.wav_pad:
            x = ops.pad_rows(x, a.wav_pad, x.shape[1] + 2 * a.wav_pad)
        feats = self.feature_extractor(x, lens0)
        fln, flns = self._ln(feats, self.fp_ln[0], self.fp_ln[1], split=self.fp_ws is not None)
        # uniform batch: the projection also writes its output as planes (the positional conv's operand; the f32
        # copy is its residual); a variable-length batch masks the padding rows first, so it splits after that
        dual = lensL is None and self.precision == "split" and self.fp_ws is not None and self.pos_ws is not None
        h = self._linear(fln, self.fp_w, self.fp_ws, self.fp_b, xs=flns, out_split="dual" if dual else False)
        h, hps = h if dual else (h, None)
        h = self.positional(h, lensL, hs=hps)
        hs = None
        layers = self.layers[:n_layers]
        def planes_in(L_):       # a layer that reads its input (QKV operand, out-projection residual) from planes
            return (self.precision == "split" and L_.wqkv_s is not None and L_.wo_s is not None and
                    a.hidden // a.heads == 64)
        if not a.stable_layer_norm:
            first = bool(layers) and planes_in(layers[0])
            h, hs = self._ln(h, self.enc_ln[0], self.enc_ln[1], out=h, split=bool(layers), planes_only=first)
        for i, L_ in enumerate(layers):
            nxt = i + 1 < len(layers)
            h, hs = self.layer(h, L_, lensL, hs, want_split=nxt and (a.stable_layer_norm or planes_in(layers[i + 1])),
                               gate=gate)
        if a.stable_layer_norm:
            h = ops.layernorm(h, self.enc_ln[0], self.enc_ln[1], a.layer_norm_eps, out=h)
        if self.proj is not None:
            h = self._linear(h, self.proj[0], self.proj_s, self.proj[1])
        return h

    __call__ = forward

    def flops(self, n_samples: int) -> float:
        """Algorithmic FLOPs of one forward over ``n_samples`` (MAC = 2 FLOP), excluding norms/activations."""
        a = self.arch
        n = n_samples + 2 * a.wav_pad
        f = 0.0
        T = n
        for i, (cd, k, s) in enumerate(zip(a.conv_dim, a.conv_kernel, a.conv_stride)):
            cin = 1 if i == 0 else a.conv_dim[i - 1]
            T = (T - k) // s + 1
            f += 2.0 * T * cd * cin * k
        L, H = T, a.hidden
        f += 2.0 * L * a.conv_dim[-1] * H                                        # projection
        f += 2.0 * L * H * (H // a.pos_groups) * a.pos_kernel                   # positional conv
        per_layer = 2.0 * L * H * 3 * H + 2.0 * L * H * H + 2.0 * 2 * L * H * a.ffn + 4.0 * L * L * H
        f += a.layers * per_layer
        if a.proj_dim:
            f += 2.0 * L * H * a.proj_dim
        return f
