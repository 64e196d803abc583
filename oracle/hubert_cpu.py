"""TEST INFRASTRUCTURE ONLY — torch-CPU fp32 restatement of the float part of the hot path.

Used as the checker for the HIP encoder/UNet at sizes the golden fixtures do not cover (full 10 s utterances,
batches).  Pinned by tests/test_oracle_hubert.py against tests/golden/hubert_*.npz and unet_head.npz, which were
produced by the reference modules themselves (gen_golden.py).

Restates:
  * HF HubertModel forward (transformers modeling_hubert.py: HubertFeatureEncoder, HubertFeatureProjection,
    HubertEncoder / HubertEncoderStableLayerNorm, HubertAttention eager path)
  * bshall HubertSoft.units (networks/hubert/model.py:45-54, 75-79, 95-172)
  * UNetBackbone + head (networks/layer/backbone/unet.py:100-119, resnet_block.py:47-50, stride_conv.py:23-47,
    forced_alignment.py:284-292)
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _sd(sd):
    out = {}
    for k, v in sd.items():
        for pre in ("module.", "hubert."):
            if k.startswith(pre):
                k = k[len(pre):]
        out[k] = torch.from_numpy(np.ascontiguousarray(v)).float() if isinstance(v, np.ndarray) else v.float()
    return out


def _wn(sd, pre):
    if pre + "weight_g" in sd:
        return torch._weight_norm(sd[pre + "weight_v"], sd[pre + "weight_g"], 2)
    return torch._weight_norm(sd[pre + "parametrizations.weight.original1"],
                              sd[pre + "parametrizations.weight.original0"], 2)


def _mha(x, wqkv, bqkv, wo, bo, heads):
    B, L, H = x.shape
    qkv = F.linear(x, wqkv, bqkv)
    q, k, v = qkv.split(H, dim=-1)
    d = H // heads
    q = q.view(B, L, heads, d).transpose(1, 2)
    k = k.view(B, L, heads, d).transpose(1, 2)
    v = v.view(B, L, heads, d).transpose(1, 2)
    a = torch.softmax((q @ k.transpose(-1, -2)) * d ** -0.5, dim=-1) @ v
    return F.linear(a.transpose(1, 2).reshape(B, L, H), wo, bo)


@torch.no_grad()
def hubert_forward(arch, state_dict, wav: torch.Tensor) -> torch.Tensor:
    """wav [B, N] f32 -> units [B, L, C_out] (same semantics as hubertfa_amd.hubert.HubertEncoder)."""
    sd = _sd(state_dict)
    hf = arch.layout == "hf"
    eps = arch.layer_norm_eps
    x = wav.float()
    if arch.do_normalize:
        x = (x - x.mean(-1, keepdim=True)) / torch.sqrt(x.var(-1, unbiased=False, keepdim=True) + 1e-7)
    if arch.wav_pad:
        x = F.pad(x, (arch.wav_pad, arch.wav_pad))
    h = x[:, None]
    for i, (k, s) in enumerate(zip(arch.conv_kernel, arch.conv_stride)):
        pre = f"feature_extractor.conv_layers.{i}." if hf else f"feature_extractor.conv{i}."
        w = sd[pre + "conv.weight"] if hf else sd[pre + "weight"]
        b = sd.get(pre + "conv.bias") if hf else None
        h = F.conv1d(h, w, b, stride=s)
        if hf and arch.feat_extract_norm == "layer":
            h = F.layer_norm(h.transpose(1, 2), (h.shape[1],), sd[pre + "layer_norm.weight"],
                             sd[pre + "layer_norm.bias"], eps).transpose(1, 2)
        elif i == 0:
            g, bb = (sd[pre + "layer_norm.weight"], sd[pre + "layer_norm.bias"]) if hf else \
                (sd["feature_extractor.norm0.weight"], sd["feature_extractor.norm0.bias"])
            h = F.group_norm(h, h.shape[1], g, bb, 1e-5)
        h = F.gelu(h)
    h = h.transpose(1, 2)
    fp = "feature_projection." + ("layer_norm" if hf else "norm")
    h = F.layer_norm(h, (h.shape[-1],), sd[fp + ".weight"], sd[fp + ".bias"], eps)
    h = F.linear(h, sd["feature_projection.projection.weight"], sd["feature_projection.projection.bias"])
    pc = "encoder.pos_conv_embed.conv." if hf else "positional_embedding.conv."
    pos = F.conv1d(h.transpose(1, 2), _wn(sd, pc), sd[pc + "bias"], padding=arch.pos_kernel // 2,
                   groups=arch.pos_groups)
    pos = F.gelu(pos[:, :, :-1]).transpose(1, 2)
    h = h + pos
    enc_ln = ("encoder.layer_norm" if hf else "norm")
    if not arch.stable_layer_norm:
        h = F.layer_norm(h, (h.shape[-1],), sd[enc_ln + ".weight"], sd[enc_ln + ".bias"], eps)
    for l in range(arch.layers):
        p = f"encoder.layers.{l}."
        if hf:
            a = p + "attention."
            wqkv = torch.cat([sd[a + f"{n}_proj.weight"] for n in "qkv"])
            bqkv = torch.cat([sd[a + f"{n}_proj.bias"] for n in "qkv"])
            wo, bo = sd[a + "out_proj.weight"], sd[a + "out_proj.bias"]
            n1, n2 = p + "layer_norm", p + "final_layer_norm"
            w1, b1 = sd[p + "feed_forward.intermediate_dense.weight"], sd[p + "feed_forward.intermediate_dense.bias"]
            w2, b2 = sd[p + "feed_forward.output_dense.weight"], sd[p + "feed_forward.output_dense.bias"]
        else:
            wqkv, bqkv = sd[p + "self_attn.in_proj_weight"], sd[p + "self_attn.in_proj_bias"]
            wo, bo = sd[p + "self_attn.out_proj.weight"], sd[p + "self_attn.out_proj.bias"]
            n1, n2 = p + "norm1", p + "norm2"
            w1, b1, w2, b2 = sd[p + "linear1.weight"], sd[p + "linear1.bias"], sd[p + "linear2.weight"], sd[p + "linear2.bias"]
        ln = lambda t, n: F.layer_norm(t, (t.shape[-1],), sd[n + ".weight"], sd[n + ".bias"], eps)  # noqa: E731
        if not arch.stable_layer_norm:
            h = ln(h + _mha(h, wqkv, bqkv, wo, bo, arch.heads), n1)
            h = ln(h + F.linear(F.gelu(F.linear(h, w1, b1)), w2, b2), n2)
        else:
            h = h + _mha(ln(h, n1), wqkv, bqkv, wo, bo, arch.heads)
            h = h + F.linear(F.gelu(F.linear(ln(h, n2), w1, b1)), w2, b2)
    if arch.stable_layer_norm:
        h = F.layer_norm(h, (h.shape[-1],), sd[enc_ln + ".weight"], sd[enc_ln + ".bias"], eps)
    if not hf and arch.proj_dim:
        h = F.linear(h, sd["proj.weight"], sd["proj.bias"])
    return h


@torch.no_grad()
def unet_head_forward(arch, state_dict, x: torch.Tensor) -> torch.Tensor:
    """x [B, T, C_in] -> logits [B, T, V+2] (UNetBackbone pads T to a multiple of factor**times, crops back)."""
    sd = {k[len("backbone."):] if k.startswith("backbone.") else k: (torch.from_numpy(np.ascontiguousarray(v))
                                                                    if isinstance(v, np.ndarray) else v).float()
          for k, v in state_dict.items()}

    def block(pre, h):
        y = F.conv1d(h.transpose(1, 2), sd[pre + "block.0.weight"], padding=1)
        y = F.hardswish(F.group_norm(y, 16, sd[pre + "block.1.weight"], sd[pre + "block.1.bias"], 1e-5))
        y = F.conv1d(y, sd[pre + "block.3.weight"], padding=1).transpose(1, 2)
        sc = F.linear(h, sd[pre + "shortcut.0.weight"]) if pre + "shortcut.0.weight" in sd else h
        y = y + sc
        return F.hardswish(F.layer_norm(y, (y.shape[-1],), sd[pre + "out.0.weight"], sd[pre + "out.0.bias"], 1e-5))

    def down(pre, h):
        t = h.transpose(1, 2)
        if t.shape[-1] % arch.factor:
            t = F.pad(t, (0, arch.factor - t.shape[-1] % arch.factor))
        return F.conv1d(t, sd[pre + "conv.weight"], sd[pre + "conv.bias"], stride=arch.factor).transpose(1, 2)

    def up(pre, h):
        return F.conv_transpose1d(h.transpose(1, 2), sd[pre + "conv.weight"], sd[pre + "conv.bias"],
                                  stride=arch.factor).transpose(1, 2)

    T = x.shape[1]
    div = arch.factor ** arch.times
    if T % div:
        x = F.pad(x, (0, 0, 0, div - T % div))
    hs = [x, block("encoders.0.", x)]
    for i in range(1, arch.times):
        hs.append(block(f"encoders.{i}.1.", down(f"encoders.{i}.0.", hs[-1])))
    y = up("bottle_neck.2.", block("bottle_neck.1.", down("bottle_neck.0.", hs[-1])))
    for i in range(arch.times - 1):
        y = up(f"decoders.{i}.1.", block(f"decoders.{i}.0.", y + hs[-1 - i]))
    y = block(f"decoders.{arch.times - 1}.", y + hs[1])
    return F.linear(y[:, :T], sd["head.weight"], sd["head.bias"])
