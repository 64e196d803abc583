"""Deterministic synthetic inputs and weights (numpy PCG64, never torch's init RNG).

No pretrained Hubert weights and no trained HubertFA checkpoint exist offline, so every
parity fixture, test and bench input is generated here.  The same seed regenerates bit-identical arrays on
any host, which is what lets the GPU box rebuild the exact weights the CPU goldens were produced with.

Naming follows the two weight layouts the reference can load:
  * HF ``HubertModel`` (cnhubert, default encoder: tools/encoder.py:81-96, configs/train_config.yaml:22)
  * bshall ``HubertSoft`` (networks/hubert/model.py:18-79, tools/encoder.py:63-78)
and the lattice producer ``LitForcedAlignmentTask.backbone/head`` (networks/task/forced_alignment.py:42-55).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


def rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


# ----------------------------------------------------------------------------------------------------------
# Architecture descriptions
# ----------------------------------------------------------------------------------------------------------
@dataclass
class HubertArch:
    """Geometry of one Hubert encoder variant.

    base  = HF ``HubertConfig()`` defaults (configuration_hubert.py) == bshall arch (model.py:18-36).
    large = feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=True, 24L/1024d/16h/4096.
    """
    layout: str = "hf"                 # "hf" (HubertModel) | "bshall" (HubertSoft)
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    conv_dim: tuple = (512, 512, 512, 512, 512, 512, 512)
    conv_kernel: tuple = (10, 3, 3, 3, 3, 2, 2)
    conv_stride: tuple = (5, 2, 2, 2, 2, 2, 2)
    feat_extract_norm: str = "group"   # "group" (GN on conv0 only) | "layer" (LN after every conv)
    conv_bias: bool = False
    stable_layer_norm: bool = False    # pre-LN layers + final LN (HubertEncoderStableLayerNorm)
    pos_kernel: int = 128
    pos_groups: int = 16
    layer_norm_eps: float = 1e-5
    proj_dim: int | None = None        # bshall HubertSoft.proj 768->256 (model.py:33,79)
    wav_pad: int = 0                   # bshall units() pads 40/40 (model.py:77)
    do_normalize: bool = False         # Wav2Vec2FeatureExtractor zero-mean/unit-var (cnhubert only)

    @property
    def out_channels(self) -> int:
        return self.proj_dim if self.proj_dim else self.hidden

    def n_frames(self, n_samples: int) -> int:
        n = n_samples + 2 * self.wav_pad
        for k, s in zip(self.conv_kernel, self.conv_stride):
            n = (n - k) // s + 1
        return n


def arch_cnhubert_base(layers: int = 12, do_normalize: bool = True) -> HubertArch:
    return HubertArch(layout="hf", layers=layers, do_normalize=do_normalize)


def arch_cnhubert_large(layers: int = 24, do_normalize: bool = True) -> HubertArch:
    return HubertArch(layout="hf", hidden=1024, layers=layers, heads=16, ffn=4096,
                      feat_extract_norm="layer", conv_bias=True, stable_layer_norm=True,
                      do_normalize=do_normalize)


def arch_hubertsoft(layers: int = 12) -> HubertArch:
    return HubertArch(layout="bshall", layers=layers, proj_dim=256, wav_pad=40)


@dataclass
class UNetArch:
    """UNetBackbone geometry (networks/layer/backbone/unet.py:9-98) + head (forced_alignment.py:53-55)."""
    input_dims: int = 768
    hidden_dims: int = 192
    output_dims: int = 192
    factor: int = 2
    times: int = 3
    scaleup: float = 1.3
    n_groups: int = 16
    vocab_size: int = 63

    def ch(self, i: int) -> int:
        return int(self.scaleup ** i) * self.hidden_dims


# ----------------------------------------------------------------------------------------------------------
# Weight generators
# ----------------------------------------------------------------------------------------------------------
class _Gen:
    def __init__(self, seed: int):
        self.r = rng(seed)
        self.sd: dict[str, np.ndarray] = {}

    def normal(self, name, shape, std, mean=0.0):
        self.sd[name] = (mean + std * self.r.standard_normal(shape)).astype(np.float32)

    def uniform(self, name, shape, lo, hi):
        self.sd[name] = self.r.uniform(lo, hi, shape).astype(np.float32)

    def ln(self, prefix, n):
        self.normal(prefix + ".weight", (n,), 0.05, 1.0)
        self.normal(prefix + ".bias", (n,), 0.02)

    def linear(self, prefix, n_out, n_in, bias=True, gain=1.0):
        self.normal(prefix + ".weight", (n_out, n_in), gain / np.sqrt(n_in))
        if bias:
            self.normal(prefix + ".bias", (n_out,), 0.02)

    def conv(self, prefix, c_out, c_in, k, bias, gain=1.0):
        self.normal(prefix + ".weight", (c_out, c_in, k), gain / np.sqrt(c_in * k))
        if bias:
            self.normal(prefix + ".bias", (c_out,), 0.02)


def synth_hubert_state_dict(arch: HubertArch, seed: int = 0) -> dict[str, np.ndarray]:
    """Seeded weights for ``arch`` in the checkpoint naming the reference loads (HF or bshall)."""
    g = _Gen(seed)
    H, C = arch.hidden, arch.conv_dim[-1]
    hf = arch.layout == "hf"
    # 1-D CNN feature extractor
    for i, (cd, k) in enumerate(zip(arch.conv_dim, arch.conv_kernel)):
        c_in = 1 if i == 0 else arch.conv_dim[i - 1]
        gain = 1.0 if i == 0 else 2.0  # keep activations O(1) through GELU
        if hf:
            g.conv(f"feature_extractor.conv_layers.{i}.conv", cd, c_in, k, arch.conv_bias, gain)
            if arch.feat_extract_norm == "layer" or i == 0:
                g.ln(f"feature_extractor.conv_layers.{i}.layer_norm", cd)
        else:
            g.conv(f"feature_extractor.conv{i}", cd, c_in, k, False, gain)
            if i == 0:
                g.ln("feature_extractor.norm0", cd)
    # feature projection
    if hf:
        g.ln("feature_projection.layer_norm", C)
        g.linear("feature_projection.projection", H, C)
    else:
        g.ln("feature_projection.norm", C)
        g.linear("feature_projection.projection", H, C)
    # positional conv embedding (weight-norm over dim=2)
    cg = H // arch.pos_groups
    pre = "encoder.pos_conv_embed.conv" if hf else "positional_embedding.conv"
    g.normal(pre + ".weight_v", (H, cg, arch.pos_kernel), 1.0)
    g.uniform(pre + ".weight_g", (1, 1, arch.pos_kernel), 0.5, 1.5)
    g.normal(pre + ".bias", (H,), 0.02)
    g.ln("encoder.layer_norm" if hf else "norm", H)
    for l in range(arch.layers):
        if hf:
            p = f"encoder.layers.{l}"
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                g.linear(f"{p}.attention.{n}", H, H, gain=1.5 if n in ("q_proj", "k_proj") else 1.0)
            g.ln(f"{p}.layer_norm", H)
            g.linear(f"{p}.feed_forward.intermediate_dense", arch.ffn, H)
            g.linear(f"{p}.feed_forward.output_dense", H, arch.ffn)
            g.ln(f"{p}.final_layer_norm", H)
        else:
            p = f"encoder.layers.{l}"
            g.normal(f"{p}.self_attn.in_proj_weight", (3 * H, H), 1.5 / np.sqrt(H))
            g.normal(f"{p}.self_attn.in_proj_bias", (3 * H,), 0.02)
            g.linear(f"{p}.self_attn.out_proj", H, H)
            g.linear(f"{p}.linear1", arch.ffn, H)
            g.linear(f"{p}.linear2", H, arch.ffn)
            g.ln(f"{p}.norm1", H)
            g.ln(f"{p}.norm2", H)
    if hf:
        g.uniform("masked_spec_embed", (H,), 0.0, 1.0)
    else:
        g.linear("proj", arch.proj_dim or 256, H)
        g.uniform("masked_spec_embed", (H,), 0.0, 1.0)
        g.normal("label_embedding.weight", (100, arch.proj_dim or 256), 1.0)
    return g.sd


def synth_unet_state_dict(arch: UNetArch, seed: int = 1) -> dict[str, np.ndarray]:
    """Seeded ``backbone.*`` + ``head.*`` weights (unet.py:43-98, resnet_block.py:17-50, stride_conv.py)."""
    g = _Gen(seed)

    def block(prefix, c_in, c_out):
        hid = max(arch.n_groups * (c_out // arch.n_groups), arch.n_groups)
        g.conv(prefix + ".block.0", hid, c_in, 3, False, 1.5)
        g.ln(prefix + ".block.1", hid)
        g.conv(prefix + ".block.3", c_out, hid, 3, False, 1.5)
        if c_in != c_out:
            g.linear(prefix + ".shortcut.0", c_out, c_in, bias=False)
        g.ln(prefix + ".out.0", c_out)

    def down(prefix, c_in, c_out):
        g.conv(prefix + ".conv", c_out, c_in, arch.factor, True)

    def up(prefix, c_in, c_out):
        # ConvTranspose1d weight is [C_in, C_out, k]
        g.normal(prefix + ".conv.weight", (c_in, c_out, arch.factor), 1.0 / np.sqrt(c_in))
        g.normal(prefix + ".conv.bias", (c_out,), 0.02)

    b = "backbone."
    block(b + "encoders.0", arch.input_dims, arch.hidden_dims)
    for i in range(1, arch.times):
        down(b + f"encoders.{i}.0", arch.ch(i - 1), arch.ch(i))
        block(b + f"encoders.{i}.1", arch.ch(i), arch.ch(i))
    down(b + "bottle_neck.0", arch.ch(arch.times - 1), arch.ch(arch.times))
    block(b + "bottle_neck.1", arch.ch(arch.times), arch.ch(arch.times))
    up(b + "bottle_neck.2", arch.ch(arch.times), arch.ch(arch.times - 1))
    for i in range(1, arch.times):
        block(b + f"decoders.{i - 1}.0", arch.ch(arch.times - i), arch.ch(arch.times - i))
        up(b + f"decoders.{i - 1}.1", arch.ch(arch.times - i), arch.ch(arch.times - i - 1))
    block(b + f"decoders.{arch.times - 1}", arch.hidden_dims, arch.output_dims)
    g.linear("head", arch.vocab_size + 2, arch.output_dims, gain=3.0)
    return g.sd


# ----------------------------------------------------------------------------------------------------------
# Inputs (SURVEY.md §8d "Synthetic inputs")
# ----------------------------------------------------------------------------------------------------------
def synth_audio(n_samples: int, sr: int = 16000, seed: int = 0) -> np.ndarray:
    """Harmonic stack (f0 ~ U(150,400), 8 partials, amp 0.3) + 0.05 N(0,1), quantised to s16, as f32/32768."""
    r = rng(seed)
    f0 = r.uniform(150.0, 400.0)
    t = np.arange(n_samples, dtype=np.float64) / sr
    x = np.zeros(n_samples, dtype=np.float64)
    for k in range(1, 9):
        x += np.sin(2 * np.pi * f0 * k * t + r.uniform(0, 2 * np.pi)) / k
    x = 0.3 * x / np.max(np.abs(x)) + 0.05 * r.standard_normal(n_samples)
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return q.astype(np.float32) / 32768.0


def synth_phone_set(n_phones: int = 62) -> list[str]:
    """Phone inventory of an opencpop-extension-sized vocab (62 phones + SP -> V=63)."""
    return [f"p{i:02d}" for i in range(n_phones)]


def synth_dictionary(n_words: int = 200, n_phones: int = 62, seed: int = 7) -> dict[str, list[str]]:
    """word -> 1..2 phones, like opencpop-extension (all entries 1-2 phones)."""
    r = rng(seed)
    phones = synth_phone_set(n_phones)
    d = {}
    for w in range(n_words):
        n = 2 if r.uniform() < 0.9 else 1
        d[f"w{w:03d}"] = [phones[int(i)] for i in r.integers(0, n_phones, n)]
    return d


def synth_vocab(n_phones: int = 62) -> dict:
    """Vocab dict in the binarizer's layout (SP=0, binarize.py:64-101)."""
    phones = synth_phone_set(n_phones)
    vocab = {"SP": 0, "AP": 0}
    for i, p in enumerate(phones):
        vocab[p] = i + 1
    return {"vocab": vocab, "vocab_size": n_phones + 1, "ignored_phonemes": ["AP", "SP"]}


def synth_lab(n_words: int, dictionary: dict, seed: int = 0) -> str:
    r = rng(seed)
    words = sorted(dictionary)
    return " ".join(words[int(i)] for i in r.integers(0, len(words), n_words))
