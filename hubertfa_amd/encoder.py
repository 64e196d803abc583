"""Drop-in ``UnitsEncoder`` (reference: tools/encoder.py:10-60) on the HIP Hubert encoders.

``UnitsEncoder(encoder, encoder_ckpt, encoder_sample_rate=16000, encoder_hop_size=320, device=None)`` and
``.encode(audio[B, N], sample_rate, hop_size) -> [B, C, T]`` keep the reference signature and semantics:
  1. resample ``sample_rate -> encoder_sample_rate`` with a 128-wide sinc (encoder.py:41-48),
  2. the <400-sample pad applied to the ORIGINAL audio, exactly as the reference does (encoder.py:51-52),
  3. the model ('cnhubert' = HF HubertModel folder, 'hubertsoft' = bshall .pt; encoder.py:17-22),
  4. nearest-index gather onto the hop grid (encoder.py:55-59).
``encode_frames`` returns the channels-last, zero-padded [B, T_pad, C] tensor the lattice head consumes, which
saves the reference's transpose round trip.

Model locations: a HF folder (config.json, model.safetensors | pytorch_model.bin, preprocessor_config.json),
a bshall checkpoint (``torch.load(path)["hubert"]``), or ``synth:<seed>`` for seeded synthetic weights.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import ops, synth
from .hubert import HubertEncoder
from .hubert import dev_lengths
from .resample import Resampler, target_length


def _g(gate) -> dict:
    """The encoder's ``gate`` keyword, only when one is set."""
    return {} if gate is None else {"gate": gate}


def _load_tensors(path: str) -> dict:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def arch_from_hf_config(cfg: dict, do_normalize: bool) -> synth.HubertArch:
    if cfg.get("hidden_act", "gelu") != "gelu" or cfg.get("feat_extract_activation", "gelu") != "gelu":
        raise ValueError("only erf-GELU Hubert configs are supported")
    if cfg.get("conv_pos_batch_norm", False):
        raise ValueError("conv_pos_batch_norm Hubert variants are not supported")
    return synth.HubertArch(
        layout="hf", hidden=cfg.get("hidden_size", 768), layers=cfg.get("num_hidden_layers", 12),
        heads=cfg.get("num_attention_heads", 12), ffn=cfg.get("intermediate_size", 3072),
        conv_dim=tuple(cfg.get("conv_dim", (512,) * 7)), conv_kernel=tuple(cfg.get("conv_kernel", (10, 3, 3, 3, 3, 2, 2))),
        conv_stride=tuple(cfg.get("conv_stride", (5, 2, 2, 2, 2, 2, 2))),
        feat_extract_norm=cfg.get("feat_extract_norm", "group"), conv_bias=cfg.get("conv_bias", False),
        stable_layer_norm=cfg.get("do_stable_layer_norm", False),
        pos_kernel=cfg.get("num_conv_pos_embeddings", 128), pos_groups=cfg.get("num_conv_pos_embedding_groups", 16),
        layer_norm_eps=cfg.get("layer_norm_eps", 1e-5), do_normalize=do_normalize)


def load_hubert(encoder: str, encoder_ckpt: str, device) -> HubertEncoder:
    """Build a HIP Hubert from the reference's encoder name + checkpoint location (encoder.py:17-30)."""
    if encoder_ckpt.startswith("synth:"):
        seed = int(encoder_ckpt.split(":", 1)[1] or 0)
        arch = {"cnhubert": synth.arch_cnhubert_base, "cnhubert-large": synth.arch_cnhubert_large,
                "hubertsoft": synth.arch_hubertsoft}[encoder]()
        return HubertEncoder(arch, synth.synth_hubert_state_dict(arch, seed=seed), device)
    if encoder in ("cnhubert", "cnhubert-large"):
        with open(os.path.join(encoder_ckpt, "config.json")) as f:
            cfg = json.load(f)
        do_norm = True   # Wav2Vec2FeatureExtractor default
        pp = os.path.join(encoder_ckpt, "preprocessor_config.json")
        if os.path.exists(pp):
            with open(pp) as f:
                do_norm = bool(json.load(f).get("do_normalize", True))
        for name in ("model.safetensors", "pytorch_model.bin"):
            p = os.path.join(encoder_ckpt, name)
            if os.path.exists(p):
                return HubertEncoder(arch_from_hf_config(cfg, do_norm), _load_tensors(p), device)
        raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin in {encoder_ckpt}")
    if encoder == "hubertsoft":
        ckpt = _load_tensors(encoder_ckpt)
        return HubertEncoder(synth.arch_hubertsoft(), ckpt["hubert"] if "hubert" in ckpt else ckpt, device)
    raise ValueError(f" [x] Unknown units encoder: {encoder}")


def plan_windows(L: int, C: int, O: int):
    """Long-form windows over L Hubert frames: (core_lo, core_hi, win_lo, win_hi) per window, cores C frames
    tiling [0, L) in order, each window its core plus up to O frames of context on either side."""
    out = []
    for k in range(-(-L // C)):
        out.append((k * C, min(L, (k + 1) * C), max(0, k * C - O), min(L, (k + 1) * C + O)))
    return out


def window_samples(a: int, b: int, hop: int = 320, rf: int = 400, pad: int = 0) -> int:
    """Samples whose extractor output is exactly frames [a, b) (frame j covers [hop j - pad, hop j + rf - pad))."""
    return hop * (b - a - 1) + rf - 2 * pad


class UnitsEncoder:
    def __init__(self, encoder, encoder_ckpt, encoder_sample_rate=16000, encoder_hop_size=320, device=None):
        if device is None:
            device = "cuda"
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("hubertfa_amd runs on the GPU only (no CPU fallback)")
        self.model = load_hubert(encoder, encoder_ckpt, self.device)
        self.resample_kernel = {}
        self.encoder_sample_rate = encoder_sample_rate
        self.encoder_hop_size = encoder_hop_size

    def _resample(self, audio, sample_rate):
        if sample_rate == self.encoder_sample_rate:
            return audio
        key = str(sample_rate)
        if key not in self.resample_kernel:
            self.resample_kernel[key] = Resampler(sample_rate, self.encoder_sample_rate, 128, self.device)
        return self.resample_kernel[key](audio, split=self.split_resample)

    @property
    def split_resample(self) -> bool:
        """Resample on the split-f16 GEMM while the encoder runs split (the range guard's f32 re-run: f32 GEMM)."""
        return getattr(self.model, "precision", "f32") == "split"

    def grid(self, n_samples: int, sample_rate: int, hop_size: int):
        n_frames = n_samples // hop_size + 1
        ratio = (hop_size / sample_rate) / (self.encoder_hop_size / self.encoder_sample_rate)
        return n_frames, ratio

    def resampled_lengths(self, lengths, sample_rate: int):
        """Per-row sample counts after resampling to the encoder rate (torchaudio: ceil(new * n / orig))."""
        return [target_length(int(n), sample_rate, self.encoder_sample_rate) for n in lengths]

    @torch.no_grad()
    def units(self, audio: torch.Tensor, sample_rate: int, lengths=None, gate=None, resampled=None) -> torch.Tensor:
        """[B, N] -> units [B, L, C].  ``lengths``: per-row sample counts of a zero-padded variable-length batch
        (every row's units then equal what that utterance gives alone).  ``resampled``: the batch already at the
        encoder rate (task.encode_batch's one-pass chain from the input rate; ``audio`` is then unused)."""
        if resampled is not None:
            audio_res = resampled
        else:
            audio = audio.to(self.device).float()
            if audio.dim() == 1:
                audio = audio[None]
            audio_res = self._resample(audio, sample_rate)
        if lengths is None:
            if audio_res.size(-1) < 400:   # reference pads the ORIGINAL audio here (encoder.py:51-52)
                if resampled is not None:
                    raise ValueError("units: the padding quirk needs the wave at sample_rate (resampled too short)")
                audio_res = torch.nn.functional.pad(audio, (0, 400 - audio_res.size(-1)))
            return self.model(audio_res, **_g(gate))   # rows with a pitch are fine (conv0 / normalise: row strides)
        lens16 = self.resampled_lengths(lengths, sample_rate)
        if min(lens16) < 400:
            raise ValueError("utterances shorter than 400 encoder samples take the reference's padding quirk "
                             "(encoder.py:51-52) and must be aligned alone")
        audio_res = audio_res.contiguous()
        if any(n != audio_res.shape[-1] for n in lens16):   # the resampler's sinc tails spill past each row's end
            ops.mask_rows(audio_res, dev_lengths(lens16, audio_res.device))
        return self.model(audio_res, lengths=lens16, **_g(gate))

    @torch.no_grad()
    def units_chunked(self, audio: torch.Tensor, chunk_frames: int, overlap_frames: int, gate=None) -> torch.Tensor:
        """Long-form units of ONE utterance [1, N] at the encoder rate from overlapping windows (BASELINE config 5).

        Window k covers global Hubert frames [kC - O, (k+1)C + O) (C = chunk_frames, O = overlap_frames, clipped
        to [0, L)); frame j of the utterance covers samples [320 j - pad, 320 j + 400 - pad) (pad = the layout's
        wave padding), so a window is the sample span of its frames and yields exactly its frame count.  All
        windows run as ONE variable-length batch (every GEMM and attention launch covers all of them) and the
        core frames [kC, (k+1)C) of each are stitched back in order.  Attention then costs O(L (C + 2O)) instead of
        O(L^2); the price is context: each frame sees its window only, and conv0's GroupNorm statistics are per
        window (the wave normalisation keeps whole-utterance statistics).  The reference has no chunking — the unchunked path stays the parity anchor."""
        m = self.model
        hop, rf, pad = 320, 400, m.arch.wav_pad
        x = audio.to(self.device).float().reshape(1, -1)
        N = x.shape[-1]
        L = m.frame_lengths(N)
        C, O = int(chunk_frames), int(overlap_frames)
        if L <= C + O:
            return m(x.contiguous(), **_g(gate))
        if m.arch.do_normalize:          # whole-utterance statistics (Wav2Vec2FeatureExtractor), not per window
            x = ops.wav_normalize(x.contiguous(), 1e-7)
        wins = plan_windows(L, C, O)
        n_win = [window_samples(a, b, hop, rf, pad) for _, _, a, b in wins]
        xs = x[0]
        batch = torch.zeros((len(wins), max(n_win)), dtype=torch.float32, device=x.device)
        for i, (_, _, a, b) in enumerate(wins):
            s0 = hop * a - pad
            lo, hi = max(0, s0), min(N, s0 + n_win[i])
            if hi > lo:
                batch[i, lo - s0:hi - s0] = xs[lo:hi]
        units = m(batch, lengths=n_win, normalized=True, **_g(gate))  # [K, Wmax, C]
        idx = np.concatenate([i * units.shape[1] + np.arange(c0 - a, c1 - a) for i, (c0, c1, a, _) in
                              enumerate(wins)])
        flat = units.reshape(-1, units.shape[-1])
        take = torch.from_numpy(idx.astype(np.int64)).pin_memory().to(x.device, non_blocking=True)
        return flat.index_select(0, take)[None]

    @torch.no_grad()
    def encode_frames(self, audio: torch.Tensor | None, sample_rate: int, hop_size: int, pad_to: int = 1,
                      lengths=None, chunk_frames: int | None = None, overlap_frames: int = 100, gate=None,
                      resampled: tuple | None = None):
        """[B, N] -> (features [B, T_pad, C] channels-last, n_frames); rows >= n_frames are zero.

        With ``lengths`` (per-row sample counts of a zero-padded batch) n_frames is a list (one per row) and
        rows >= n_frames[b] of row b are zero; T_pad covers the longest row.  ``gate``: called before each
        attention launch (HubertEncoder.attention_block).  ``resampled`` = (the batch at the encoder rate, N at
        ``sample_rate``): the wave at ``sample_rate`` was never formed (task.encode_batch's one-pass chain), only
        its length, which the frame grid takes (encoder.py:56-57)."""
        enc = None if resampled is None else resampled[0]
        n_in = audio.shape[-1] if resampled is None else int(resampled[1])
        rows = audio.shape[0] if resampled is None else enc.shape[0]
        if chunk_frames is not None and lengths is None and rows == 1:
            audio_res = self._resample(audio.to(self.device).float(), sample_rate) if enc is None else enc
            units = self.units_chunked(audio_res.contiguous(), chunk_frames, overlap_frames, gate=gate)
        else:
            units = self.units(audio, sample_rate, lengths, gate=gate, resampled=enc)
        if lengths is None:
            n_frames, ratio = self.grid(n_in, sample_rate, hop_size)
            T_pad = (n_frames + pad_to - 1) // pad_to * pad_to
            return ops.units_gather(units.contiguous(), n_frames, T_pad, ratio), n_frames
        nfs = [self.grid(int(n), sample_rate, hop_size)[0] for n in lengths]
        _, ratio = self.grid(int(lengths[0]), sample_rate, hop_size)
        Ls = [self.model.frame_lengths(n) for n in self.resampled_lengths(lengths, sample_rate)]
        T_pad = (max(nfs) + pad_to - 1) // pad_to * pad_to
        dev = units.device
        feats = ops.units_gather(units.contiguous(), max(nfs), T_pad, ratio, n_frames_b=dev_lengths(nfs, dev),
                                 U_b=dev_lengths(Ls, dev))
        return feats, nfs

    def encode(self, audio, sample_rate, hop_size):
        """[B, N] -> [B, C, T] like the reference; under the split-f16 range guard (a batch whose activations
        leave f16 range is recomputed on the f32 GEMMs)."""
        from .task import guarded
        feats, n = guarded(self.model, ops.split_flag(self.device),
                           lambda: self.encode_frames(audio, sample_rate, hop_size))
        return feats[:, :n].transpose(1, 2)
