"""TEST INFRASTRUCTURE: rebuilds the checkpoint files the reference's loaders read, from the seeded synthetic
weights (hubertfa_amd.synth), so the same files exist here (where tests/golden/gen_golden.py loads them through
the reference) and on the GPU box (where the product's loaders read them).  Base-size conv stacks are ~17 MB of
f32 per file, which is why the files are rebuilt instead of committed; what the reference computed from them is
committed (tests/golden/loaders.npz / loaders.json).

Layouts (the reference call sites that read them):
  * HF folder — HubertModel.from_pretrained / Wav2Vec2FeatureExtractor.from_pretrained (tools/encoder.py:86-89):
      "hf"        model.safetensors written by HubertModel.save_pretrained (weight norm as a parametrization),
                  preprocessor_config.json do_normalize=true;
      "hf_nonorm" the same with do_normalize=false;
      "hf_legacy" pytorch_model.bin in the older layout: weight_g / weight_v names under a "hubert." prefix (what
                  a HubertForCTC / HubertForPreTraining export holds), plus a config.json.
  * bshall .pt — torch.load(path)["hubert"] with DataParallel's "module." prefix (tools/encoder.py:69-71).
  * Lightning .ckpt — state_dict (backbone.*, head.*, and every loss module's buffers) + hyper_parameters
    (networks/task/forced_alignment.py:36 save_hyperparameters; infer.py:59 load_from_checkpoint).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from hubertfa_amd import synth

HF_KINDS = ("hf", "hf_nonorm", "hf_legacy")
LOADER_LAYERS = 2
HF_SEED, SOFT_SEED, CKPT_SEED = 31, 32, 33


def loader_arch(kind: str):
    if kind == "soft":
        return synth.arch_hubertsoft()               # HubertSoft() has a fixed 12-layer encoder
    return synth.arch_cnhubert_base(layers=LOADER_LAYERS, do_normalize=kind != "hf_nonorm")


def hf_config(arch):
    from transformers import HubertConfig
    cfg = HubertConfig(hidden_size=arch.hidden, num_hidden_layers=arch.layers, num_attention_heads=arch.heads,
                       intermediate_size=arch.ffn, feat_extract_norm=arch.feat_extract_norm,
                       do_stable_layer_norm=arch.stable_layer_norm, conv_bias=arch.conv_bias)
    cfg._attn_implementation = "eager"
    return cfg


def hf_state_dict(sd, prefix: str = "", legacy: bool = False) -> dict:
    """synth's HF-named weights -> HubertModel's parametrized names, or (``legacy``) weight_g / weight_v under
    ``prefix``."""
    out = {}
    for k, v in sd.items():
        if not legacy:
            k = k.replace("pos_conv_embed.conv.weight_g", "pos_conv_embed.conv.parametrizations.weight.original0")
            k = k.replace("pos_conv_embed.conv.weight_v", "pos_conv_embed.conv.parametrizations.weight.original1")
        out[prefix + k] = torch.from_numpy(np.ascontiguousarray(v))
    return out


def save_hf_folder(path: str, arch, sd, do_normalize: bool = True, legacy: bool = False, prefix: str = "") -> None:
    """config.json + weights + preprocessor_config.json, as the reference's cnhubert adapter expects them."""
    from transformers import HubertModel, Wav2Vec2FeatureExtractor
    os.makedirs(path, exist_ok=True)
    if legacy:
        hf_config(arch).save_pretrained(path)
        torch.save(hf_state_dict(sd, prefix, legacy=True), os.path.join(path, "pytorch_model.bin"))
    else:
        m = HubertModel(hf_config(arch)).eval()
        missing, unexpected = m.load_state_dict(hf_state_dict(sd), strict=False)
        assert not unexpected and not missing, (missing, unexpected)
        m.save_pretrained(path)
    Wav2Vec2FeatureExtractor(feature_size=1, sampling_rate=16000, padding_value=0.0, do_normalize=do_normalize,
                             return_attention_mask=False).save_pretrained(path)


def write_hf_folder(path: str, kind: str) -> None:
    arch = loader_arch(kind)
    sd = synth.synth_hubert_state_dict(arch, seed=HF_SEED)
    save_hf_folder(path, arch, sd, do_normalize=arch.do_normalize, legacy=kind == "hf_legacy",
                   prefix="hubert." if kind == "hf_legacy" else "")


def write_bshall(path: str, arch=None, seed: int = SOFT_SEED) -> None:
    arch = arch or loader_arch("soft")
    sd = synth.synth_hubert_state_dict(arch, seed=seed)
    torch.save({"hubert": {"module." + k: torch.from_numpy(v) for k, v in sd.items()}}, path)


def write_lightning_ckpt(path: str, meta: dict, hubert_model_path: str = "dependencies/cnhubert") -> dict:
    """A .ckpt in Lightning 2.x's layout: the module's state_dict (UNet + head + the loss modules' registered
    buffers, which inference ignores), hyper_parameters as save_hyperparameters() records the __init__ arguments,
    and the trainer bookkeeping Lightning adds (epoch, global_step, loops, callbacks, optimizer and scheduler
    states)."""
    import yaml
    vocab = synth.synth_vocab(62)
    ua = synth.UNetArch(vocab_size=vocab["vocab_size"])
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_unet_state_dict(ua, seed=CKPT_SEED).items()}
    for k, shape in meta["loss_buffers"].items():
        sd[k] = torch.ones(shape)                      # GHM EMA statistics (ones at init)
    hc = dict(meta["hubert_config"], model_path=hubert_model_path)
    hp = {"vocab_text": yaml.safe_dump(vocab), "vowel_text": yaml.safe_dump({"vowel": []}),
          "model_config": dict(meta["model_config"]), "hubert_config": hc,
          "melspec_config": dict(meta["melspec_config"]), "optimizer_config": dict(meta["optimizer_config"]),
          "loss_config": json.loads(json.dumps(meta["loss_config"]))}
    ck = {"epoch": 7, "global_step": 12000, "pytorch-lightning_version": "2.4.0", "state_dict": sd,
          "loops": {"predict_loop": {"state_dict": {}, "batch_progress": {"total": {"ready": 0}}}},
          "callbacks": {"ModelCheckpoint{'monitor': None, 'mode': 'min'}": {"best_model_score": None,
                                                                            "dirpath": "ckpt"}},
          "optimizer_states": [{"state": {0: {"step": torch.tensor(12000.0),
                                              "exp_avg": torch.zeros(4), "exp_avg_sq": torch.zeros(4)}},
                                "param_groups": [{"lr": 1e-3, "weight_decay": 0.1, "params": [0]}]}],
          "lr_schedulers": [{"total_steps": 100000, "last_epoch": 12000, "_step_count": 12001}],
          "hparams_name": "kwargs", "hyper_parameters": hp}
    torch.save(ck, path)
    return ck
