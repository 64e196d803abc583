"""Test helper: the CPU oracle of the whole infer path for one utterance (wave -> decode), and the GPU-side
comparison the parity tests share.

Oracle chain (all under oracle/, test infrastructure only):
  oracle.resample (16k -> 44.1k, width 6; 44.1k -> 16k, width 128)  ~ tools/load_wav.py:7, tools/encoder.py:46-48
  oracle.hubert_cpu.hubert_forward                                   ~ tools/encoder.py:91-96 (HF HubertModel)
  nearest-frame gather                                               ~ tools/encoder.py:55-59
  oracle.hubert_cpu.unet_head_forward                                ~ forced_alignment.py:284-292
  oracle.decode.decode (C Viterbi)                                   ~ tools/alignment_decoder.py:26-143
"""
from __future__ import annotations

import numpy as np
import torch

LOGPROB_TOL = 1e-4          # north star: per-frame log-probs within 1e-4 (fp32)


class OraclePath:
    def __init__(self, ckpt, encoder: str = "cnhubert"):
        import yaml
        from hubertfa_amd import synth
        self.vocab = yaml.safe_load(ckpt["hyper_parameters"]["vocab_text"])
        self.arch = {"cnhubert": synth.arch_cnhubert_base, "cnhubert-large": synth.arch_cnhubert_large,
                     "hubertsoft": synth.arch_hubertsoft}[encoder]()
        self.sd = synth.synth_hubert_state_dict(self.arch, seed=0)        # = load_hubert("synth:0")
        self.ua = synth.UNetArch(input_dims=self.arch.out_channels, vocab_size=self.vocab["vocab_size"])
        self.usd = {k: v.numpy() for k, v in ckpt["state_dict"].items()}

    def units(self, wav16: np.ndarray):
        from oracle import hubert_cpu, resample as ores
        x44 = ores.resample(torch.from_numpy(np.ascontiguousarray(wav16[None], np.float32)), 16000, 44100, 6)
        units = hubert_cpu.hubert_forward(self.arch, self.sd, ores.resample(x44, 44100, 16000, 128))
        return x44.shape[-1], units

    def logits(self, wav16: np.ndarray):
        from oracle import hubert_cpu
        n44, units = self.units(wav16)
        nf = n44 // 512 + 1
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(nf)).long(),
                          max=units.shape[1] - 1)
        return n44, hubert_cpu.unet_head_forward(self.ua, self.usd, units[:, idx])

    def align(self, wav16: np.ndarray, ph_seq, word_seq, p2w):
        """-> (ph_seq, ph_intervals, word_seq, word_intervals, confidence, extras) of oracle.decode.decode."""
        from oracle import decode as odec
        n44, lg = self.logits(wav16)
        return odec.decode(self.vocab, lg[:, :, 2:], lg[:, :, 0], n44 / 44100, ph_seq, word_seq, p2w)

    def check(self, res_b: dict, lattice_b: np.ndarray, wav16, ph_seq, word_seq, p2w, tag: str = "") -> float:
        """Assert one GPU utterance against the oracle: log-probs <= 1e-4, phone path and boundary frames
        bit-exact, words identical, intervals/confidence to f32 round-off.  Returns the log-prob error."""
        ph, ph_iv, w, w_iv, conf, ex = self.align(wav16, ph_seq, word_seq, p2w)
        T = res_b["T"]
        ids = np.array([self.vocab["vocab"][p] for p in ph_seq])
        err = float(np.abs(lattice_b[:T, :len(ids)] - ex["ph_prob_log"][:, ids]).max())
        assert err < LOGPROB_TOL, f"{tag}: per-frame log-prob error {err:.2e} > {LOGPROB_TOL}"
        assert np.array_equal(res_b["ph_idx_seq"], ex["idx"]), f"{tag}: phone path differs"
        assert np.array_equal(res_b["ph_time_int"], ex["tint"]), f"{tag}: boundary frames differ"
        assert list(res_b["ph_seq"]) == list(ph) and list(res_b["word_seq"]) == list(w), f"{tag}: sequences"
        np.testing.assert_allclose(res_b["ph_intervals"], ph_iv, atol=1e-5)
        np.testing.assert_allclose(res_b["word_intervals"], w_iv, atol=1e-5)
        np.testing.assert_allclose(res_b["confidence"], conf, rtol=1e-4)
        return err
