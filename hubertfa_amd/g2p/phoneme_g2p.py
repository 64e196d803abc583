"""``PhonemeG2P`` (reference: networks/g2p/phoneme_g2p.py:4-18): every non-SP token is a one-phone word,
separated by SP."""
from __future__ import annotations

from .base_g2p import BaseG2P


class PhonemeG2P(BaseG2P):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    def _g2p(self, input_text):
        words = [t for t in input_text.strip().split(" ") if t != "SP"]
        ph_seq, p2w = ["SP"], [-1]
        for i, w in enumerate(words):
            ph_seq += [w, "SP"]
            p2w += [i, -1]
        return ph_seq, words, p2w
