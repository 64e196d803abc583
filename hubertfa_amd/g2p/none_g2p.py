"""``NoneG2P`` (reference: networks/g2p/none_g2p.py:6-24): the text already is the phone sequence; repeated SP
collapses, SP framing is added; every phone is its own word."""
from __future__ import annotations

import numpy as np

from .base_g2p import BaseG2P


class NoneG2P(BaseG2P):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    def _g2p(self, input_text):
        ph_seq = ["SP"]
        for tok in input_text.strip().split(" "):
            if not (tok == "SP" and ph_seq[-1] == "SP"):
                ph_seq.append(tok)
        if ph_seq[-1] != "SP":
            ph_seq.append("SP")
        return ph_seq, ph_seq, np.arange(len(ph_seq))
