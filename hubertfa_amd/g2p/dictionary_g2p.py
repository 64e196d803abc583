"""``DictionaryG2P`` (reference: networks/g2p/dictionary_g2p.py:6-42).

Dictionary file: one ``word<TAB>ph1 ph2 ...`` entry per line.  Words are split on single spaces; unknown words
are skipped with a warning; an ``SP`` at the first or last position of a word's pronunciation is dropped with a
warning; ``SP`` is inserted after every word unless its pronunciation already ended with one.
"""
from __future__ import annotations

import warnings

from .base_g2p import BaseG2P


class DictionaryG2P(BaseG2P):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        with open(kwargs["dictionary"], "r") as f:
            lines = f.read().strip().split("\n")
        self.dictionary = {}
        for line in lines:
            cols = line.split("\t")
            self.dictionary[cols[0].strip()] = cols[1].strip().split(" ")

    def _g2p(self, input_text):
        ph_seq, p2w, word_seq = ["SP"], [-1], []
        for word in input_text.strip().split(" "):
            phones = self.dictionary.get(word)
            if phones is None:
                warnings.warn(f"Word {word} is not in the dictionary. Ignored.")
                continue
            w_idx = len(word_seq)
            word_seq.append(word)
            last = len(phones) - 1
            for i, ph in enumerate(phones):
                if ph == "SP" and i in (0, last):
                    warnings.warn(f"The first or last phoneme of word {word} is SP, which is not allowed. "
                                  "Please check your dictionary.")
                    continue
                ph_seq.append(ph)
                p2w.append(w_idx)
            if ph_seq[-1] != "SP":
                ph_seq.append("SP")
                p2w.append(-1)
        return ph_seq, word_seq, p2w
