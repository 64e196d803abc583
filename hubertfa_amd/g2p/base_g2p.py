"""``BaseG2P`` (reference: networks/g2p/base_g2p.py:19-65).

Contract kept: ``__call__`` checks that the phone sequence starts and ends with ``SP`` and never has two ``SP`` in
a row (AssertionError otherwise); ``get_dataset`` pairs every ``*.wav`` with its ``.<in_format>`` transcript,
silently drops files that fail (the reference swallows the exception), prints ``Loaded N samples.`` and returns an
indexable dataset of ``(wav_path, ph_seq, word_seq, ph_idx_to_word_idx)`` tuples.
"""
from __future__ import annotations

import pathlib


class AlignmentDataset:
    """Indexable (wav_path, ph_seq, word_seq, ph_idx_to_word_idx) rows (stands in for DataFrameDataset)."""

    def __init__(self, rows):
        self.rows = list(rows)

    def __getitem__(self, index):
        return tuple(self.rows[index])

    def __len__(self):
        return len(self.rows)

    def __iter__(self):
        return (tuple(r) for r in self.rows)


class BaseG2P:
    def __init__(self, **kwargs):
        self.in_format = "lab"

    def _g2p(self, input_text):
        """text -> (ph_seq, word_seq, ph_idx_to_word_idx); -1 marks an SP phone."""
        raise NotImplementedError

    def __call__(self, text):
        ph_seq, word_seq, ph_idx_to_word_idx = self._g2p(text)
        assert ph_seq[0] == "SP" and ph_seq[-1] == "SP"
        assert all(not (a == "SP" and b == "SP") for a, b in zip(ph_seq[:-1], ph_seq[1:]))
        return ph_seq, word_seq, ph_idx_to_word_idx

    def set_in_format(self, in_format):
        self.in_format = in_format

    def get_dataset(self, wav_paths):
        rows = []
        fmt = getattr(self, "in_format", "lab")
        for wav_path in wav_paths:
            wav_path = pathlib.Path(wav_path)
            try:
                lab_path = wav_path.with_suffix("." + fmt)
                if not lab_path.exists():
                    continue
                text = lab_path.read_text(encoding="utf-8").strip()
                rows.append((wav_path, *self(text)))
            except Exception as e:  # noqa: BLE001 — per-file failures are dropped, as the reference does
                e.args = (f" Error when processing {wav_path}: {e} ",)
        print(f"Loaded {len(rows)} samples.")
        return AlignmentDataset(rows)
