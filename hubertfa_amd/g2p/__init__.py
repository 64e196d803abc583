"""G2P plugins with the reference's plugin API (networks/g2p/__init__.py): ``<Name>G2P(**cli_kwargs)``
subclassing ``BaseG2P`` and implementing ``_g2p(text) -> (ph_seq, word_seq, ph_idx_to_word_idx)``."""
from .base_g2p import BaseG2P, AlignmentDataset
from .dictionary_g2p import DictionaryG2P
from .none_g2p import NoneG2P
from .phoneme_g2p import PhonemeG2P

__all__ = ["BaseG2P", "AlignmentDataset", "DictionaryG2P", "NoneG2P", "PhonemeG2P"]
