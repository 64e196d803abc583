"""The C-ABI library loads on a CPU-only host and exports every symbol include/hfa.h declares."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "hfa.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(hfa_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert "hfa_viterbi_forward" in names and "hfa_last_error" in names
    assert len(names) >= 6


def test_library_exports_every_declared_symbol():
    from hubertfa_amd import _lib, ops  # noqa: F401  (ops registers the encoder signatures)
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhfa.so not built (run __graft_entry__.build())")
    L = _lib.lib()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    assert L.hfa_build_arch() == b"gfx950"
    # every declared symbol has a Python signature, so no entry point is called untyped
    assert not [n for n in _declared() if n not in _lib._SIGS]


def test_ops_refuse_cpu_tensors():
    import torch
    from hubertfa_amd import ops, _lib
    x = torch.zeros(1, 4, 4)
    with pytest.raises(_lib.HFALibraryError):
        ops.viterbi_backtrack(x, x.to(torch.int8), torch.zeros(1, 4, dtype=torch.int32),
                              torch.ones(1, dtype=torch.int32), torch.ones(1, dtype=torch.int32))
