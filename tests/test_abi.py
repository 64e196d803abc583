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


def test_no_packed_f32_in_device_code():
    """libhfa carries no packed-f32 VALU (v_pk_fma/mul/add_f32): on MI355X their results came out wrong in groups
    of lanes, now and then, while MFMA waves of another kernel shared the CU.  The Makefile builds
    with the packed-fp32-ops target feature off; this checks the shipped code objects."""
    import re
    import shutil
    import subprocess
    import tempfile
    from hubertfa_amd._lib import LIB_PATH
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(LIB_PATH) or not shutil.which(f"{llvm}/llvm-objcopy"):
        pytest.skip("library or llvm tools absent")
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB_PATH, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        offs = [m.start() for m in re.finditer(re.escape(magic), data)]
        assert offs, "no offload bundles in libhfa.so"
        n_mfma = 0
        for i, o in enumerate(offs):
            part = os.path.join(td, f"b{i}.bin")
            co = os.path.join(td, f"b{i}.co")
            open(part, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
            subprocess.run([f"{llvm}/clang-offload-bundler", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
            dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                                 text=True, check=True).stdout
            bad = re.findall(r"v_pk_\w*f32", dis)
            assert not bad, f"bundle {i}: {len(bad)} packed-f32 instructions, e.g. {bad[0]}"
            n_mfma += dis.count("v_mfma")
        assert n_mfma > 0, "disassembly found no MFMA: extraction failed"


def test_split_gemm_tile_choice():
    """The split GEMM's automatic tile for the workload's large grids (host query, no GPU): 256 x 256 unless a
    192-wide tile fills the last round of CUs much better (profiles/r03/split_tiles_c5.txt)."""
    pytest.importorskip("torch")
    from hubertfa_amd import ops
    tile = lambda M, N, Z=1, epi=0, K=768: ops._split_name(M, N, K, Z, True, epi, 768).split("<")[1].split(",")[1:3]  # noqa: E731
    assert tile(15968, 2304) == [" 192", " 256"]          # config 2 QKV: 567 big tiles = 2.2 rounds
    assert tile(15968, 3072, epi=1) == [" 256", " 256"]   # config 2 FFN1: 756 tiles = 2.95 rounds
    assert tile(17924, 3072, epi=1) == [" 256", " 256"]   # config 5 windows: 852 tiles (was 128 x 128)
    assert tile(17924, 2304) == [" 256", " 256"]          # 639 tiles (was 128 x 128)
    assert tile(15968, 768, K=3072) == [" 192", " 256"]   # FFN2: one round of 252 tiles (not 189)
    assert tile(15968, 768) == [" 128", " 192"]           # out-projection (K = 768): 500 tiles, two per CU
    assert tile(17924, 768) == [" 256", " 256"]           # config 5 windows: 192 x 256 would take a second round
    assert tile(15999, 512, Z=32, epi=1) == [" 256", " 256"]   # extractor conv1
    assert tile(499, 512, Z=32, epi=1) == [" 128", " 128"]     # extractor conv6: 128 big tiles, half a round
    # narrow N (profiles/r05/side_tiles.txt, gemm.hip split_cfg): the UNet's 192-channel convs / linears at K <= 1152
    # on exact 64-wide tiles; wider K keeps 128 x 128; the 44.1 k -> 16 k resampler's N = 160 on one 192-wide column
    # tile; unmeasured widths (N = 320) keep 128 x 128
    assert tile(864, 192, Z=32) == [" 128", " 64"]        # UNet level 0 (K = 768)
    assert tile(864, 192, Z=32, K=1536) == [" 128", " 128"]
    assert tile(1000, 160, Z=256, K=1184) == [" 128", " 192"]   # resampler 44.1 k -> 16 k: 8 groups x 32 rows
    assert tile(864, 320, Z=32) == [" 128", " 128"]
    # the grouped positional conv (Cg = 48, k = 128): the LDS-window kernel, named as launched (the K argument)
    assert ops._split_name(499, 48, 6144, 512, False, 1, 48) == "posconv_split_kernel<1, 3, 4>"   # 512-row tiles
    assert ops._split_name(200, 48, 6144, 512, False, 1, 48) == "posconv_split_kernel<1, 3, 2>"
    assert ops._split_name(499, 64, 8192, 512, False, 1, 64) == "posconv_split_kernel<1, 4, 2>"   # Hubert-large


def test_abi_version_and_host_queries():
    """The library reports the C-ABI version the binding is written for (hfa_lattice_prologue gained dp /
    curr, hfa_gemm_split_kernel_name gained K, the UNet exports went: version 2), the DP's range limit comes from the
    library (alignment_decoder asks it), and the split tile override refuses the retired tuning-only tiles."""
    from hubertfa_amd import _lib, ops  # noqa: F401
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhfa.so not built")
    L = _lib.lib()
    assert L.hfa_abi_version() == _lib.ABI_VERSION == 2
    hdr = open(os.path.join(REPO, "include", "hfa.h")).read()
    assert re.search(r"#define HFA_ABI_VERSION 2\b", hdr)
    assert L.hfa_viterbi_range_max_states() == 8192
    for cfg in (1, 7, 11, 14, 21, 22, 26, 27, -1):
        assert L.hfa_gemm_split_tuning(cfg) == _lib.HFA_EINVAL, cfg
    for cfg in (15, 16, 17, 18, 19, 20, 23, 24, 25, 0):
        assert L.hfa_gemm_split_tuning(cfg) == 0, cfg
    # the name query answers from the built tiles only (every one a single-accumulator 16x16x32 tile)
    for M, N in ((15968, 2304), (15968, 768), (499, 512), (864, 192), (15968, 3072)):
        assert ops._split_name(M, N, 768, 1, True, 1, 768).endswith(", true, 32, 16, false>")
