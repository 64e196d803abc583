"""ctypes binding of libhfa.so, the C-ABI of hand-written gfx950 kernels (include/hfa.h).

The product path has no fallback: if the library is missing or fails to load, every op raises
``HFALibraryError``.  Signatures are declared once in ``_SIGS``; ``check(rc)`` turns a negative status into an
exception carrying ``hfa_last_error()``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HFA_LIB", os.path.join(_HERE, "_build", "libhfa.so"))

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS = {
    "hfa_last_error": [],
    "hfa_abi_version": [],
    "hfa_build_arch": [],
    # alignment decoder (viterbi.hip)
    "hfa_viterbi_forward": [I, I, I, P, P, P, P, P, P, P, P, P, P, P],
    "hfa_viterbi_forward_steps": [I, I, I, P, P, P, P, P, P, P, P, P, P, I, I, P],
    "hfa_viterbi_backtrack": [I, I, I, P, P, P, P, P, P, P, P, P, P],
    "hfa_lattice_prologue": [I, I, I, I, P, P, P, LL, LL, P, LL, LL, P, P, P, P, P, P, P, P, P, P, P],
    "hfa_viterbi_init": [I, I, I, P, P, P, P, P, P, P],
    "hfa_viterbi_tuning": [I],
    "hfa_viterbi_range_max_states": [],
    # WAV front end (wav.cpp, host memory)
    "hfa_wav_info": [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32),
                     ctypes.POINTER(ctypes.c_int32)],
    "hfa_wav_read": [ctypes.c_char_p, ctypes.c_int32, P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                     ctypes.POINTER(ctypes.c_int32)],
}
_RESTYPE = {"hfa_last_error": ctypes.c_char_p, "hfa_build_arch": ctypes.c_char_p}


HFA_EINVAL = -1000
ABI_VERSION = 2          # include/hfa.h HFA_ABI_VERSION: the argument lists _SIGS and the kernel modules declare


class HFALibraryError(RuntimeError):
    """A libhfa failure; ``rc`` is the status (HFA_EINVAL for a bad argument, -(hipError_t) for a HIP error, None
    when the library itself is missing)."""

    def __init__(self, msg: str, rc: int | None = None):
        super().__init__(msg)
        self.rc = rc


class HFAArgumentError(HFALibraryError, ValueError):
    """rc == HFA_EINVAL: the call's arguments (one input's shape, a file's contents) were rejected before anything
    ran on the device, so the device is still healthy and the caller may go on with other inputs."""


_lib = None


def register(name: str, argtypes: list, restype=ctypes.c_int):
    """Kernel modules declare their entry points here before first use."""
    _SIGS[name] = argtypes
    if restype is not ctypes.c_int:
        _RESTYPE[name] = restype
    if _lib is not None:
        _bind(_lib, name)


_missing = set()


def _bind(L, name):
    # a symbol this library build lacks (an older build under A/B timing) fails loudly when called, not at load;
    # tests/test_abi.py holds the shipped build to every symbol include/hfa.h declares
    try:
        fn = getattr(L, name)
    except AttributeError:
        _missing.add(name)
        return
    fn.argtypes = _SIGS[name]
    fn.restype = _RESTYPE.get(name, ctypes.c_int)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HFALibraryError(
                f"libhfa.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (make -C hubertfa_amd/csrc). There is no CPU fallback.")
        try:
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise HFALibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name in _SIGS:
            _bind(L, name)
        got = L.hfa_abi_version()
        if got != ABI_VERSION:       # an older / newer build: its argument lists differ
            raise HFALibraryError(f"{LIB_PATH} has C-ABI version {got}, this binding is written for {ABI_VERSION}: "
                                  f"rebuild it (make -C hubertfa_amd/csrc)")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().hfa_last_error()
        cls = HFAArgumentError if rc == HFA_EINVAL else HFALibraryError
        raise cls(f"{what or 'libhfa'} failed (rc={rc}): {msg.decode() if msg else ''}", rc)


def call(name: str, *args) -> None:
    L = lib()
    if name in _missing:
        raise HFALibraryError(f"{LIB_PATH} does not export {name}")
    check(getattr(L, name)(*args), name)
