"""Host sanitizers (ASan/UBSan on the host code), CPU only.

* The C restatement of the alignment DP (oracle/viterbi_oracle.c), built with -fsanitize=address,undefined and
  driven over random lattices by oracle/oracle_fuzz.c (T = 1, S = 1, T < S, SP framing, ties, -inf holes).
* libhfa's host code (argument validation, plan / kernel-name queries, tuning hooks, error strings) built with
  host-side ASan + UBSan (hubertfa_amd/csrc/Makefile `asan`, device code as shipped) and driven with bad arguments
  through every entry point of include/hfa.h (tests/native/abi_invalid_args.cpp): each must return its error code
  with its own message, and no sanitizer may fire.  GPU AddressSanitizer is not available on the MI355X pool.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def test_oracle_dp_asan_ubsan():
    if shutil.which("gcc") is None:
        pytest.skip("gcc absent")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "sanitize"], check=True)
    p = subprocess.run([os.path.join(REPO, "oracle", "_build", "oracle_fuzz_asan"), "500"], capture_output=True,
                       text=True, env=ENV, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "0 bad" in p.stdout and "ERROR" not in p.stderr


def test_libhfa_host_asan_ubsan_invalid_arguments():
    exe = os.path.join(REPO, "hubertfa_amd", "_build_asan", "abi_invalid_args")
    src = os.path.join(REPO, "tests", "native", "abi_invalid_args.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        if not os.path.exists("/opt/rocm/bin/hipcc"):
            pytest.skip("hipcc absent: the host-sanitizer build is made by __graft_entry__.build()")
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "hubertfa_amd", "csrc"), "asan", "-j8"], check=True,
                       timeout=900)
    p = subprocess.run([exe], capture_output=True, text=True, env=ENV, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert " 0 failures" in p.stdout and "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
