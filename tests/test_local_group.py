"""The in-process rank group (i-emic_amd/csrc/local_group.h, the transport of the in-process
multi-rank tests and of scripts/band_iters.py) under the host sanitizers: the library's own
header is built into tests/emul/local_group_stress.cpp with ThreadSanitizer (clang's runtime:
GCC 11's libtsan does not intercept pthread_cond_clockwait and reports a false double lock)
and with AddressSanitizer, and 8 host threads drive all-reduces of varying length, halo
batches over the mailbox, and the release of the group while contexts are still attached
(the last context to leave deletes it).  Any race, use after free or wrong result fails."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "emul", "local_group_stress.cpp")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def _build_run(tmp_path, cxx, san, extra_env):
    exe = str(tmp_path / f"lg_{san}")
    subprocess.run([cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-o", exe, SRC, "-lpthread"],
                   check=True)
    env = dict(os.environ, **extra_env)
    r = subprocess.run([exe, "8", "300", "3"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr
    assert "local group stress ok" in r.stdout


@pytest.mark.skipif(not os.path.exists(CLANG), reason="clang++ of the ROCm LLVM not present")
def test_local_group_thread_sanitizer(tmp_path):
    _build_run(tmp_path, CLANG, "thread", {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not present")
def test_local_group_address_sanitizer(tmp_path):
    _build_run(tmp_path, "g++", "address", {"ASAN_OPTIONS": "detect_leaks=1"})
