"""The C-ABI drop-in library: builds, loads and exports every entry point of
include/iemic.h; without a GPU it refuses loudly (no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from iemic import _lib, config as cf

HEADER = os.path.join(ROOT, "include", "iemic.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(iemic_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "i-emic_amd"), "-j8"], check=True,
                   stdout=subprocess.DEVNULL)
    return _lib.lib()


def test_header_declares_binding(built):
    assert header_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_all_symbols(built):
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], check=True,
                        capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (iemic_\w+)", nm))
    missing = set(header_symbols()) - exported
    assert not missing, missing


def test_gfx950_code_object(built):
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layout_matches_header(built):
    """ctypes mirrors of iemic_grid / iemic_krylov / info structs have the C sizes."""
    src = r'''
#include <stdio.h>
#include "iemic.h"
int main(void){printf("%zu %zu %zu %zu\n", sizeof(iemic_grid), sizeof(iemic_krylov),
 sizeof(iemic_solve_info), sizeof(iemic_newton_info)); return 0;}
'''
    tmp = os.path.join(ROOT, "tests", "_build")
    os.makedirs(tmp, exist_ok=True)
    cfile = os.path.join(tmp, "sizes.c")
    exe = os.path.join(tmp, "sizes")
    with open(cfile, "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), cfile, "-o", exe], check=True)
    got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == [C.sizeof(_lib.Grid), C.sizeof(_lib.Krylov), C.sizeof(_lib.SolveInfo),
                   C.sizeof(_lib.NewtonInfo)]


def test_no_gpu_fails_loudly(built):
    if built.iemic_device_count() > 0:
        pytest.skip("a GPU is present")
    from iemic.ocean import Ocean
    c = cf.preset("test6x6x4", mixing=0)
    with pytest.raises(_lib.IemicError, match="no HIP device"):
        Ocean(c)


@pytest.mark.gpu
def test_unrestated_mixing_rejected(built):
    """Mixing parameters outside the restated vmix_fun subset (here MIXP != 0: neutral
    physics) are refused loudly, not silently ignored."""
    if built.iemic_device_count() <= 0:
        pytest.skip("needs a device to reach the configuration check")
    from iemic.ocean import Ocean
    c = cf.preset("test6x6x4", mixing=1)
    oc = Ocean(c)
    oc.setPar("MIXP", 1.0)
    with pytest.raises(_lib.IemicError, match="neutral physics"):
        oc.computeRHS()


@pytest.mark.gpu
def test_device_vectors_outlive_close(built):
    """Ocean.close() with DeviceVecs still alive (a continuation's saved state, say): the
    pool is freed at once, the context stays valid for the live vectors and is destroyed
    when the last one is released, so no device buffer leaks and none is freed twice."""
    from iemic.ocean import Ocean
    c = cf.preset("test6x6x4", mixing=0)
    oc = Ocean(c)
    ops = oc.vec_ops()
    oc.setState(cf.synthetic_state(c, oc.landmask().reshape(c.l + 2, c.m + 2, c.n + 2), amp_ts=1e-3))
    a = ops.state()
    b = ops.copy(a)
    del b                                       # back into the pool
    assert len(oc._vpool) == 1 and oc._vlive == 1
    oc.close()
    assert oc._vpool == [] and oc._h is not None
    assert ops.dot(a, a) > 0.0                  # the context still serves the live vector
    del a
    assert oc._h is None
    with pytest.raises(_lib.IemicError):
        ops.state()
