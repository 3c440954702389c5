"""The C++ host class (i-emic_amd/csrc/ocean.hpp, the Ocean-shaped surface a C++ i-emic
build links) driven by tests/cpp/ocean_driver.cpp: builds on the CPU; on the GPU its
residual is bit-identical to the oracle's and its solve satisfies J s = -F."""
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from helpers import golden_landm, mask_fix
from iemic import config as cf

DRIVER = os.path.join(ROOT, "tests", "_build", "ocean_driver")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "i-emic_amd"), "-j8"], check=True,
                   stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True,
                   stdout=subprocess.DEVNULL)
    return DRIVER


def test_driver_builds(driver):
    assert os.access(driver, os.X_OK)


def write_problem(path, c, L, x):
    pars = c.par_list()
    with open(path, "wb") as f:
        f.write(struct.pack("11i", c.n, c.m, c.l, int(c.periodic), c.tres, c.sres,
                            c.forcing_type, c.inhomogeneous_mixing, c.coriolis, c.int_sign,
                            len(pars)))
        f.write(struct.pack("8d", c.xmin, c.xmax, c.ymin, c.ymax, c.hdim, c.qz, c.alpha_t,
                            c.alpha_s))
        for idx, v in pars:
            f.write(struct.pack("=id", idx, v))
        f.write(np.ascontiguousarray(L, dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(x, dtype=np.float64).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["natl8", "gateway16"])
def test_cpp_ocean_newton_solve(oracle_lib, driver, tmp_path, name):
    c = cf.preset(name, mixing=0)
    L0 = golden_landm(name)
    L = mask_fix(oracle_lib, c, L0)
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    inp, out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_problem(inp, c, L0, x)
    p = subprocess.run([driver, inp, out], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    data = np.fromfile(out, dtype=np.float64)
    F, s = data[:c.nrows], data[c.nrows:]
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    oF = o.rhs(x)
    ri = o.rowintcon
    if ri >= 0:
        assert abs(F[ri] - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
        F[ri] = oF[ri]
    np.testing.assert_array_equal(F.view(np.int64), oF.view(np.int64))
    ov, _ = o.jacobian(x)
    res = np.linalg.norm(-oF - o.spmv(ov, s)) / np.linalg.norm(oF)
    assert res <= 1e-7, p.stdout
