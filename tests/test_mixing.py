"""Vertical mixing (Mixing = 1 / 2; mix_imp.f vmix_fun / vmix_jac).

* The oracle's restatement against the reference's own Fortran output with mixing
  (tests/golden/make_golden_mix.py): Fortran CSR (beg/jco/co incl. the coloured
  forward-difference mixing entries), coB and rhs B bit-exact (SHA-256), on test6x6x4,
  natl8 (Mixing = 1), gateway16 (Mixing = 2, synthetic state and the reference's fixture
  state ocean_reference.h5) and global 4 deg.
* The device assembly code (stencil.h) run on the CPU by the emulation harness against the
  oracle: J and F bit-exact (the harness uses the host libm tanh, like the oracle).
* On the GPU (through the C ABI): J columns identical and values / F within the
  tolerance of the device tanh (the forward difference divides a libm-level difference of
  tanh values by eps = 1e-8), and a Newton step with mixing.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN
from iemic import config as cf

with open(os.path.join(GOLDEN, "manifest_mix.json")) as _f:
    MANM = json.load(_f)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def h5_state():
    from helpers import golden
    return golden("gateway16")["h5_x"]


def setup(oracle_lib, name, kind="synthetic"):
    c = cf.preset(name, mixing=MANM[name]["mixing"] if name in MANM else 1)
    L = cf.init_landmask(c, cf.landmask(c))
    x = h5_state() if kind == "h5" else cf.synthetic_state(c, cf.landmask(c))
    return c, L, x


CASES = [(n, s) for n in MANM for s in MANM[n]["states"]]


@pytest.mark.parametrize("name,kind", CASES)
def test_oracle_mixing_matches_fortran(oracle_lib, name, kind):
    c, L, x = setup(oracle_lib, name, kind)
    ent = MANM[name]["states"][kind]
    assert sha(L.reshape(-1).astype(np.int32)) == MANM[name]["landm_sha"]
    assert sha(x) == ent["x_sha"]
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    beg, jco, co, coB = o.fortran_matrix(x)
    B = o.fortran_rhs(x)
    assert len(co) == ent["nnz"]
    assert sha(beg) == ent["beg_sha"]
    assert sha(jco) == ent["jco_sha"]
    assert sha(co) == ent["co_sha"]
    assert sha(coB) == ent["coB_sha"]
    assert sha(B) == ent["B_sha"]


def test_mixing_changes_the_operator(oracle_lib):
    """Sanity: with Mixing the T/S rows differ from the Mixing = 0 operator."""
    c, L, x = setup(oracle_lib, "natl8")
    o1 = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    c0 = c.with_(mixing=0)
    o0 = oracle_lib.Oracle(c0.ref_dict(), L, c0.par_list())
    v1, _ = o1.jacobian(x)
    v0, _ = o0.jacobian(x)
    assert np.count_nonzero(v1 != v0) > 100
    assert np.max(np.abs(o1.rhs(x) - o0.rhs(x))) > 1.0


@pytest.mark.parametrize("name", ["test6x6x4", "natl8", "gateway16"])
def test_emulated_mixing_bitexact(oracle_lib, emul, name):
    c, L, x = setup(oracle_lib, name)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    e = emul(c, L)
    rowptr, col, val, B = e.jacobian_csr(x)
    ov, oB = o.jacobian(x)
    np.testing.assert_array_equal(rowptr, o.rowptr)
    np.testing.assert_array_equal(col, o.col)
    np.testing.assert_array_equal(val, ov)
    F, oF = e.rhs(x), o.rhs(x)
    ri = o.rowintcon
    if ri >= 0:
        assert abs(F[ri] - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
        F[ri] = oF[ri]
    np.testing.assert_array_equal(bits(F), bits(oF))


def test_mixing2_first_evaluation_decides(oracle_lib, emul):
    """Mixing = 2: a zero T field at the first evaluation switches mixing off for good
    (vmix_control sets vmix_fix), as in the reference."""
    c, L, x = setup(oracle_lib, "gateway16")
    c0 = c.with_(mixing=0)
    o2 = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    o0 = oracle_lib.Oracle(c0.ref_dict(), L, c0.par_list())
    o2.rhs(np.zeros(c.nrows))
    np.testing.assert_array_equal(o2.rhs(x), o0.rhs(x))
    e = emul(c, L)
    e.rhs(np.zeros(c.nrows))
    np.testing.assert_array_equal(e.rhs(x), o0.rhs(x))


def test_device_tanh_is_host_libm():
    """stencil.h's libm_tanh (the device mixing's tanh) equals the host C library's tanh bit
    for bit: random arguments over [2^-60, 2^7] of both signs, the branch points of tanh
    and expm1, and the specials."""
    import ctypes as C
    from helpers import emul_lib
    lib = emul_lib()
    lib.emul_tanh.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_long]
    rng = np.random.default_rng(11)
    e = rng.integers(-60, 8, 400_000)
    x = np.ldexp(1.0 + rng.random(e.size), e) * rng.choice([-1.0, 1.0], e.size)
    edges = np.array([0.0, -0.0, 2.0 ** -55, 2.0 ** -54, 0.5 * np.log(2), 1.5 * np.log(2), 0.25,
                      0.5, 1.0, 22.0, 28.0, 56 * np.log(2) / 2, 709.78 / 2, np.inf, -np.inf])
    x = np.concatenate([x, edges, -edges, np.nextafter(edges, 0), np.nextafter(edges, np.inf)])
    x = np.ascontiguousarray(x[np.isfinite(x) | np.isinf(x)])
    y = np.zeros_like(x)
    lib.emul_tanh(x.ctypes.data_as(C.POINTER(C.c_double)), y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    import math                         # the C library's tanh (numpy has its own SIMD one)
    ref = np.array([math.tanh(v) for v in x.tolist()])
    np.testing.assert_array_equal(y.view(np.int64), ref.view(np.int64))


# ---- GPU ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["test6x6x4", "natl8", "gateway16", "global4", "global2"])
def test_gpu_mixing_parity(oracle_lib, name):
    """Mixing = 1 (the benchmark's physics): the device J and F equal the oracle's bit for
    bit, the forward-difference mixing entries included (libm_tanh in stencil.h is the
    host libm's tanh), up to the 2-degree bench size."""
    from iemic.ocean import Ocean
    c, L, x = setup(oracle_lib, name)
    # analyze_jacobian off: the mask-fix cycle evaluates the zero state, which would fix
    # Mixing = 2 off before x is seen (the golden landm is already the fixed one here)
    oc = Ocean(c, landm=L, analyze_jacobian=False)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    oc.setState(x)
    F = oc.computeRHS()
    oc.computeJacobian()
    rowptr, col, val = oc.exportCSR()
    ov, _ = o.jacobian(x)
    oF = o.rhs(x)
    np.testing.assert_array_equal(rowptr, o.rowptr)
    np.testing.assert_array_equal(col, o.col)
    np.testing.assert_array_equal(val.view(np.int64), ov.view(np.int64))
    # the integral-condition entry (SRES = 0) is a global dot product: summation order
    ric = oc.rowintcon
    keep = np.ones(c.nrows, bool)
    if ric >= 0:
        keep[ric] = False
        assert abs(F[ric] - oF[ric]) <= 1e-13 * max(abs(oF[ric]), np.max(np.abs(oF)))
    np.testing.assert_array_equal(F[keep].view(np.int64), oF[keep].view(np.int64))


@pytest.mark.gpu
def test_gpu_mixing_newton_step(oracle_lib):
    from iemic.ocean import Ocean
    c, L, _ = setup(oracle_lib, "global4")
    x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
    oc = Ocean(c, landm=L, analyze_jacobian=False,
               solver_params={"FGMRES tolerance": 1e-8, "FGMRES iterations": 200,
                              "FGMRES restarts": 10})
    oc.setState(x)
    info = oc.newtonStep()
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    f0 = np.linalg.norm(o.rhs(x))
    assert abs(info.norm_f0 - f0) <= 1e-10 * f0
    assert info.solve.converged == 1
    ov, _ = o.jacobian(x)
    lin = np.linalg.norm(o.rhs(x) + o.spmv(ov, oc.getState() - x)) / f0
    assert lin <= 1e-8, lin
