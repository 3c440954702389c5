"""The device assembly code (i-emic_amd/csrc/stencil.h), run on the CPU by the emulation
harness, against the oracle: bit-exact Jacobian (Epetra-shaped CSR on the maximal graph),
mass diagonal B and residual F.  The same templates are compiled into the HIP kernels;
tests/test_gpu_parity.py repeats the comparison on the device.
"""
import numpy as np
import pytest

from helpers import golden, golden_landm, manifest, mask_fix
from iemic import config as cf

SMALL = ["test6x6x4", "natl8", "2dmoc", "2dmoc_run", "gateway16"]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


@pytest.mark.parametrize("name", SMALL + ["global4"])
@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_emulated_assembly_bitexact(oracle_lib, emul, name, kind):
    c = cf.preset(name, mixing=0)
    L = golden_landm(name)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    e = emul(c, L)
    x = np.zeros(c.nrows) if kind == "zero" else cf.synthetic_state(c, L)
    rowptr, col, val, B = e.jacobian_csr(x)
    ov, oB = o.jacobian(x)
    np.testing.assert_array_equal(rowptr, o.rowptr)
    np.testing.assert_array_equal(col, o.col)
    np.testing.assert_array_equal(val, ov)          # -0.0 == 0.0 allowed (explicit zeros)
    np.testing.assert_array_equal(bits(B), bits(oB))
    F = e.rhs(x)
    oF = o.rhs(x)
    ri = o.rowintcon
    if ri >= 0:   # the integral condition is a reduction: summation order differs
        assert abs(F[ri] - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
        F[ri] = oF[ri]
    np.testing.assert_array_equal(bits(F), bits(oF))


@pytest.mark.parametrize("name", ["test6x6x4", "natl8", "2dmoc"])
def test_oracle_graph_equals_placed_fortran(oracle_lib, name):
    """THCM.C:1074-1173 placement: oracle J == golden Fortran CSR placed in the max graph."""
    c = cf.preset(name, mixing=0)
    g = golden(name)
    L = golden_landm(name)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L)
    ref = oracle_lib.fortran_to_graph(o.rowptr, o.col, g["synthetic_beg"], g["synthetic_jco"],
                                      g["synthetic_co"], o.rowintcon)
    val, B = o.jacobian(x)
    ri = o.rowintcon
    keep = np.ones(len(val), bool)
    if ri >= 0:
        keep[o.rowptr[ri]:o.rowptr[ri + 1]] = False
        ic = o.intcond_coeff()
        np.testing.assert_array_equal(val[~keep], c.int_sign * ic[o.col[~keep]])
    np.testing.assert_array_equal(val[keep], ref[keep])
    F = o.rhs(x)
    Bref = g["synthetic_B"]
    Fref = -Bref
    if ri >= 0:
        Fref[ri] = F[ri]
    np.testing.assert_array_equal(F, Fref)
    np.testing.assert_array_equal(B, np.where(np.arange(c.nrows) == ri, 0.0, g["synthetic_coB"]))


@pytest.mark.parametrize("name", ["natl8", "gateway16"])
def test_mask_fix_restatement(oracle_lib, name):
    """analyzeJacobian1 fix-up cycle converges (Ocean.C:273-333, 519)."""
    c = cf.preset(name, mixing=0)
    L = mask_fix(oracle_lib, c, golden_landm(name))
    L2 = mask_fix(oracle_lib, c, L, max_fix=1)
    np.testing.assert_array_equal(L, L2)
