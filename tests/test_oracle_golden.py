"""The oracle (oracle/thcm_oracle.c) against the reference's own Fortran output.

Golden fixtures come from tests/golden/make_golden.py (reference THCM Fortran run in this
container).  Every check is bit-exact: SHA-256 over the float64 bytes of the Fortran CSR
(beg/jco/co in fillcolA order), the mass diagonal coB and rhs B, for the zero state, the
seeded synthetic state and the state of the reference's own fixture
test/ocean/ocean_reference.h5.
"""
import hashlib

import numpy as np
import pytest

from helpers import golden, golden_landm, manifest
from iemic import config as cf

MAN = manifest()
CASES = [(name, st) for name in MAN for st in MAN[name]["states"]]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", list(MAN))
def test_landmask_pipeline(name):
    """config.landmask + init_ border handling == the Fortran's local mask
    (global.F90 topofit/readmask, usrc.F90:83-107)."""
    c = cf.preset(name, mixing=0)
    L = cf.init_landmask(c, cf.landmask(c))
    assert sha(L.reshape(-1).astype(np.int32)) == MAN[name]["landm_sha"]


@pytest.mark.parametrize("name,st", CASES)
def test_oracle_matches_fortran(oracle_lib, name, st):
    c = cf.preset(name, mixing=0)
    g = golden(name)
    L = golden_landm(name)
    ent = MAN[name]["states"][st]
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    if st == "h5":
        x = g["h5_x"]
    elif st == "zero":
        x = np.zeros(c.nrows)
    else:
        x = cf.synthetic_state(c, L)
    assert sha(x) == ent["x_sha"], "state generator drifted"
    beg, jco, co, coB = o.fortran_matrix(x)
    B = o.fortran_rhs(x)
    assert len(co) == ent["nnz"]
    if f"{st}_co" in g:   # full arrays kept: report the first difference
        np.testing.assert_array_equal(beg, g[f"{st}_beg"])
        np.testing.assert_array_equal(jco, g[f"{st}_jco"])
        np.testing.assert_array_equal(co.view(np.int64), g[f"{st}_co"].view(np.int64))
        np.testing.assert_array_equal(B.view(np.int64), g[f"{st}_B"].view(np.int64))
    assert sha(beg) == ent["beg_sha"]
    assert sha(jco) == ent["jco_sha"]
    assert sha(co) == ent["co_sha"]
    assert sha(coB) == ent["coB_sha"]
    assert sha(B) == ent["B_sha"]


@pytest.mark.parametrize("name", list(MAN))
def test_oracle_parameters_and_intcond(oracle_lib, name):
    c = cf.preset(name, mixing=0)
    g = golden(name)
    o = oracle_lib.Oracle(c.ref_dict(), golden_landm(name), c.par_list())
    par = MAN[name]["par"]
    for p in range(1, 31):
        assert o.get_par(p) == par[p], p
    ic = o.intcond_coeff()
    if c.sres == 0:
        nz = np.nonzero(ic)[0]
        np.testing.assert_array_equal(nz + 1, g["intcond_ind"][g["intcond_val"] != 0])
        np.testing.assert_array_equal(ic[nz], g["intcond_val"][g["intcond_val"] != 0])


@pytest.mark.parametrize("name", ["coupled_natl8", "coupled_natl8s"])
def test_graph_to_fortran_inverts_fillcola(oracle_lib, name):
    """oracle.graph_to_fortran re-emits the reference's Fortran CSR (fillcolA order,
    |v| > 1e-10) from maximal-graph values: on the Fortran's own arrays (zero and synthetic
    states) the round trip is exact, so the SHA-256 check of the GPU Jacobian against
    manifest_coupled.json (tests/test_gpu_coupled.py) pins it to the Fortran."""
    c = cf.preset(name)
    g = golden(name)
    o = oracle_lib.Oracle(c.ref_dict(), cf.landmask(c), c.par_list())
    for kind in ("zero", "synthetic"):
        beg0, jco0, co0 = g[f"{kind}_beg"], g[f"{kind}_jco"], g[f"{kind}_co"]
        val = oracle_lib.fortran_to_graph(o.rowptr, o.col, beg0, jco0, co0, -1)
        beg, jco, co = oracle_lib.graph_to_fortran(c.n, c.m, c.l, c.periodic, o.rowptr, o.col, val)
        assert beg.dtype == beg0.dtype and jco.dtype == jco0.dtype and co.dtype == co0.dtype
        np.testing.assert_array_equal(beg, beg0)
        np.testing.assert_array_equal(jco, jco0)
        np.testing.assert_array_equal(co.view(np.int64), co0.view(np.int64))
