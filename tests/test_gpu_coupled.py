"""GPU: the coupled ocean + atmosphere model (BASELINE config C4)
through the C ABI.

* Ocean in coupled mode: Jacobian and residual bitwise against the reference Fortran
  (coupled_natl8 full arrays; coupled4 residual by SHA-256, Jacobian equal to the CPU
  emulation that is pinned to the Fortran on coupled_natl8).
* Atmosphere (AtmosLocal / Atmosphere): residual and Jacobian against the restatement
  oracle/atmos_oracle.py (local rows bitwise; the two dense integral rows are reductions,
  rtol 1e-13).
* CoupledModel::applyMatrix against the block matrix assembled from the device ocean CSR
  (bit-exact, above) and the oracle's atmosphere and coupling blocks: rtol 1e-12 of |A||x|.
* CoupledModel FGMRES with the forward block Gauss-Seidel preconditioner to 1e-8,
  explicit residual checked with that assembled matrix.
"""
import hashlib

import numpy as np
import pytest
import scipy.sparse as sp

from helpers import golden
from iemic import config as cf
from oracle import atmos_oracle as ao
from test_coupled import atm_args, coupled_manifest, landm_of

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def setup(name):
    from iemic.ocean import Ocean
    c = cf.preset(name)
    g = golden(name)
    L = landm_of(name)
    oc = Ocean(c, landm=L, analyze_jacobian=False)
    t, q, a, pars = atm_args(g)
    oc.setAtmosphere(t, q, a, g["atm_p"], pars)
    return c, g, L, oc


def atmos_oracle(c, g, L):
    surf = (L[c.l, 1:c.m + 1, 1:c.n + 1] != 0).astype(int)
    at = ao.AtmosOracle(c.n, c.m, c.xmin, c.xmax, c.ymin, c.ymax, c.periodic, surf,
                        Ooa=g["deps"][0], Os=g["deps"][1],
                        params={**ao.COUPLED_RUN_PARAMS,
                                "Combined Forcing": c.start_params["Combined Forcing"]})
    at.suno_ocean = np.array(at.suno[1:])
    return at


@pytest.mark.parametrize("name", ["coupled_natl8", "coupled_natl8s"])
@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_gpu_coupled_ocean_natl8_bitexact(oracle_lib, name, kind):
    c, g, L, oc = setup(name)
    np.testing.assert_array_equal(bits(oc.getDeps()), bits(g["deps"]))
    x = g[f"{kind}_x"]
    oc.setState(x)
    oc.computeJacobian()
    rowptr, col, val = oc.exportCSR()
    ref = oracle_lib.fortran_to_graph(rowptr, col, g[f"{kind}_beg"], g[f"{kind}_jco"],
                                      g[f"{kind}_co"], -1)
    np.testing.assert_array_equal(val, ref)
    F = oc.computeRHS().copy()
    np.testing.assert_array_equal(bits(F), bits(-g[f"{kind}_B"]))


@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_gpu_coupled4_ocean_bitexact(oracle_lib, kind):
    """the C4 ocean (96x38x12, Mixing 1, coupled T) against the reference Fortran itself:
    the GPU Jacobian, re-emitted in fillcolA's Fortran CSR order (oracle.graph_to_fortran,
    pinned exactly to the Fortran arrays on coupled_natl8 / natl8s), has the SHA-256 of the
    Fortran beg / jco / co arrays, and -F that of the Fortran rhs B (manifest_coupled.json,
    written by tests/golden/make_golden_coupled.py)."""
    name = "coupled4"
    c, g, L, oc = setup(name)
    man = coupled_manifest()[name]["states"][kind]
    np.testing.assert_array_equal(bits(oc.getDeps()), bits(g["deps"]))
    x = np.zeros(c.nrows) if kind == "zero" else cf.synthetic_state(c, cf.landmask(c))
    assert hashlib.sha256(x.tobytes()).hexdigest() == man["x_sha"]
    oc.setState(x)
    oc.computeJacobian()
    rowptr, col, val = oc.exportCSR()
    beg, jco, co = oracle_lib.graph_to_fortran(c.n, c.m, c.l, c.periodic, rowptr, col, val)
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(beg) == man["beg_sha"]
    assert sha(jco) == man["jco_sha"]
    assert sha(co) == man["co_sha"]
    F = oc.computeRHS().copy()
    assert sha(-F) == man["B_sha"]


@pytest.fixture(scope="module")
def coupled4():
    from iemic.coupled import Atmosphere, CoupledModel
    name = "coupled4"
    c, g, L, oc = setup(name)
    atm = Atmosphere(oc, {**ao.COUPLED_RUN_PARAMS,
                          "Combined Forcing": c.start_params["Combined Forcing"]})
    cm = CoupledModel(oc, atm, {"FGMRES iterations": 150, "FGMRES restarts": 6})
    return c, g, L, oc, atm, cm


def test_gpu_atmosphere_matches_oracle(coupled4):
    c, g, L, oc, atm, cm = coupled4
    at = atmos_oracle(c, g, L)
    np.testing.assert_array_equal(bits(atm.getCommPars()), bits(g["atm_pars"]))
    np.testing.assert_array_equal(bits(atm.getPdist()), bits(at.pdist))
    pint, area, ri, rp = atm.integral_coeff()
    np.testing.assert_array_equal(bits(pint), bits(at.pint))
    assert area == at.total_area and ri == at.rowint and rp == at.rowP
    xa = g["xa"]
    rng = np.random.default_rng(5)
    sst = 0.3 * rng.standard_normal(c.n * c.m)
    atm.setState(xa)
    atm.setOceanTemperature(sst)
    F = atm.computeRHS()
    oF = at.rhs(xa, sst)
    for r in (ri, rp):
        assert abs(F[r] - oF[r]) <= 1e-13 * max(1.0, abs(oF[r]))
    keep = np.ones(at.dim, bool)
    keep[[ri, rp]] = False
    np.testing.assert_array_equal(bits(F[keep]), bits(oF[keep]))
    atm.computeJacobian()
    val, col = atm.jacobian_ell()
    rows = np.repeat(np.arange(at.dim - 1), 7)
    m = col.reshape(-1) >= 0
    J = sp.csr_matrix((val.reshape(-1)[m], (rows[m], col.reshape(-1)[m])), shape=(at.dim, at.dim))
    oJ = at.jacobian(xa).tolil()
    oJ[ri, :] = 0
    oJ[rp, :] = 0
    D = (J - oJ.tocsr()).tocoo()
    assert np.all(D.data == 0.0), np.abs(D.data).max()


def assembled(cm, c, g, L, oc):
    """[J_o C_oa; C_ao J_a] from the device ocean CSR and the oracle's blocks."""
    at = atmos_oracle(c, g, L)
    oc.computeJacobian()
    rowptr, col, val = oc.exportCSR()
    Jo = sp.csr_matrix((val, col, rowptr), shape=(c.nrows, c.nrows))
    xa = cm.atmos.getState()
    Ja = at.jacobian(xa)
    Cao = at.block_from_ocean(c.l)
    Coa = at.block_to_ocean(c.l, at.surf, oc.getDeps(), oc.getPar("Combined Forcing"),
                            oc.getPar("Solar Forcing"), coupled_s=bool(c.coupled_s))
    return sp.bmat([[Jo, Coa], [Cao, Ja]]).tocsr()


def make_coupled(name, **sp):
    from iemic.coupled import Atmosphere, CoupledModel
    c, g, L, oc = setup(name)
    atm = Atmosphere(oc, {**ao.COUPLED_RUN_PARAMS,
                          "Combined Forcing": c.start_params["Combined Forcing"]})
    return c, g, L, oc, atm, CoupledModel(oc, atm, sp or None)


def test_gpu_coupled_salinity_spmv_and_solve():
    """coupled T and S (E - P salinity flux) on natl8: applyMatrix against the assembled
    block matrix and an FGMRES solve to 1e-8."""
    c, g, L, oc, atm, cm = make_coupled("coupled_natl8s", **{"FGMRES iterations": 200,
                                                            "FGMRES restarts": 4})
    oc.setState(g["synthetic_x"])
    atm.setState(g["xa"])
    cm.computeJacobian()
    A = assembled(cm, c, g, L, oc)
    v = np.random.default_rng(2).standard_normal(cm.N)
    y = cm.applyMatrix(v)
    scale = abs(A) @ np.abs(v)
    assert np.max(np.abs(y - A @ v) / np.maximum(scale, 1e-300)) <= 1e-12
    F = cm.computeRHS()
    dx = cm.solve(-F)
    r = np.linalg.norm(A @ dx + F) / np.linalg.norm(F)
    assert cm.last_solve.converged and r <= 1e-7, (cm.last_solve.iters, r)


def test_gpu_coupled_spmv(coupled4):
    c, g, L, oc, atm, cm = coupled4
    x = cf.synthetic_state(c, cf.landmask(c))
    oc.setState(x)
    atm.setState(g["xa"])
    cm.computeJacobian()
    A = assembled(cm, c, g, L, oc)
    rng = np.random.default_rng(11)
    v = rng.standard_normal(cm.N)
    y = cm.applyMatrix(v)
    ref = A @ v
    scale = abs(A) @ np.abs(v)
    assert np.max(np.abs(y - ref) / np.maximum(scale, 1e-300)) <= 1e-12


def test_gpu_coupled_fgmres(coupled4):
    c, g, L, oc, atm, cm = coupled4
    x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
    oc.setState(x)
    atm.setState(g["xa"])
    cm.computeJacobian()
    F = cm.computeRHS()
    dx = cm.solve(-F)
    info = cm.last_solve
    print("coupled FGMRES iterations", info.iters, "explicit", info.explicit_rel_res)
    A = assembled(cm, c, g, L, oc)
    r = np.linalg.norm(A @ dx + F) / np.linalg.norm(F)
    assert info.converged and r <= 1e-7, (info.iters, r)


def test_gpu_coupled_idr4(coupled4):
    """config C4's IDR(4) solver path (IDRSolver.H:109-340) on the coupled system."""
    c, g, L, oc, atm, cm = coupled4
    x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
    oc.setState(x)
    atm.setState(g["xa"])
    cm.computeJacobian()
    F = cm.computeRHS()
    old = dict(cm.solver_params)
    cm.solver_params.update({"Solver": "IDR", "IDR s": 4, "FGMRES iterations": 400,
                             "FGMRES restarts": 0})
    try:
        dx = cm.solve(-F)
    finally:
        cm.solver_params = old
    info = cm.last_solve
    print("coupled IDR(4) iterations", info.iters, "explicit", info.explicit_rel_res)
    A = assembled(cm, c, g, L, oc)
    r = np.linalg.norm(A @ dx + F) / np.linalg.norm(F)
    assert info.converged and r <= 1e-7, (info.iters, r)


def test_gpu_coupled_newton_step(coupled4):
    """A Newton step of the coupled model reduces ||F|| (Newton.H:76-123)."""
    c, g, L, oc, atm, cm = coupled4
    x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
    oc.setState(x)
    atm.setState(g["xa"])
    rec = cm.newtonStep()
    print("coupled Newton step", rec)
    assert rec["converged"] and rec["norm_f1"] < rec["norm_f0"]


def test_gpu_coupled_continuation(coupled4):
    """run_coupled's driver: pseudo-arclength continuation (Continuation.H) of the coupled
    model in Combined Forcing from the rest state of both models, a few steps; every
    corrector converges and the branch advances."""
    from iemic.continuation import Continuation
    c, g, L, oc, atm, cm = coupled4
    cm.setState(np.zeros(cm.N))
    cm.setPar("Combined Forcing", 0.0)
    cont = Continuation(cm, {"continuation parameter": "Combined Forcing",
                             "initial step size": 1e-2, "maximum step size": 0.05,
                             "destination 0": 1.0, "maximum number of steps": 3,
                             "Newton tolerance": 1e-4})
    cont.run()
    print("coupled continuation", [(h.par, h.newton_iters, h.norm_f) for h in cont.history])
    assert len(cont.history) >= 2
    assert cm.getPar("Combined Forcing") > 0.0
    assert all(np.isfinite(h.norm_f) for h in cont.history)


def test_gpu_atmosphere_state_file(coupled4, tmp_path):
    """Atmosphere state files (Model::saveStateToFile + additionalExports): the written
    file reads back through the HDF5 reader, and loadStateFromFile restores state and
    parameters."""
    from iemic import h5
    c, g, L, oc, atm, cm = coupled4
    atm.setState(g["xa"])
    atm.setPar("Humidity Forcing", 0.75)
    f = str(tmp_path / "atmos.h5")
    atm.saveStateToFile(f)
    t = h5.read(f)
    np.testing.assert_array_equal(t["/State/Values"][0][0], g["xa"])
    assert float(np.asarray(t["/Parameters/Humidity Forcing"][0]).reshape(-1)[0]) == 0.75
    assert t["/E/Values"][0].size == c.n * c.m and t["/P/Values"][0].size == c.n * c.m
    atm.setState(np.zeros(atm.dim))
    atm.setPar("Humidity Forcing", 1.0)
    assert atm.loadStateFromFile(f) == 0
    np.testing.assert_array_equal(atm.getState(), g["xa"])
    assert atm.getPar("Humidity Forcing") == 0.75
    atm.setPar("Humidity Forcing", 1.0)


@pytest.mark.parametrize("nranks,npx", [(2, 1), (4, 2)])
def test_gpu_coupled_subdomains(oracle_lib, nranks, npx):
    """The coupled model over Decomp2D subdomains (CoupledModel.C:274-343 distributes it on
    the ocean's maps): in-process ranks on one GPU, the atmosphere replicated on every rank
    (the SST and the coupling rows' surface T summed over the ranks, the packed dots counting
    the atmosphere once).  The ocean Jacobian rows are bit-identical to one rank's, J v
    matches to 1e-13 of |J||v|, and a coupled Newton step solves the assembled one-rank
    system to 1e-8 with the same initial residual."""
    import threading
    from iemic import _lib
    from iemic.coupled import Atmosphere, CoupledModel
    from iemic.ocean import Ocean
    name = "coupled4"
    c = cf.preset(name)
    g = golden(name)
    L = landm_of(name)
    t, q, a, pars = atm_args(g)
    x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
    xa = g["xa"]
    sp_ = {"FGMRES iterations": 150, "FGMRES restarts": 6}
    prm = {**ao.COUPLED_RUN_PARAMS, "Combined Forcing": c.start_params["Combined Forcing"]}

    def model(**kw):
        oc = Ocean(c, landm=L, analyze_jacobian=False, **kw)
        oc.setAtmosphere(t, q, a, g["atm_p"], pars)
        atm = Atmosphere(oc, prm)
        return oc, atm, CoupledModel(oc, atm, sp_)

    oc1, atm1, cm1 = model()
    oc1.setState(x)
    atm1.setState(xa)
    cm1.computeJacobian()
    rp1, col1, val1 = oc1.exportCSR()
    v = np.random.default_rng(7).standard_normal(cm1.N)
    y1 = cm1.applyMatrix(v)
    A = assembled(cm1, c, g, L, oc1)
    group = _lib.lib().iemic_local_group_new(nranks)
    out = [None] * nranks

    def work(r):
        try:
            oc, atm, cm = model(local_group=group, rank=r, nranks=nranks, npx=npx)
            oc.setState(x)
            atm.setState(xa)
            cm.computeJacobian()
            csr = oc.exportCSR()
            y = cm.applyMatrix(v)
            rec = cm.newtonStep()
            out[r] = dict(rows=oc.owned_rows(), csr=csr, y=y, rec=rec, x1=oc.getState(),
                          xa1=atm.getState(), lay=oc.layout())
            cm.close(); atm.close(); oc.close()
        except Exception as e:  # noqa: BLE001
            out[r] = repr(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for h in th:
        h.start()
    for h in th:
        h.join()
    _lib.lib().iemic_local_group_free(group)
    assert all(isinstance(o, dict) for o in out), out
    x1 = np.zeros(cm1.N)
    scale = abs(A) @ np.abs(v)
    for o in out:
        rows = o["rows"]
        rp, col, val = o["csr"]
        for k, qr in enumerate(rows):
            np.testing.assert_array_equal(col[rp[k]:rp[k + 1]], col1[rp1[qr]:rp1[qr + 1]])
            np.testing.assert_array_equal(bits(val[rp[k]:rp[k + 1]]), bits(val1[rp1[qr]:rp1[qr + 1]]))
        sel = np.concatenate([rows, np.arange(c.nrows, cm1.N)])
        assert np.max(np.abs(o["y"][sel] - y1[sel]) / np.maximum(scale[sel], 1e-300)) <= 1e-13
        x1[rows] = o["x1"][rows]
        np.testing.assert_array_equal(o["xa1"], out[0]["xa1"])     # the replicas agree
        assert o["rec"]["converged"]
        assert o["rec"]["norm_f0"] == out[0]["rec"]["norm_f0"]
    x1[c.nrows:] = out[0]["xa1"]
    oc1.setState(x)
    atm1.setState(xa)
    F = cm1.computeRHS()
    f0 = np.linalg.norm(F)
    assert abs(out[0]["rec"]["norm_f0"] - f0) <= 1e-12 * f0
    dx = x1 - np.concatenate([x, xa])
    lin = np.linalg.norm(A @ dx + F) / f0
    assert lin <= 1e-7, lin
