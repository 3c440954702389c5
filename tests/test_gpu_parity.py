"""GPU parity: the HIP path through the C ABI against the oracle on the same inputs.

Bar: Jacobian values, mass diagonal and residual bit-exact (the kernels
are compiled with -ffp-contract=off and restate the reference arithmetic); the single
intcond residual entry (SRES=0) is a parallel reduction, rtol 1e-13; SpMV sums in a
different order than the CSR oracle, rtol 1e-13 in the max norm relative to |J||x|.
"""
import numpy as np
import pytest

from helpers import golden_landm, mask_fix
from iemic import config as cf

pytestmark = pytest.mark.gpu

NAMES = ["test6x6x4", "natl8", "2dmoc", "2dmoc_run", "gateway16", "global4"]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


@pytest.fixture(scope="module")
def Ocean():
    from iemic.ocean import Ocean
    return Ocean


def make(Ocean, orc, name, mixing=0, **kw):
    c = cf.preset(name, mixing=mixing)
    L0 = golden_landm(name) if name not in ("global2", "global1") else cf.init_landmask(c, cf.landmask(c))
    oc = Ocean(c, landm=L0, **kw)
    L = mask_fix(orc, c, L0)
    o = orc.Oracle(c.ref_dict(), L, c.par_list())
    return c, oc, o, L


@pytest.mark.parametrize("name", NAMES)
def test_mask_fix_matches(oracle_lib, Ocean, name):
    c, oc, o, L = make(Ocean, oracle_lib, name)
    np.testing.assert_array_equal(oc.landmask(), cf.init_landmask(c, L).reshape(-1))


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_jacobian_rhs_bitexact(oracle_lib, Ocean, name, kind):
    c, oc, o, L = make(Ocean, oracle_lib, name)
    x = np.zeros(c.nrows) if kind == "zero" else cf.synthetic_state(c, L)
    oc.setState(x)
    oc.computeJacobian()
    rowptr, col, val = oc.exportCSR()
    ov, oB = o.jacobian(x)
    np.testing.assert_array_equal(rowptr, o.rowptr)
    np.testing.assert_array_equal(col, o.col)
    np.testing.assert_array_equal(val, ov)
    np.testing.assert_array_equal(bits(oc.diagB()), bits(oB))
    F = oc.computeRHS().copy()
    oF = o.rhs(x)
    ri = o.rowintcon
    if ri >= 0:
        assert abs(F[ri] - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
        F[ri] = oF[ri]
    np.testing.assert_array_equal(bits(F), bits(oF))


@pytest.mark.timeout(600)
def test_global1_full_size(oracle_lib, Ocean):
    """SURVEY config C5, the 1-degree grid (384x152x32, Mixing = 1): 11,206,656 rows and
    192,314,880 maximal-graph entries.  J and F bit-exact against the oracle, and one
    Newton step whose FGMRES solve reaches 1e-8 on the oracle's own J."""
    c, oc, o, L = make(Ocean, oracle_lib, "global1", mixing=1,
                       solver_params={"FGMRES tolerance": 1e-8, "FGMRES iterations": 100,
                                      "FGMRES restarts": 30})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    _, col, val = oc.exportCSR()
    ov, _ = o.jacobian(x)
    assert len(val) == 192_314_880
    np.testing.assert_array_equal(col, o.col)
    del col
    np.testing.assert_array_equal(bits(val), bits(ov))
    del val
    F0 = o.rhs(x)
    np.testing.assert_array_equal(bits(oc.computeRHS()), bits(F0))
    info = oc.newtonStep()
    assert info.solve.converged == 1 and info.solve.explicit_rel_res <= 1e-8
    lin = np.linalg.norm(F0 + o.spmv(ov, oc.getState() - x)) / np.linalg.norm(F0)
    assert lin <= 1e-8, lin
    print(f"global1 Newton step: {info.solve.iters} FGMRES steps, |F0| {info.norm_f0:.4e} "
          f"|F1| {info.norm_f1:.4e}, {info.t_total_ms:.0f} ms")


@pytest.mark.parametrize("name", NAMES)
def test_spmv(oracle_lib, Ocean, name):
    c, oc, o, L = make(Ocean, oracle_lib, name)
    x = cf.synthetic_state(c, L)
    oc.setState(x)
    oc.computeJacobian()
    ov, _ = o.jacobian(x)
    v = cf.synthetic_vector(c, seed=11)
    y = oc.applyMatrix(v)
    ref = o.spmv(ov, v)
    scale = o.spmv(np.abs(ov), np.abs(v))
    assert np.all(np.abs(y - ref) <= 1e-13 * scale + 1e-300)


def test_global2_full_size(oracle_lib, Ocean):
    """BASELINE configuration: J and F bit-exact at 1,400,832 rows."""
    c, oc, o, L = make(Ocean, oracle_lib, "global2")
    x = cf.synthetic_state(c, L)
    oc.setState(x)
    oc.computeJacobian()
    _, col, val = oc.exportCSR()
    ov, oB = o.jacobian(x)
    assert len(val) == 23_798_016 or len(val) == len(ov)
    np.testing.assert_array_equal(val, ov)
    F = oc.computeRHS()
    np.testing.assert_array_equal(bits(F), bits(o.rhs(x)))


@pytest.mark.parametrize("name", ["test6x6x4", "natl8", "2dmoc", "2dmoc_run", "gateway16",
                                  "global4"])
def test_block_gs_apply_matches_cpu(oracle_lib, Ocean, name):
    """GPU block Gauss-Seidel apply (Schur solve by block cyclic reduction) == CPU twin
    (Schur solve by band LU with partial pivoting)."""
    c, oc, o, L = make(Ocean, oracle_lib, name, solver_params={"Preconditioner": 2, "TS sweeps": 3,
                                                               "Dyn iterations": 1,
                                                               "TS multigrid cycles": 0})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    oc.buildPreconditioner(force=True)
    ov, _ = o.jacobian(x)
    P = oracle_lib.BlockGS(o, ov, 3)
    r = cf.synthetic_vector(c, seed=3)
    z = oc.applyPrecon(r)
    zc = P.apply(r)
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-8 * np.max(np.abs(zc))


@pytest.mark.parametrize("name", ["natl8", "gateway16", "global4", "global2"])
def test_block_gs_default_apply_matches_cpu(oracle_lib, Ocean, name):
    """The default block GS (4 damped defect-correction passes on the dynamics block, the
    first two with the Schur solve, one T/S aggregation-multigrid V-cycle with z-line
    smoothing, Mixing = 1) == its CPU twin
    (prec_oracle.c: band-LU Schur, block-Thomas z-lines)."""
    c, oc, o, L = make(Ocean, oracle_lib, name, mixing=1, solver_params={"Preconditioner": 2})
    sp = oc.solver_params
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    oc.buildPreconditioner(force=True)
    ov, _ = o.jacobian(x)
    P = oracle_lib.BlockGS(o, ov, 3, dyn_iters=sp["Dyn iterations"], dyn_omega=sp["Dyn damping"],
                           ts_mg=sp["TS multigrid cycles"], schur_passes=sp["Schur passes"])
    r = cf.synthetic_vector(c, seed=3)
    z, zc = oc.applyPrecon(r), P.apply(r)
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-8 * np.max(np.abs(zc))


@pytest.mark.parametrize("name,ts_at", [("global4", 1), ("global4", 2), ("global2", 2), ("global2", 3)])
def test_block_gs_early_ts_matches_cpu(oracle_lib, Ocean, name, ts_at):
    """T/S right-hand side after ts_at of the 4 dynamics passes (the T/S multigrid on the
    side stream, beside the remaining passes) == the CPU twin with the same ts_at; and it
    differs from the default (the T/S rhs after the last pass), so the fork is exercised."""
    c, oc, o, L = make(Ocean, oracle_lib, name, mixing=1,
                       solver_params={"Preconditioner": 2, "TS after dyn pass": ts_at})
    sp = oc.solver_params
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    oc.buildPreconditioner(force=True)
    ov, _ = o.jacobian(x)
    kw = dict(dyn_iters=sp["Dyn iterations"], dyn_omega=sp["Dyn damping"], ts_mg=sp["TS multigrid cycles"],
              schur_passes=sp["Schur passes"])
    r = cf.synthetic_vector(c, seed=3)
    z = oc.applyPrecon(r)
    zc = oracle_lib.BlockGS(o, ov, 3, ts_at=ts_at, **kw).apply(r)
    z0 = oracle_lib.BlockGS(o, ov, 3, **kw).apply(r)
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-8 * np.max(np.abs(zc))
    assert np.max(np.abs(z0 - zc)) > 1e-6 * np.max(np.abs(zc))


@pytest.mark.parametrize("name,sp_k", [("global4", 1), ("global4", 3), ("global2", 0), ("global2", 3)])
def test_block_gs_schur_passes_matches_cpu(oracle_lib, Ocean, name, sp_k):
    """sp_k of the 4 dynamics passes solve the Schur system, the first sp_k - 1 and the last
    (1: the first only; 0: every pass); the others take pbar = 0, no Schur reduction or solve.
    == the CPU twin with the same schur_passes; and it differs from the default (2: the first
    and the last)."""
    c, oc, o, L = make(Ocean, oracle_lib, name, mixing=1,
                       solver_params={"Preconditioner": 2, "Schur passes": sp_k})
    sp = oc.solver_params
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    oc.buildPreconditioner(force=True)
    ov, _ = o.jacobian(x)
    kw = dict(dyn_iters=sp["Dyn iterations"], dyn_omega=sp["Dyn damping"], ts_mg=sp["TS multigrid cycles"])
    r = cf.synthetic_vector(c, seed=3)
    z = oc.applyPrecon(r)
    zc = oracle_lib.BlockGS(o, ov, 3, schur_passes=sp_k, **kw).apply(r)
    z0 = oracle_lib.BlockGS(o, ov, 3, schur_passes=2, **kw).apply(r)
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-8 * np.max(np.abs(zc))
    assert np.max(np.abs(z0 - zc)) > 1e-6 * np.max(np.abs(zc))


@pytest.mark.parametrize("mixing", [0, 1])
def test_block_gs_apply_global2(oracle_lib, Ocean, mixing):
    """The same at the bench size (2 degrees, 192x76x16, 8,996 water columns: 192 blocks of
    76 latitudes in the Schur cyclic reduction, 8 levels)."""
    c, oc, o, L = make(Ocean, oracle_lib, "global2", mixing=mixing,
                       solver_params={"Preconditioner": 2, "TS sweeps": 3, "Dyn iterations": 1,
                                      "TS multigrid cycles": 0})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    oc.buildPreconditioner(force=True)
    ov, _ = o.jacobian(x)
    zc = oracle_lib.BlockGS(o, ov, 3).apply(cf.synthetic_vector(c, seed=3))
    z = oc.applyPrecon(cf.synthetic_vector(c, seed=3))
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-8 * np.max(np.abs(zc))


@pytest.mark.parametrize("name,dyn", [("natl8", 2), ("gateway16", 3), ("global4", 2),
                                      ("global4", 4)])
@pytest.mark.parametrize("mr", [False, True])
def test_dyn_defect_correction(oracle_lib, Ocean, name, dyn, mr):
    """Block GS with defect-correction passes on the dynamics block: converges FGMRES in
    fewer steps; with a fixed step (the default damping) it is a linear operator
    (apply(a r1 + r2) = a apply(r1) + apply(r2)), with minimal-residual steps a
    deterministic nonlinear one (FGMRES is flexible)."""
    its = {}
    for d in (1, dyn):
        c, oc, o, L = make(Ocean, oracle_lib, name,
                           solver_params={"Preconditioner": 2, "FGMRES iterations": 500,
                                          "FGMRES tolerance": 1e-8, "Dyn iterations": d,
                                          "Dyn minimal residual": mr})
        x = cf.synthetic_state(c, L, amp_ts=1e-3)
        oc.setState(x)
        oc.computeJacobian()
        ov, _ = o.jacobian(x)
        b = o.spmv(ov, cf.synthetic_vector(c, seed=5))
        sol = oc.solve(b)
        res = np.linalg.norm(b - o.spmv(ov, sol)) / np.linalg.norm(b)
        assert oc.last_solve.converged == 1 and res <= 1e-7
        its[d] = oc.last_solve.iters
        if d > 1:
            r1, r2 = cf.synthetic_vector(c, seed=3), cf.synthetic_vector(c, seed=4)
            z = oc.applyPrecon(2.5 * r1 + r2)
            if not mr:
                zl = 2.5 * oc.applyPrecon(r1) + oc.applyPrecon(r2)
                assert np.max(np.abs(z - zl)) <= 1e-9 * np.max(np.abs(zl))
            assert np.array_equal(z, oc.applyPrecon(2.5 * r1 + r2))
    assert its[dyn] <= its[1], its


@pytest.mark.parametrize("name", ["natl8", "2dmoc", "gateway16", "global4"])
def test_ts_multigrid(oracle_lib, Ocean, name):
    """T/S solve by one aggregation-multigrid V-cycle instead of 12 plain sweeps: still a
    linear preconditioner, FGMRES converges to 1e-8 in no more iterations."""
    its = {}
    for mg in (0, 1):
        c, oc, o, L = make(Ocean, oracle_lib, name,
                           solver_params={"Preconditioner": 2, "FGMRES iterations": 500,
                                          "FGMRES tolerance": 1e-8, "TS multigrid cycles": mg,
                                          "TS sweeps": 12})
        x = cf.synthetic_state(c, L, amp_ts=1e-3)
        oc.setState(x)
        oc.computeJacobian()
        ov, _ = o.jacobian(x)
        b = o.spmv(ov, cf.synthetic_vector(c, seed=5))
        sol = oc.solve(b)
        res = np.linalg.norm(b - o.spmv(ov, sol)) / np.linalg.norm(b)
        assert oc.last_solve.converged == 1 and res <= 1e-7, (mg, res)
        its[mg] = oc.last_solve.iters
        if mg:
            r1, r2 = cf.synthetic_vector(c, seed=3), cf.synthetic_vector(c, seed=4)
            z = oc.applyPrecon(2.5 * r1 + r2)
            zl = 2.5 * oc.applyPrecon(r1) + oc.applyPrecon(r2)
            assert np.max(np.abs(z - zl)) <= 1e-9 * np.max(np.abs(zl))
            assert np.array_equal(oc.applyPrecon(r1), oc.applyPrecon(r1))   # deterministic
    assert its[1] <= its[0] + 2, its


@pytest.mark.parametrize("name,prec", [("test6x6x4", 1), ("test6x6x4", 2), ("natl8", 2), ("2dmoc", 2),
                                       ("2dmoc_run", 2), ("gateway16", 2), ("global4", 2)])
def test_fgmres_solve(oracle_lib, Ocean, name, prec):
    c, oc, o, L = make(Ocean, oracle_lib, name,
                       solver_params={"Preconditioner": prec, "FGMRES iterations": 500,
                                      "FGMRES tolerance": 1e-8})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    ov, _ = o.jacobian(x)
    # J is singular (pressure null modes): the right-hand side must lie in its range
    b = o.spmv(ov, cf.synthetic_vector(c, seed=5))
    sol = oc.solve(b)
    res = np.linalg.norm(b - o.spmv(ov, sol)) / np.linalg.norm(b)
    assert oc.last_solve.converged == 1
    assert res <= 1e-7
    assert abs(oc.last_solve.explicit_rel_res - res) <= 1e-9


@pytest.mark.parametrize("orth", ["DCGS2", "DGKS"])
@pytest.mark.parametrize("name,prec", [("natl8", 0), ("natl8", 1), ("global4", 0), ("global4", 1)])
def test_fgmres_long_cycle(oracle_lib, Ocean, name, prec, orth):
    """One 500-step cycle with a weak (prec 1, block Jacobi) or no preconditioner: the
    Krylov candidates stay normalised (DCGS2's lagged normalisation), so a long cycle ends
    without a spurious non-finite error or false breakdown, the residual decreases and the
    reported explicit residual is the true one of the oracle's J."""
    c, oc, o, L = make(Ocean, oracle_lib, name,
                       solver_params={"Preconditioner": prec, "FGMRES iterations": 500,
                                      "FGMRES restarts": 0, "FGMRES tolerance": 1e-8,
                                      "Orthogonalization": orth})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    ov, _ = o.jacobian(x)
    b = o.spmv(ov, cf.synthetic_vector(c, seed=5))
    sol = oc.solve(b)
    res = np.linalg.norm(b - o.spmv(ov, sol)) / np.linalg.norm(b)
    s_ = oc.last_solve
    assert np.all(np.isfinite(sol))
    assert res <= 1.0 + 1e-12          # minimal residual over the cycle: never above ||b||
    assert s_.converged == 1 or s_.iters == 500
    assert abs(s_.explicit_rel_res - res) <= 1e-8 + 1e-6 * res


def test_fgmres_nonfinite_is_an_error(oracle_lib, Ocean):
    """A NaN reaching the Krylov basis raises instead of passing for a breakdown (res = 0)."""
    from iemic._lib import IemicError
    c, oc, o, L = make(Ocean, oracle_lib, "natl8", solver_params={"Preconditioner": 2})
    oc.setState(cf.synthetic_state(c, L, amp_ts=1e-3))
    oc.computeJacobian()
    b = cf.synthetic_vector(c, seed=5)
    b[len(b) // 2] = np.nan
    with pytest.raises(IemicError, match="non-finite"):
        oc.solve(b)


def test_nan_state_fails_cleanly(oracle_lib, Ocean):
    """A NaN state (a diverging Newton iterate): the Newton step reports an error instead of
    faulting -- the NaN reaches the Schur operator through the integral-condition correction,
    so the set-up's inverses see NaN pivot candidates (k_cr_inv, advisor round 4) -- and the
    context stays usable: the next step from a finite state converges exactly as before
    (scripts/nan_probe.py shows the same solve bitwise before and after)."""
    from iemic._lib import IemicError
    c, oc, o, L = make(Ocean, oracle_lib, "global4",
                       solver_params={"Preconditioner": 2, "FGMRES tolerance": 1e-10})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    ref = oc.newtonStep()
    assert ref.solve.converged == 1
    xn = x.copy()
    xn[::7] = np.nan
    oc.setState(xn)
    with pytest.raises(IemicError):
        oc.newtonStep()
    oc.setState(x)
    info = oc.newtonStep()
    assert info.solve.converged == 1 and info.solve.iters == ref.solve.iters
    assert info.norm_f1 == ref.norm_f1


def _land_rows(c, L):
    Li = L[1:-1, 1:-1, 1:-1].reshape(-1)
    return np.repeat((Li != 0).astype(float), 6)


@pytest.mark.parametrize("name,prec", [("test6x6x4", 2), ("natl8", 2), ("gateway16", 2),
                                       ("global4", 2)])
def test_newton_step(oracle_lib, Ocean, name, prec):
    c, oc, o, L = make(Ocean, oracle_lib, name,
                       solver_params={"Preconditioner": prec, "FGMRES tolerance": 1e-10})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    f0 = np.linalg.norm(o.rhs(x))
    info = oc.newtonStep()
    x1 = oc.getState()
    f1 = np.linalg.norm(o.rhs(x1))
    assert abs(info.norm_f0 - f0) <= 1e-12 * f0
    assert abs(info.norm_f1 - f1) <= 1e-10 * max(f1, 1e-300) + 1e-14 * f0
    # the step solves the linearised system: ||F + J dx|| <= tol-level * ||F||
    ov, _ = o.jacobian(x)
    F0 = o.rhs(x)
    lin = np.linalg.norm(F0 + o.spmv(ov, x1 - x)) / np.linalg.norm(F0)
    assert info.solve.converged == 1
    assert lin <= 1e-8


def test_intcond_correction(oracle_lib, Ocean):
    """THCM::setIntCondCorrection on an SRES = 0 grid: the integral-condition entry of F
    becomes intSign (coeff . x - coeff . x0); every other entry is unchanged."""
    c, oc, o, L = make(Ocean, oracle_lib, "natl8")
    ric = oc.rowintcon
    assert ric >= 0
    x0 = cf.synthetic_state(c, L, amp_ts=1e-3)
    corr = oc.setIntCondCorrection(x0)
    coeff = o.intcond_coeff()
    assert abs(corr - coeff @ x0) <= 1e-13 * np.abs(coeff) @ np.abs(x0)
    x = cf.synthetic_state(c, L, seed=99, amp_ts=1e-3)
    oc.setState(x)
    F = oc.computeRHS()
    oF = o.rhs(x)
    keep = np.ones(c.nrows, bool)
    keep[ric] = False
    np.testing.assert_array_equal(F[keep], oF[keep])
    sign = o.d["int_sign"]
    assert abs(F[ric] - (oF[ric] - sign * corr)) <= 1e-12 * max(1.0, abs(oF[ric]))
    assert abs(oc.setIntCondCorrection() - coeff @ x) <= 1e-12 * np.abs(coeff) @ np.abs(x)


@pytest.mark.parametrize("name,s", [("natl8", 4), ("gateway16", 4), ("global4", 4), ("global4", 8)])
def test_idr_solve(oracle_lib, Ocean, name, s):
    """IDR(s) (IDRSolver.H:109-340) with the block-GS preconditioner: the solution meets the
    tolerance on the oracle's J, and the reported explicit residual is the true one."""
    c, oc, o, L = make(Ocean, oracle_lib, name,
                       solver_params={"Solver": "IDR", "IDR s": s, "FGMRES tolerance": 1e-8,
                                      "FGMRES iterations": 1000, "FGMRES restarts": 0})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    oc.computeJacobian()
    ov, _ = o.jacobian(x)
    b = o.spmv(ov, cf.synthetic_vector(c, seed=5))
    sol = oc.solve(b)
    res = np.linalg.norm(b - o.spmv(ov, sol)) / np.linalg.norm(b)
    assert oc.last_solve.converged == 1, (oc.last_solve.iters, res)
    assert res <= 2e-8
    assert abs(oc.last_solve.explicit_rel_res - res) <= 1e-9


def test_idr_newton_step_global2(oracle_lib, Ocean):
    """The bench's Newton step (2 degrees, Mixing = 1) with IDR(4) instead of FGMRES."""
    c, oc, o, L = make(Ocean, oracle_lib, "global2", mixing=1,
                       solver_params={"Solver": "IDR", "IDR s": 4, "FGMRES tolerance": 1e-8,
                                      "FGMRES iterations": 2000, "FGMRES restarts": 0})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    info = oc.newtonStep()
    F0 = o.rhs(x)
    ov, _ = o.jacobian(x)
    lin = np.linalg.norm(F0 + o.spmv(ov, oc.getState() - x)) / np.linalg.norm(F0)
    assert info.solve.converged == 1 and lin <= 2e-8, (info.solve.iters, lin)
    print(f"IDR(4) global2 Newton step: {info.solve.iters} iterations, {info.t_total_ms:.0f} ms")


@pytest.mark.parametrize("name,omega", [("global4", 1.1), ("global2", 1.1), ("global2", 0.95)])
def test_stagnation_safeguard(oracle_lib, Ocean, name, omega):
    """Defect-correction passes with a step too long for the state (omega = 1.1: the passes'
    error propagation has eigenvalues near 1 - 2 omega; at the 2-degree branch state FGMRES
    used to stall at 2e-4 after 1890 steps): a restart cycle that cuts the true residual less
    than 4x switches the passes to minimal-residual steps, and the Newton step converges.  At
    the default omega nothing switches (the default path is unchanged)."""
    import os
    from conftest import ROOT
    c, oc, o, L = make(Ocean, oracle_lib, name, mixing=1,
                       solver_params={"FGMRES tolerance": 1e-8, "FGMRES iterations": 90,
                                      "FGMRES restarts": 20, "Dyn damping": omega})
    if name == "global2":
        with np.load(os.path.join(ROOT, "bench_data", "global2_cf05.npz"), allow_pickle=False) as d:
            x = d["x"].astype(np.float64)
    else:
        x = cf.synthetic_state(c, L, amp_ts=1e-3)
    oc.setState(x)
    info = oc.newtonStep()
    F0 = o.rhs(x)
    ov, _ = o.jacobian(x)
    lin = np.linalg.norm(F0 + o.spmv(ov, oc.getState() - x)) / np.linalg.norm(F0)
    print(f"{name} omega {omega}: {info.solve.iters} FGMRES steps, safeguard {info.solve.safeguard}, "
          f"lin {lin:.2e}")
    assert info.solve.converged == 1 and lin <= 2e-8, (info.solve.iters, lin)
    if omega < 1.0:
        assert info.solve.safeguard == 0
    if name == "global2" and omega > 1.0:
        assert info.solve.safeguard == 1


@pytest.mark.timeout(300)
def test_global2_bench_state_parity(oracle_lib, Ocean):
    """The benchmarked input itself (bench.py's default line): the 2-degree branch state
    bench_data/global2_cf05.npz with Mixing = 1 (convective adjustment active).  J values and
    F bit-exact against the oracle, and the Newton step the bench times: its solve reaches
    ||F + J dx|| <= 1e-8 ||F|| with the oracle's J, its new residual is the oracle's F at the
    new state, and ||F1|| agrees with the CPU port's Newton step (same algorithm, oracle/
    prec_oracle.c) to 1e-10 relative -- north_star's bar at the exact benchmarked input."""
    import os
    from conftest import ROOT
    sp = {"FGMRES tolerance": 1e-8, "FGMRES iterations": 90, "FGMRES restarts": 20}
    c, oc, o, L = make(Ocean, oracle_lib, "global2", mixing=1, solver_params=sp)
    with np.load(os.path.join(ROOT, "bench_data", "global2_cf05.npz"), allow_pickle=False) as d:
        x = d["x"].astype(np.float64)
    # bench.py steps at the preset's Combined Forcing 0.5 from this state (continued to 0.50002)
    oc.setState(x)
    oc.computeJacobian()
    _, col, val = oc.exportCSR()
    ov, _ = o.jacobian(x)
    np.testing.assert_array_equal(col, o.col)
    del col
    np.testing.assert_array_equal(bits(val), bits(ov))
    del val
    F0 = o.rhs(x)
    np.testing.assert_array_equal(bits(oc.computeRHS()), bits(F0))
    info = oc.newtonStep()
    assert info.solve.converged == 1 and info.solve.explicit_rel_res <= 1e-8
    x1 = oc.getState()
    lin = np.linalg.norm(F0 + o.spmv(ov, x1 - x)) / np.linalg.norm(F0)
    assert lin <= 1e-8, lin
    F1 = o.rhs(x1)
    assert abs(info.norm_f1 - np.linalg.norm(F1)) <= 1e-13 * np.linalg.norm(F1)
    # the CPU port's Newton step from the same state (bench.py's cpu_baseline algorithm)
    P = oracle_lib.BlockGS(o, ov, 12, dyn_iters=4, dyn_omega=0.95, ts_mg=1,
                           schur_passes=oc.solver_params["Schur passes"])
    dx, its, rel, _ = P.fgmres(np.ascontiguousarray(-F0), tol=1e-8, m=90, maxit=90 * 21)
    f1_cpu = np.linalg.norm(o.rhs(x + dx))
    print(f"bench state: GPU {info.solve.iters} FGMRES steps |F1| {info.norm_f1:.16e}; "
          f"CPU port {its} steps |F1| {f1_cpu:.16e}")
    assert abs(info.norm_f1 - f1_cpu) <= 1e-10 * f1_cpu, (info.norm_f1, f1_cpu)
