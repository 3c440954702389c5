"""The reference's own ocean unit and integration tests, run on the GPU model.

* test_ocean.C (test/ocean: 8x8x4 mask_natl8, Mixing = 1, SRES = 0):
  - RHSNorm (:33-41): ||F(0)|| < 1e-6 at the trivial state and the starting parameters;
  - MassMat (:45-109): B = -Ro on the U/V rows, 0 on W/P, -1 on T (and S) of every ocean
    cell, 0 on the integral-condition row;
  - Continuation + Integrals (:178-307): after the test's continuation in Combined Forcing
    the salt advection volume integral vanishes (1e-10) and every S column of J integrated
    with the integral-condition coefficients vanishes below the top two layers (1e-7), the
    column-by-column value (method 1, J e_S) equal in norm to Ocean::getColumnIntegral
    (method 2) within 1e-7.
* intt_2dmoc.C (test/2dmoc: 3x6x6 two-dimensional Atlantic MOC, SRES = 0, Coriolis off):
  the five-leg continuation chain Combined Forcing -> CMPR -> Salinity Forcing -> CMPR ->
  Salinity Forcing gives psi_max = 14.7 +- 0.1 Sv and psi_min = 0 +- 1e-4 Sv (Ocean::getPsiM);
  continuing to the other branch gives the mirrored extrema within 1e-4 (:15-135).

Parameters are the reference XML files' (quoted where used); the preconditioner is the
build's block Gauss-Seidel (the reference's Trilinos solve is replaced).
"""
import numpy as np
import pytest

from iemic import config as cf
from iemic.continuation import Continuation

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Ocean():
    from iemic.ocean import Ocean
    return Ocean


# test/ocean/solver_params.xml
OCEAN_SOLVER = {"FGMRES tolerance": 1e-6, "FGMRES iterations": 500, "FGMRES restarts": 0}
# test/ocean/continuation_params.xml
OCEAN_CONTINUATION = {
    "continuation parameter": "Combined Forcing", "initial step size": 1.0e-2,
    "minimum step size": 1.0e-8, "maximum step size": 1.0e-1, "destination 0": 1.0,
    "maximum number of steps": 5, "Newton tolerance": 1.0e-4, "destination tolerance": 1.0e-4,
    "maximum Newton iterations": 15, "backtracking steps": 5, "post processing": "at final point",
    "epsilon increment": 1.0e-5, "state tangent scaling": 1.0, "reject failed iteration": True,
    "enable Newton Chord hybrid solve": True, "backtracking increase": 1.2, "tangent type": "S",
    "predictor bound": 3000.0}


def natl8(Ocean):
    c = cf.preset("natl8")                      # test/ocean/ocean_params.xml
    c.start_params["Combined Forcing"] = 0.0    # its "Starting Parameters"
    return c, Ocean(c, solver_params=OCEAN_SOLVER)


def test_ocean_rhs_norm(Ocean):
    """test_ocean.C RHSNorm: the trivial state solves the unforced problem."""
    c, oc = natl8(Ocean)
    oc.setState(np.zeros(c.nrows))
    F = oc.computeRHS()
    assert np.linalg.norm(F) < 1e-6, np.linalg.norm(F)


def test_ocean_mass_matrix(Ocean):
    """test_ocean.C MassMat: applyMassMat(1) on the ocean cells of the borderless mask."""
    c, oc = natl8(Ocean)
    oc.setState(np.zeros(c.nrows))
    oc.computeJacobian()
    out = oc.applyMassMat(np.ones(c.nrows))
    assert out.size == c.nrows
    rosb = oc.getPar("Rossby-Number")
    L = oc.landmask().reshape(c.l + 2, c.m + 2, c.n + 2)[1:-1, 1:-1, 1:-1].reshape(-1)
    ocean = np.flatnonzero(L == 0)
    assert ocean.size > 0
    B = out.reshape(-1, 6)[ocean]
    for var in (0, 1):                          # U, V: -Ro where nonzero
        nz = B[:, var] != 0
        assert np.all(B[nz, var] == -rosb)
    assert np.all(B[:, 2] == 0.0) and np.all(B[:, 3] == 0.0)
    assert np.all(B[:, 4] == -1.0)
    nz = B[:, 5] != 0
    assert np.all(B[nz, 5] == -1.0)
    ri = oc.rowintcon                         # SRES = 0: the integral-condition row
    assert ri >= 0 and out[ri] == 0.0


def test_ocean_continuation_integrals(Ocean):
    """test_ocean.C Continuation + Integrals: continue from rest, then the discrete
    conservation checks on the end state and its Jacobian."""
    c, oc = natl8(Ocean)
    oc.setState(np.zeros(c.nrows))
    cont = Continuation(oc, OCEAN_CONTINUATION)
    assert cont.run() == 0
    assert oc.getPar("Combined Forcing") > 0.0
    assert np.linalg.norm(oc.getMassMat()) != 0.0
    adv, _ = oc.integralChecks()
    assert abs(adv) < 1e-10, adv
    oc.computeJacobian()
    coef = oc.getIntCondCoeff()
    ri = oc.rowintcon
    coef[ri] = 0.0
    N, M, L = c.n, c.m, c.l
    tmp = np.zeros(c.nrows)
    ints = []
    e = np.zeros(c.nrows)
    for k in range(L):
        for j in range(M):
            for i in range(N):
                rowS = 6 * ((k * M + j) * N + i) + 5       # FIND_ROW2(_NUN_,N,M,L,i,j,k,SS)
                e[rowS] = 1.0
                dot = float(coef @ oc.applyMatrix(e))
                e[rowS] = 0.0
                tmp[rowS] = dot
                if k < L - 2:                                # all but the top rows
                    ints.append(dot)
    assert np.max(np.abs(ints)) < 1e-7, np.max(np.abs(ints))
    col = oc.getColumnIntegral()
    assert abs(np.linalg.norm(tmp) - np.linalg.norm(col)) < 1e-7


# test/2dmoc/continuation_params.xml
MOC_CONTINUATION = {
    "continuation parameter": "Combined Forcing", "initial step size": 1.0e-1,
    "minimum step size": 1.0e-8, "maximum step size": 1.0, "increase step size": 2.0,
    "decrease step size": 2.0, "destination 0": 1.0, "maximum number of steps": -1,
    "Newton tolerance": 1.0e-3, "destination tolerance": 1.0e-6,
    "maximum Newton iterations": 15, "backtracking steps": 5, "corrector residual test": "D",
    "epsilon increment": 1.0e-6, "state tangent scaling": 1.0,
    "enable Newton Chord hybrid solve": False, "backtracking increase": 1.0,
    "tangent type": "S", "predictor bound": 100.0}
# test/2dmoc/solver_params.xml
MOC_SOLVER = {"FGMRES tolerance": 1e-3, "FGMRES iterations": 500, "FGMRES restarts": 0}


@pytest.mark.timeout(600)
def test_2dmoc_continuation_chain_psim(Ocean):
    """intt_2dmoc.C: the chain of continuations to the asymmetric state 1, its overturning
    extrema, then continuation to the mirrored state 2."""
    c = cf.preset("2dmoc")                      # test/2dmoc/ocean_params.xml (3x6x6)
    c.start_params["Combined Forcing"] = 0.0
    oc = Ocean(c, solver_params=MOC_SOLVER)
    oc.setState(np.zeros(c.nrows))
    p = dict(MOC_CONTINUATION)
    legs = [("Combined Forcing", 1.0, 0.1), ("CMPR", -0.2, -0.5), ("Salinity Forcing", 0.02, 0.5),
            ("CMPR", 0.0, 0.5), ("Salinity Forcing", 0.04, 0.5)]
    for name, dest, ds in legs:
        if name != "Combined Forcing":
            p.update({"continuation parameter": name, "destination 0": dest, "initial step size": ds})
        assert Continuation(oc, p).run() == 0, (name, dest)
        assert abs(oc.getPar(name) - dest) < 1e-5, (name, oc.getPar(name), dest)
    psiMin1, psiMax1 = oc.getPsiM()
    print(f"2dmoc state 1: psiMax {psiMax1:.6f} Sv, psiMin {psiMin1:.3e} Sv")
    assert abs(psiMax1 - 14.7) <= 1e-1, psiMax1
    assert abs(psiMin1) <= 1e-4, psiMin1
    for dest, ds in ((0.03, -0.5), (0.04, -0.5)):
        p.update({"continuation parameter": "Salinity Forcing", "destination 0": dest,
                  "initial step size": ds})
        assert Continuation(oc, p).run() == 0, dest
    psiMin2, psiMax2 = oc.getPsiM()
    print(f"2dmoc state 2: psiMax {psiMax2:.3e} Sv, psiMin {psiMin2:.6f} Sv")
    assert abs(psiMin1 + psiMax2) <= 1e-4, (psiMin1, psiMax2)
    assert abs(psiMax1 + psiMin2) <= 1e-4, (psiMax1, psiMin2)


def test_global1_continuation_step():
    """Config C5 (run/ocean at 1 degree, 11.2 M unknowns): one pseudo-arclength continuation
    step (Continuation.H:230-298, 587-813) from the committed near-solution branch state
    (bench_data/global1_cf05.npz, Combined Forcing 0.5): the Euler predictor, then the
    bordered Newton corrector converges (update below run/ocean's Newton tolerance 1e-2
    within the iteration limit) with a residual below the predicted one's, and Newton steps
    at the corrected parameter keep reducing it."""
    import os
    from iemic import config as cf
    from iemic.continuation import Continuation
    from iemic.ocean import Ocean
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with np.load(os.path.join(root, "bench_data", "global1_cf05.npz"), allow_pickle=False) as d:
        x0 = d["x"].astype(np.float64)
        par0 = float(d["par"])
    c = cf.preset("global1", mixing=1)
    oc = Ocean(c, solver_params={"FGMRES tolerance": 1e-4, "FGMRES iterations": 90, "FGMRES restarts": 20})
    oc.setState(x0)
    oc.setPar("Combined Forcing", par0)
    f_start = np.linalg.norm(oc.computeRHS())
    cont = Continuation(oc, {"continuation parameter": "Combined Forcing", "initial step size": 0.1,
                             "Newton tolerance": 1e-2, "normalize strategy": "N",
                             "corrector residual test": "D", "predictor bound": 3000.0,
                             "post processing": "never"})
    cont.initialize()
    cont.createInitialTangent()
    cont.store()
    assert cont.eulerPredictor() == 0
    f_pred = np.linalg.norm(oc.getRHS("V"))
    assert cont.newtonCorrector() == 0
    f_corr = cont.normRHStest
    print(f"C5 step: |F| start {f_start:.3e}, predicted {f_pred:.3e}, corrected {f_corr:.3e} "
          f"after {cont.newtonIter} Newton iterations, par {cont.par:.5f}")
    assert cont.par > par0
    assert f_corr < f_pred
    # then Newton at the corrected parameter (solves to 1e-8): the residual keeps dropping
    oc.solver_params["FGMRES tolerance"] = 1e-8
    seq = [f_corr]
    for _ in range(2):
        info = oc.newtonStep()
        seq.append(info.norm_f1)
    print("Newton sequence at the corrected parameter:", seq)
    assert seq[1] < seq[0] and seq[2] < seq[1]
    oc.close()
