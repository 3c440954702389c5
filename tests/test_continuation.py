"""Pseudo-arclength continuation (iemic.continuation, restating Continuation.H).

* CPU: the driver on small analytic models (a linear branch and the monotone nonlinear
  branch of x^3 + x = lambda) lands on its destination with the reference's defaults.
* GPU: the reference's own regression test src/tests/reft_ocean.C -- the 16x16x16
  gateway ocean (test/ocean/reft_ocean_params.xml) continued in Combined Forcing from 0 to
  the destination 0.02 with reft_continuation_params.xml -- reproduces the stored end
  state test/ocean/ocean_reference.h5 (decoded in tests/golden/gateway16.npz): the 2-norms
  of the u, v, T and S fields agree to 1e-3, the reference test's own criterion
  (reft_ocean.C:52-85).
"""
import numpy as np
import pytest

from iemic.continuation import Continuation


class ToyModel:
    """Model surface over F(x; lam) (dense, numpy)."""

    def __init__(self, F, J, n, par=0.0):
        self.F, self.J = F, J
        self.x = np.zeros(n)
        self.lam = par
        self._F = F(self.x, par)
        self._sol = np.zeros(n)

    def computeRHS(self):
        self._F = self.F(self.x, self.lam)
        return self._F

    def computeJacobian(self):
        self._J = self.J(self.x, self.lam)

    def solve(self, b):
        self._sol = np.linalg.solve(self._J, b)
        return self._sol

    def getState(self, mode="C"):
        return self.x.copy() if mode == "C" else self.x

    def setState(self, x):
        self.x = np.array(x, dtype=float)

    def getRHS(self, mode="C"):
        return self._F.copy() if mode == "C" else self._F

    def getSolution(self, mode="C"):
        return self._sol.copy() if mode == "C" else self._sol

    def getPar(self, name):
        return self.lam

    def setPar(self, name, v):
        self.lam = float(v)

    def preProcess(self):
        pass

    def postProcess(self):
        pass


def test_linear_branch_reaches_destination():
    c = np.array([1.0, -2.0, 0.5])
    m = ToyModel(lambda x, l: x - l * c, lambda x, l: np.eye(3), 3)
    cont = Continuation(m, {"destination 0": 1.0, "initial step size": 0.1,
                            "maximum number of steps": 200, "destination tolerance": 1e-10})
    assert cont.run() == 0
    assert abs(m.lam - 1.0) < 1e-10
    np.testing.assert_allclose(m.x, c, atol=1e-9)


def test_nonlinear_branch():
    """F = x^3 + x - lam: a monotone nonlinear branch x(lam), continued to lam = 2."""
    m = ToyModel(lambda x, l: x ** 3 + x - l, lambda x, l: np.diag(3 * x ** 2 + 1), 2)
    cont = Continuation(m, {"destination 0": 2.0, "initial step size": 0.05,
                            "maximum number of steps": 500, "destination tolerance": 1e-9,
                            "Newton tolerance": 1e-10})
    assert cont.run() == 0
    assert abs(m.lam - 2.0) < 1e-9
    np.testing.assert_allclose(m.x, 1.0, atol=1e-8)    # x^3 + x = 2 -> x = 1
    assert len(cont.history) > 3


REFT_CONTINUATION = {                 # test/ocean/reft_continuation_params.xml
    "continuation parameter": "Combined Forcing", "initial step size": 2.0e-3,
    "minimum step size": 1.0e-8, "maximum step size": 1.0e-1, "destination 0": 0.02,
    "maximum number of steps": 20, "optimal Newton iterations": 3.0,
    "Newton tolerance": 1.0e-2, "destination tolerance": 1.0e-4,
    "post processing": "at final point", "epsilon increment": 1.0e-5,
    "state tangent scaling": 1.0e-3, "reject failed iteration": True,
    "enable Newton Chord hybrid solve": False, "tangent type": "S",
    "predictor bound": 3000.0}


@pytest.mark.gpu
def test_reft_ocean_continuation_matches_reference_h5():
    from helpers import golden
    from iemic import config as cf
    from iemic.ocean import Ocean
    c = cf.preset("gateway16")          # reft_ocean_params.xml (Mixing 2, Rho Mixing off, ...)
    c.start_params["Combined Forcing"] = 0.0
    oc = Ocean(c, solver_params={"FGMRES tolerance": 1e-6, "FGMRES iterations": 500,
                                 "FGMRES restarts": 0})     # test/ocean/solver_params.xml
    cont = Continuation(oc, REFT_CONTINUATION)
    assert cont.run() == 0
    assert abs(oc.getPar("Combined Forcing") - 0.02) < 1e-4
    x = oc.getState()
    y = golden("gateway16")["h5_x"]
    for var in (0, 1, 4, 5):                # u, v, T, S (reft_ocean.C:58)
        nx, ny = np.linalg.norm(x[var::6]), np.linalg.norm(y[var::6])
        assert abs(nx - ny) <= 1e-3, (var, nx, ny)


def test_backtracking_halves_the_step():
    """Continuation.H:816-855: with no decrease of ||F|| the corrector step is halved back
    (cumulative reductions -1/2, -1/4, ...) until ||F|| < increase * ||F_old||."""
    m = ToyModel(lambda x, l: x ** 3 - l, lambda x, l: np.diag(3 * x ** 2), 1, par=1.0)
    cont = Continuation(m, {"enable backtracking": True, "backtracking steps": 3,
                            "backtracking increase": 1.0})
    cont.initialize()
    m.x = np.array([10.0])
    cont.state = m.x.copy()
    m.computeRHS()
    cont.normRHS = 1.0                      # pretend the old residual was small
    cont.normRHStest = float(np.linalg.norm(m.computeRHS()))
    stateDir = np.array([8.0])
    assert cont.runBackTracking(stateDir, 0.0) == 1     # never below 1.0: fails after 3 steps
    assert cont.backTrack == 3
    np.testing.assert_allclose(m.x, [10.0 - 4.0 - 2.0 - 1.0])
    # a step that already decreases enough is left alone
    m.x = np.array([1.0]); cont.normRHS = 5.0; cont.normRHStest = 0.0
    assert cont.runBackTracking(stateDir, 0.0) == 0 and cont.backTrack == 0
