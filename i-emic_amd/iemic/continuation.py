"""Pseudo-arclength continuation over the GPU ocean model.

Restates ``Continuation<Model>`` (src/continuation/Continuation.H) on the Model surface
the reference drives (``computeRHS``, ``computeJacobian``, ``solve``, ``applyMatrix``,
``getState/getRHS/getSolution``, ``getPar/setPar``, ``preProcess/postProcess``): Euler
predictor, Newton corrector on the bordered system with two solves against the same
Jacobian (Continuation.H:587-813; the preconditioner is built once per Jacobian and reused
by both solves), finite-difference dF/dpar (389-418), secant/Euler tangents and their
normalisation (421-544), step-size control (952-982), reset/restore (1004-1050) and the
secant landing on destinations (858-933).  Parameter names and defaults are the
reference's (getDefaultInitParameters, Continuation.H:1330-1366).

Vector algebra goes through an ops object (the reference's Utils::dot / norm / update on
Epetra vectors of the solve map): a model with ``vec_ops()`` (the GPU ``Ocean``) supplies
device vectors in HBM whose dots and norms are summed over its ranks, so the state, tangent,
dF/dpar and the corrector's two solutions never leave the GPU and the same driver runs on
every rank of a decomposed model; other models (host numpy vectors in the reference row
order) get ``HostOps``.  The ops are functional (every result is a new vector), which is
how the code below reads Continuation.H's Epetra Update calls.  Eigenvalue analysis (JDQZ)
and user monitors are not restated.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

DEFAULTS = {
    "continuation parameter": "Combined Forcing",
    "initial step size": 1.0e-2, "minimum step size": 1.0e-8, "maximum step size": 1.0e3,
    "increase step size": 1.25, "decrease step size": 2.0, "epsilon increment": 1.0e-5,
    "maximum number of steps": -1, "maximum Newton iterations": 7,
    "minimum Newton iterations": 1, "optimal Newton iterations": 3.5,
    "Newton tolerance": 1.0e-4, "destination tolerance": 1.0e-7,
    "detection of special points": "D", "state tangent scaling": 1.0,
    "normalize strategy": "N", "reject failed iteration": True,
    "give up at minimum step size": True, "enable Newton Chord hybrid solve": False,
    "tangent type": "S", "corrector residual test": "D", "initial tangent type": "E",
    "post processing": "at every point", "predictor bound": 1e3,
    # Continuation.H:1336-1338
    "enable backtracking": False, "backtracking steps": 0, "backtracking increase": 0.0,
}


def _sgn(x: float) -> int:
    return (x > 0) - (x < 0)


class HostOps:
    """Vector algebra and model access for a model with host numpy vectors."""

    def __init__(self, model):
        self.model = model

    @staticmethod
    def lincomb(a, x, b=0.0, y=None):
        return a * x + b * y if y is not None else a * x

    @staticmethod
    def copy(x):
        return x.copy()

    @staticmethod
    def dot(x, y) -> float:
        return float(np.dot(x, y))

    @staticmethod
    def norm(x) -> float:
        return float(np.linalg.norm(x))

    @staticmethod
    def norm_inf(x) -> float:
        return float(np.max(np.abs(x)))

    def state(self):
        return self.model.getState("C")

    def set_state(self, v):
        self.model.setState(v)

    def rhs(self):
        self.model.computeRHS()
        return self.model.getRHS("C")

    def solve(self, b):
        return self.model.solve(b).copy()


def ops_for(model):
    """DeviceOps for a model that keeps its vectors on the GPU, HostOps otherwise."""
    return model.vec_ops() if hasattr(model, "vec_ops") else HostOps(model)


@dataclass
class _Storage:
    state0: Optional[np.ndarray] = None
    state00: Optional[np.ndarray] = None
    stateDot0: Optional[np.ndarray] = None
    par0: float = 0.0
    par00: float = 0.0
    parDot0: float = 0.0
    ds0: float = 0.0
    ds00: float = 0.0


@dataclass
class StepRecord:
    step: int
    par: float
    ds: float
    norm_x: float
    norm_f: float
    newton_iters: int


class Continuation:
    """``Continuation<Model>`` (Continuation.H) for a Model with the Ocean surface."""

    def __init__(self, model, params: Optional[dict] = None):
        p = dict(DEFAULTS)
        if params:
            p.update(params)
        self.model = model
        self.ops = ops_for(model)
        self.p = p
        self.parName = p["continuation parameter"]
        self.dsInit = float(p["initial step size"])
        self.dsMin = float(p["minimum step size"])
        self.dsMax = float(p["maximum step size"])
        self.scale2 = float(p["decrease step size"])
        self.epsilon = float(p["epsilon increment"])
        self.maxSteps = int(p["maximum number of steps"])
        self.maxNewton = int(p["maximum Newton iterations"])
        self.minNewton = int(p["minimum Newton iterations"])
        self.optNewton = float(p["optimal Newton iterations"])
        self.newtonTol = float(p["Newton tolerance"])
        self.destTol = float(p["destination tolerance"])
        self.detectMode = p["detection of special points"]
        self.tanScaling = float(p["state tangent scaling"])
        self.normalizeStrategy = p["normalize strategy"]
        self.rejectFailed = bool(p["reject failed iteration"])
        self.giveUpAtdsMin = bool(p["give up at minimum step size"])
        self.chordHybrid = bool(p["enable Newton Chord hybrid solve"])
        self.tangentType = p["tangent type"]
        self.residualTest = p["corrector residual test"]
        self.initialTangent = p["initial tangent type"]
        self.postProcessMode = p["post processing"]
        self.predictorBound = float(p["predictor bound"])
        self.backTracking = bool(p["enable backtracking"])
        self.numBackTrackingSteps = int(p["backtracking steps"])
        self.backTrackIncrease = float(p["backtracking increase"])
        self.backTrack = 0
        self.destinations = []
        for i in range(999):
            d = p.get(f"destination {i}")
            if d is None or d == -999.0:
                break
            self.destinations.append(float(d))
        self.destinationsBackup = list(self.destinations)
        self.history: list[StepRecord] = []

    # ---- helpers -------------------------------------------------------------------
    def _norm(self, v):
        return self.ops.norm(v)

    def _set_state(self, x):
        self.ops.set_state(x)

    # ---- Continuation.H:1158-1230 initialize ----------------------------------------
    def initialize(self):
        self.ds = self.dsInit
        self.Fcur = self.ops.rhs()
        self.state = self.ops.state()
        self.rhs = self.Fcur
        self.par = self.model.getPar(self.parName)
        self.st = _Storage(ds0=self.ds, ds00=self.ds, par0=self.par, par00=self.par,
                           parDot0=0.0, state0=self.state)
        self.destinations = list(self.destinationsBackup)
        self.signMonitor = [0] * len(self.destinations)
        self.secant = False
        N = getattr(self.model, "N", None) or len(self.state)
        if self.normalizeStrategy == "O":
            self.zeta = 1.0 / N
        else:
            self.zeta = self.tanScaling / N
        self.newtonIter = 0
        self.sumNewtonIter = 0
        self.parDot = 0.0
        self.stateDot = None
        self.step_ = 0
        self.resetCounter = 0
        self.reachedLastDest = False
        self.abortFlag = False
        self.fixStepSize = False
        self.dsStart = self.ds

    # ---- 389-418 ---------------------------------------------------------------------
    def computeDFDPar(self, mode: str):
        # mode "A": the residual of the current state is the last one computed (Fcur)
        if mode == "F":
            self.Fcur = self.ops.rhs()
        self.rhsCopy = self.Fcur
        self.model.setPar(self.parName, self.par + self.epsilon)
        Fe = self.ops.rhs()
        self.model.setPar(self.parName, self.par)
        self.dFdPar = self.ops.lincomb(1.0 / self.epsilon, Fe, -1.0 / self.epsilon, self.rhsCopy)

    # ---- 300-384 ---------------------------------------------------------------------
    def createInitialTangent(self):
        self.computeDFDPar("F")
        if self.initialTangent in ("E", "S"):
            self.model.preProcess()
            self.model.computeJacobian()
            self.stateDot = self.ops.solve(self.ops.lincomb(-1.0, self.dFdPar))
        else:
            self.stateDot = self.ops.lincomb(-1.0, self.dFdPar)
        self.normalize()

    # ---- 497-544 ---------------------------------------------------------------------
    def normalize(self):
        ops = self.ops
        if self.normalizeStrategy == "O":
            self.zeta = self.tanScaling / self._norm(self.stateDot)
            self.stateDot = ops.lincomb(self.zeta, self.stateDot)
            nrm = self._norm(self.stateDot)
            normComb = math.sqrt(nrm * nrm + 1)
            self.stateDot = ops.lincomb(1.0 / normComb, self.stateDot)
            self.parDot = 1.0 / normComb
        else:
            nrm = self._norm(self.stateDot)
            normComb = math.sqrt(self.zeta * nrm * nrm + 1)
            self.parDot = 1.0 / normComb
            self.stateDot = ops.lincomb(self.parDot, self.stateDot)

    # ---- 421-494 ---------------------------------------------------------------------
    def createTangent(self, mode: str):
        ops = self.ops
        if mode == "S":
            state = ops.state()
            self.stateDot = ops.lincomb(1.0 / self.st.ds0, state, -1.0 / self.st.ds0, self.st.state0)
            self.par = self.model.getPar(self.parName)
            self.parDot = (self.par - self.st.par0) / self.st.ds0
        else:
            if self.chordHybrid:
                self.computeDFDPar("F")
                self.model.computeJacobian()
                self.stateDot = ops.solve(ops.lincomb(-1.0, self.dFdPar))
            elif self.newtonIter != 0:
                self.stateDot = ops.lincomb(-1.0, self.stateDot)
            self.normalize()

    # ---- 547-583 ---------------------------------------------------------------------
    def eulerPredictor(self) -> int:
        self.state = self.ops.lincomb(1.0, self.state, self.ds, self.stateDot)
        self._set_state(self.state)
        self.par = self.par + self.ds * self.parDot
        self.model.setPar(self.parName, self.par)
        self.Fcur = self.ops.rhs()
        return 1 if self._norm(self.Fcur) > self.predictorBound else 0

    # ---- 587-813 ---------------------------------------------------------------------
    def newtonCorrector(self) -> int:
        ops = self.ops
        res = 100.0
        y = None
        self.newtonIter = 0
        while self.newtonIter < self.maxNewton:
            mode = "F" if self.newtonIter == 0 else "A"
            self.computeDFDPar(mode)
            R = ops.lincomb(-1.0, self.rhsCopy)
            self.normRHS = self._norm(self.rhsCopy)
            stateDiff = ops.lincomb(1.0, ops.state(), -1.0, self.st.state0)
            parDiff = self.par - self.st.par0
            if self.normalizeStrategy == "O":
                rbp = self.ds - ops.dot(self.stateDot, stateDiff) * self.zeta - self.parDot * parDiff
            else:
                rbp = (self.ds * self.ds) - ops.dot(stateDiff, stateDiff) * self.zeta - parDiff * parDiff
            self.model.computeJacobian()
            # two solves with the same Jacobian (the preconditioner is computed once)
            if not self.chordHybrid:
                y = ops.solve(self.dFdPar)
            z = ops.solve(R)
            if self.normalizeStrategy == "O":
                if self.chordHybrid:
                    parDir = ((rbp - self.zeta * ops.dot(self.stateDot, z)) /
                              (self.parDot + self.zeta * ops.dot(self.stateDot, self.stateDot)))
                else:
                    parDir = ((rbp - self.zeta * ops.dot(self.stateDot, z)) /
                              (self.parDot - self.zeta * ops.dot(self.stateDot, y)))
            else:
                if self.chordHybrid:
                    parDir = ((rbp - 2 * self.zeta * ops.dot(stateDiff, z)) /
                              (2 * parDiff + 2 * (self.zeta / parDiff) * ops.dot(stateDiff, stateDiff)))
                else:
                    parDir = ((rbp - 2 * self.zeta * ops.dot(stateDiff, z)) /
                              (2 * parDiff - 2 * self.zeta * ops.dot(stateDiff, y)))
            stateDir = (ops.lincomb(1.0, z, parDir, self.stateDot) if self.chordHybrid
                        else ops.lincomb(1.0, z, -parDir, y))
            self.state = ops.lincomb(1.0, ops.state(), 1.0, stateDir)
            self._set_state(self.state)
            self.par = self.par + parDir
            self.model.setPar(self.parName, self.par)
            self.newtonIter += 1
            self.sumNewtonIter += 1
            self.Fcur = ops.rhs()
            self.normRHStest = self._norm(self.Fcur)
            if self.normRHStest > self.predictorBound:
                return 1
            # no decrease: backtracking along the Newton direction (Continuation.H:724-731)
            if self.backTracking and self.normRHS < self.normRHStest:
                if self.runBackTracking(stateDir, parDir):
                    return 1
            n0 = self._norm(self.st.state0)
            if self._norm(stateDir) > 1e3 * n0 and n0 > 0:
                return 1
            if self.residualTest == "R":
                res = self.normRHStest
            else:
                res = max(abs(parDir), ops.norm_inf(stateDir))
            if res < self.newtonTol and self.newtonIter >= self.minNewton:
                break
        if not self.chordHybrid and y is not None:
            self.stateDot = y
        if res > self.newtonTol and self.rejectFailed:
            return 1
        return 0

    # ---- 816-855 ---------------------------------------------------------------------
    def runBackTracking(self, stateDir, parDir) -> int:
        """Halve the step back along (stateDir, parDir) until ||F|| drops below
        increase * ||F_old|| or the step budget is spent."""
        reduction = -1.0 / 2
        increase = self.backTrackIncrease
        self.backTrack = 0
        while self.backTrack != self.numBackTrackingSteps:
            if self.normRHStest < self.normRHS * increase:
                break
            self.state = self.ops.lincomb(1.0, self.ops.state(), reduction, stateDir)
            self._set_state(self.state)
            self.par = self.par + reduction * parDir
            self.model.setPar(self.parName, self.par)
            self.Fcur = self.ops.rhs()
            self.normRHStest = self._norm(self.Fcur)
            reduction /= 2.0
            self.backTrack += 1
        if self.normRHStest > self.normRHS * increase and self.numBackTrackingSteps > 0:
            return 1
        return 0

    # ---- 1052-1090 store / restore ----------------------------------------------------
    def store(self):
        self.st.state00 = self.st.state0
        self.st.state0 = self.ops.state()
        self.st.stateDot0 = self.stateDot          # the ops never modify a vector in place
        self.st.par00 = self.st.par0
        self.st.par0 = self.model.getPar(self.parName)
        self.st.ds00 = self.st.ds0
        self.st.ds0 = self.ds
        self.st.parDot0 = self.parDot

    def restore(self):
        self.state = self.st.state0
        self._set_state(self.state)
        self.stateDot = self.st.stateDot0
        self.par = self.st.par0
        self.model.setPar(self.parName, self.par)
        self.parDot = self.st.parDot0
        self.ds = self.st.ds0

    def reset(self):
        self.step_ -= 1
        self.restore()
        s = _sgn(self.ds)
        self.ds = s * max(abs(self.ds) / self.scale2, abs(self.dsMin))
        self.resetCounter += 1
        self.fixStepSize = True
        if abs(self.ds) <= abs(self.dsMin) and (self.resetCounter >= 100 or self.giveUpAtdsMin):
            self.abortFlag = True

    # ---- 952-982 ---------------------------------------------------------------------
    def adjustStep(self):
        if self.secant or self.fixStepSize:
            self.fixStepSize = False
            return
        factor = self.optNewton / float(self.newtonIter)
        factor = min(max(factor, 0.5), 2.0)
        self.ds *= factor
        if abs(self.ds) > abs(self.dsMax):
            self.ds = _sgn(self.ds) * abs(self.dsMax)
        if abs(self.ds) < abs(self.dsMin):
            self.ds = _sgn(self.ds) * abs(self.dsMin)

    # ---- 858-933 ---------------------------------------------------------------------
    def detect(self):
        if not self.destinations:
            return
        dest = self.destinations[0]
        self.par = self.model.getPar(self.parName)
        if self.detectMode == "D":
            f0, f1 = self.st.par0 - dest, self.par - dest
        else:
            f0, f1 = self.st.parDot0, self.parDot
        if self.signMonitor[0] == 0:
            self.signMonitor[0] = _sgn(f1)
        if self.signMonitor[0] != _sgn(f1) and not self.secant:
            self.secant = True
            self.dsStart = self.ds
        else:
            self.signMonitor[0] = _sgn(f1)
        if self.secant:
            self.ds = -f1 * self.ds / (f1 - f0)
            self.createTangent("S")
        if self.secant and abs(f1) < self.destTol:
            self.secant = False
            self.ds = self.dsStart
            self.fixStepSize = True
            self.destinations.pop(0)
            self.signMonitor.pop(0)
            if not self.destinations:
                self.reachedLastDest = True
            else:
                self.signMonitor[0] = _sgn(self.par - self.destinations[0])

    # ---- 230-298 ---------------------------------------------------------------------
    def step(self) -> int:
        self.model.preProcess()
        if self.eulerPredictor():
            return 1
        if self.newtonCorrector():
            return 1
        self.createTangent(self.tangentType)
        if self.postProcessMode == "at every point":
            self.model.postProcess()
        return 0

    # ---- 184-228 ---------------------------------------------------------------------
    def run(self) -> int:
        self.initialize()
        self.createInitialTangent()
        while not self.reachedLastDest and self.step_ != self.maxSteps and not self.abortFlag:
            self.step_ += 1
            self.store()
            if self.step():
                self.reset()
                continue
            self.history.append(StepRecord(self.step_, self.par, self.ds,
                                           self._norm(self.ops.state()),
                                           self.normRHStest, self.newtonIter))
            self.detect()
            self.adjustStep()
        if self.abortFlag:
            return 1
        if self.postProcessMode != "at every point":
            self.model.postProcess()
        return 0
