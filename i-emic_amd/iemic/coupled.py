"""Atmosphere and CoupledModel host interfaces over the device library.

Mirrors the reference's Model surface for the coupled configuration (BASELINE config C4):

* ``Atmosphere`` -- src/atmosphere/Atmosphere.H: ``computeRHS``, ``computeJacobian``,
  ``applyMatrix``, ``applyPrecon``, ``setPar`` (AtmosLocal allParameters_,
  AtmosLocal.C:154-170), ``getState/setState``, ``setOceanTemperature``, ``getCommPars``.
* ``CoupledModel`` -- src/coupledmodel/CoupledModel.H: ``synchronize``, ``computeRHS``,
  ``computeJacobian``, ``applyMatrix``, ``solve`` (FGMRES + forward block Gauss-Seidel,
  "Preconditioning" = 'F'), ``setPar`` on every model.

Everything computes on the GPU through the C ABI (include/iemic.h); errors raise
``IemicError``.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .ocean import Ocean

__all__ = ["Atmosphere", "CoupledModel", "ATMOS_PARAMS"]

# XML parameter names (AtmosLocal::setParameters, AtmosLocal.C:109-151) -> struct fields
ATMOS_PARAMS = {
    "atmospheric density": "rhoa", "oceanic density": "rhoo",
    "atmospheric scale height": "hdima", "humidity scale height": "hdimq",
    "heat capacity": "cpa", "temperature eddy diffusivity": "D0",
    "humidity eddy diffusivity": "kappa", "radiative flux param A": "arad",
    "radiative flux param B": "brad", "solar constant": "sun0",
    "atmospheric absorption coefficient": "c0", "Dalton number": "ce",
    "exchange coefficient ch": "ch", "mean atmospheric surface wind speed": "uw",
    "background temperature atmosphere": "t0a", "background temperature ocean": "t0o",
    "background temperature seaice": "t0i", "temperature scale": "tdim",
    "atmos reference humidity": "q0", "atmos humidity scale": "qdim",
    "latent heat of vaporization": "lv", "horizontal velocity of the ocean": "udim",
    "radius of the earth": "r0dim", "reference albedo": "a0", "albedo excursion": "da",
    "restoring timescale tauf (in days)": "tauf_days",
    "restoring timescale tauc (in days)": "tauc_days",
    "melt temperature threshold (deg C)": "Tm",
    "rain/snow temperature threshold (deg C)": "Tr",
    "accumulation precipitation threshold (m/y)": "Pa",
    "melt threshold width (deg C)": "epm", "rain/snow threshold width (deg C)": "epr",
    "accumulation threshold width (m/y)": "epa",
}
# run/coupled/atmosphere_params.xml (the reference's coupled run) over the defaults
RUN_COUPLED_ATMOS = {
    "restoring timescale tauf (in days)": 10.0, "restoring timescale tauc (in days)": 1.0,
    "radiative flux param A": 216.0, "radiative flux param B": 1.5,
    "background temperature seaice": -5.0, "atmos reference humidity": 8e-3,
    "atmos humidity scale": 1e-3, "temperature eddy diffusivity": 3.4e6,
    "humidity eddy diffusivity": 3.1e6, "reference albedo": 0.3, "albedo excursion": 0.4,
    "melt temperature threshold (deg C)": 0.0, "melt threshold width (deg C)": 5.0,
    "accumulation precipitation threshold (m/y)": -100.0,
    "accumulation threshold width (m/y)": 5.0,
    "rain/snow temperature threshold (deg C)": 150.0, "rain/snow threshold width (deg C)": 5.0,
    "Combined Forcing": 1.0, "Solar Forcing": 1.0, "Humidity Forcing": 1.0,
    "Latent Heat Forcing": 1.0, "Albedo Forcing": 0.0,
}
# continuation parameters (AtmosLocal allParameters_)
ATMOS_PARS = ["Combined Forcing", "Solar Forcing", "Longwave Forcing", "Humidity Forcing",
              "Latent Heat Forcing", "Albedo Forcing", "T Eddy Diffusivity"]


class Atmosphere:
    """The atmosphere model on the ocean's grid and GPU (Atmosphere.C:13-165)."""

    def __init__(self, ocean: Ocean, params: Optional[dict] = None):
        p = _lib.AtmosParams()
        check(lib().iemic_atmos_default_params(C.byref(p)), "iemic_atmos_default_params")
        params = dict(params or {})
        ch_given = "exchange coefficient ch" in params
        for k, v in params.items():
            if k in ATMOS_PARAMS:
                setattr(p, ATMOS_PARAMS[k], float(v))
            elif k in ATMOS_PARS:
                p.par[ATMOS_PARS.index(k)] = float(v)
            else:
                raise KeyError(f"unknown atmosphere parameter {k!r}")
        if not ch_given:
            p.ch = 0.94 * p.ce          # AtmosLocal.C:122 default follows the Dalton number
        h = C.c_void_p()
        check(lib().iemic_atmos_create(C.byref(h), ocean._h, C.byref(p)), "iemic_atmos_create")
        self._h = h
        self._par = {name: float(p.par[i]) for i, name in enumerate(ATMOS_PARS)}
        self.ocean = ocean
        self.dim = lib().iemic_atmos_dim(h)
        self.n, self.m = ocean.cfg.n, ocean.cfg.m

    def close(self):
        if getattr(self, "_h", None):
            lib().iemic_atmos_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def setPar(self, name, value: float) -> None:
        idx = ATMOS_PARS.index(name) if isinstance(name, str) else int(name)
        check(lib().iemic_atmos_set_par(self._h, idx, float(value)), "iemic_atmos_set_par")
        self._par[ATMOS_PARS[idx]] = float(value)

    def getPar(self, name) -> float:
        return self._par[name if isinstance(name, str) else ATMOS_PARS[int(name)]]

    def setState(self, x: np.ndarray) -> None:
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.size == self.dim
        check(lib().iemic_atmos_set_state(self._h, ptr(x)), "iemic_atmos_set_state")

    def getState(self) -> np.ndarray:
        x = np.zeros(self.dim)
        check(lib().iemic_atmos_get_state(self._h, ptr(x)), "iemic_atmos_get_state")
        return x

    def setOceanTemperature(self, sst: np.ndarray) -> None:
        sst = np.ascontiguousarray(sst, dtype=np.float64)
        check(lib().iemic_atmos_set_sst(self._h, ptr(sst)), "iemic_atmos_set_sst")

    def computeRHS(self) -> np.ndarray:
        F = np.zeros(self.dim)
        check(lib().iemic_atmos_rhs(self._h, ptr(F)), "iemic_atmos_rhs")
        return F

    def computeJacobian(self) -> None:
        check(lib().iemic_atmos_jacobian(self._h), "iemic_atmos_jacobian")

    def applyMatrix(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.dim)
        check(lib().iemic_atmos_spmv(self._h, ptr(x), ptr(y)), "iemic_atmos_spmv")
        return y

    def applyPrecon(self, r: np.ndarray) -> np.ndarray:
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros(self.dim)
        check(lib().iemic_atmos_prec_apply(self._h, ptr(r), ptr(z)), "iemic_atmos_prec_apply")
        return z

    # ---- state files (Model::saveStateToFile + Atmosphere::additionalExports 1679-1714) ----
    def _sst(self) -> np.ndarray:
        """the ocean's surface temperature the atmosphere currently sees (interfaceT)."""
        oc = self.ocean
        c = oc.cfg
        x = oc.getState()
        return x.reshape(c.l, c.m, c.n, 6)[c.l - 1, :, :, 4].reshape(-1).copy()

    def saveStateToFile(self, filename: str, sst: Optional[np.ndarray] = None) -> None:
        """HDF5 in the reference's layout: State (Epetra_MultiVector), Parameters (the
        AtmosLocal continuation names), Grid, and the additional exports E and P
        (dimensional), sst and MaskGlobal/Surface.  Written by iemic.h5."""
        import math
        from . import h5
        c = self.ocean.cfg
        x = self.getState()
        cp = self.getCommPars()
        tdim, qdim, nuq, eta, dqso, Eo0 = cp[0], cp[1], cp[2], cp[3], cp[4], cp[7]
        sst = self._sst() if sst is None else np.asarray(sst, dtype=np.float64)
        pint, _, _, _ = self.integral_coeff()
        water = pint != 0.0
        q = x[1:3 * self.n * self.m:3]
        E = np.where(water, Eo0 + eta * qdim * ((tdim / qdim) * dqso * sst - q), 0.0)
        P = np.where(water, self.getPdist() * (Eo0 + eta * qdim * x[-1]), 0.0)
        xmin, xmax = math.radians(c.xmin), math.radians(c.xmax)
        ymin, ymax = math.radians(c.ymin), math.radians(c.ymax)
        dx, dy = (xmax - xmin) / c.n, (ymax - ymin) / c.m
        tree = {
            "State": {"Values": x.reshape(1, -1), "GlobalLength": np.array(len(x), dtype=np.int32),
                      "NumVectors": np.array(1, dtype=np.int32),
                      "__type__": np.array([b"Epetra_MultiVector"], dtype="S19")},
            "Parameters": {name: np.array(self._par[name]) for name in ATMOS_PARS},
            "Grid": {"n": np.array(c.n, dtype=np.int32), "m": np.array(c.m, dtype=np.int32),
                     "l": np.array(1, dtype=np.int32), "nun": np.array(3, dtype=np.int32),
                     "aux": np.array(1, dtype=np.int32), "xmin": np.array(xmin), "xmax": np.array(xmax),
                     "ymin": np.array(ymin), "ymax": np.array(ymax),
                     "x": xmin + dx * (np.arange(c.n) + 0.5), "y": ymin + dy * (np.arange(c.m) + 0.5)},
            "E": {"Values": E.reshape(1, -1)},
            "P": {"Values": P.reshape(1, -1)},
            "sst": {"Values": sst.reshape(1, -1)},
            "MaskGlobal": {"Surface": (~water).astype(np.int32)},
        }
        h5.write(filename, tree)

    def loadStateFromFile(self, filename: str) -> int:
        """Model::loadStateFromFile: the state and the known parameters; 1 if no file."""
        import os
        from . import h5
        if not os.path.exists(filename):
            return 1
        t = h5.read(filename)
        if "/State/Values" not in t:
            raise _lib.IemicError(f"The group <State> is not contained in hdf5 {filename}")
        x = np.asarray(t["/State/Values"][0], dtype=np.float64).reshape(-1)
        if x.size != self.dim:
            raise _lib.IemicError(f"{filename}: state of length {x.size}, this model has {self.dim}")
        self.setState(x)
        for path, (v, _) in t.items():
            if path.startswith("/Parameters/") and path.split("/", 2)[2] in ATMOS_PARS:
                self.setPar(path.split("/", 2)[2], float(np.asarray(v).reshape(-1)[0]))
        return 0

    def getCommPars(self) -> np.ndarray:
        out = np.zeros(18)
        check(lib().iemic_atmos_commpars(self._h, ptr(out)), "iemic_atmos_commpars")
        return out

    def getPdist(self) -> np.ndarray:
        out = np.zeros(self.n * self.m)
        check(lib().iemic_atmos_pdist(self._h, ptr(out)), "iemic_atmos_pdist")
        return out

    def jacobian_ell(self):
        """(values, columns) of the local rows, (dim-1) x 7; columns -1 unused."""
        val = np.zeros((self.dim - 1) * 7)
        col = np.zeros((self.dim - 1) * 7, dtype=np.int32)
        check(lib().iemic_atmos_export_ell(self._h, ptr(val), ptr(col, C.c_int)),
              "iemic_atmos_export_ell")
        return val.reshape(-1, 7), col.reshape(-1, 7)

    def integral_coeff(self):
        pint = np.zeros(self.n * self.m)
        area = C.c_double()
        ri, rp = C.c_int(), C.c_int()
        check(lib().iemic_atmos_integral_coeff(self._h, ptr(pint), C.byref(area), C.byref(ri),
                                               C.byref(rp)), "iemic_atmos_integral_coeff")
        return pint, area.value, ri.value, rp.value


class CoupledModel:
    """CoupledModel (CoupledModel.C:58-162) over one Ocean and one Atmosphere, solving
    scheme 'C' (fully coupled) with preconditioning 'F' (forward block Gauss-Seidel)."""

    def __init__(self, ocean: Ocean, atmos: Atmosphere, solver_params: Optional[dict] = None):
        h = C.c_void_p()
        check(lib().iemic_coupled_create(C.byref(h), ocean._h, atmos._h), "iemic_coupled_create")
        self._h = h
        self.ocean, self.atmos = ocean, atmos
        self.N = ocean.N + atmos.dim
        sp = {"FGMRES iterations": 200, "FGMRES tolerance": 1e-8, "FGMRES restarts": 4}
        if solver_params:
            sp.update(solver_params)
        self.solver_params = sp
        self.last_solve = None

    def close(self):
        if getattr(self, "_h", None):
            lib().iemic_coupled_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def setPar(self, name: str, value: float) -> None:
        """CoupledModel::setPar: every model that knows the parameter takes it."""
        from .config import PAR_INDEX
        if name in PAR_INDEX:
            self.ocean.setPar(name, value)
        if name in ATMOS_PARS:
            self.atmos.setPar(name, value)

    def synchronize(self) -> None:
        check(lib().iemic_coupled_synchronize(self._h), "iemic_coupled_synchronize")

    # ---- the Model surface Continuation / Newton drive (Model.H, Combined_MultiVec) ------
    def getState(self, mode: str = "C") -> np.ndarray:
        return np.concatenate([self.ocean.getState(), self.atmos.getState()])

    def setState(self, x: np.ndarray) -> None:
        x = np.asarray(x, dtype=np.float64)
        self.ocean.setState(x[:self.ocean.N])
        self.atmos.setState(x[self.ocean.N:])

    def getRHS(self, mode: str = "C") -> np.ndarray:
        F = getattr(self, "_F", None)
        if F is None:
            F = self.computeRHS()
        return F.copy() if mode == "C" else F

    def getPar(self, name: str) -> float:
        """CoupledModel::getPar: the first model that knows the parameter."""
        from .config import PAR_INDEX
        if name in PAR_INDEX:
            return self.ocean.getPar(name)
        return float(self.atmos.getCommPars()[16]) if name == "Combined Forcing" else 0.0

    def preProcess(self) -> None:
        self.ocean.preProcess()

    def postProcess(self) -> None:
        pass

    def computeRHS(self) -> np.ndarray:
        Fo = np.zeros(self.ocean.N)
        Fa = np.zeros(self.atmos.dim)
        check(lib().iemic_coupled_rhs(self._h, ptr(Fo), ptr(Fa)), "iemic_coupled_rhs")
        self._F = np.concatenate([Fo, Fa])
        return self._F

    def computeJacobian(self) -> None:
        check(lib().iemic_coupled_jacobian(self._h), "iemic_coupled_jacobian")

    def applyMatrix(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.N)
        check(lib().iemic_coupled_spmv(self._h, ptr(x), ptr(y)), "iemic_coupled_spmv")
        return y

    def newtonStep(self, allow_unconverged: bool = False) -> dict:
        """One Newton iteration of the coupled model as the reference's Newton /
        Continuation drives it (src/newton/Newton.H:76-123): F(x), J(x), solve J dx = -F,
        x += dx, F(x + dx).  Returns the residual norms and the solve record.  The update
        is applied either way; a solve that missed its tolerance raises IemicError (as
        Ocean.newtonStep does) unless allow_unconverged."""
        F0 = self.computeRHS()
        self.computeJacobian()
        dx = self.solve(-F0)
        xo = self.ocean.getState() + dx[:self.ocean.N]
        xa = self.atmos.getState() + dx[self.ocean.N:]
        self.ocean.setState(xo)
        self.atmos.setState(xa)
        F1 = self.computeRHS()
        if not self.last_solve.converged and not allow_unconverged:
            sp = self.solver_params
            method = (f"IDR({int(sp.get('IDR s', 4))})" if str(sp.get("Solver", "FGMRES")).upper() == "IDR"
                      else "FGMRES")
            raise _lib.IemicError(
                f"coupled Newton step: {method} did not converge ({self.last_solve.iters} steps, "
                f"relative residual {self.last_solve.explicit_rel_res:.3e}); the update was applied")
        return dict(norm_f0=self._norm(F0), norm_f1=self._norm(F1),
                    iters=int(self.last_solve.iters), converged=bool(self.last_solve.converged),
                    explicit_rel_res=float(self.last_solve.explicit_rel_res))

    def _norm(self, v: np.ndarray) -> float:
        """2-norm of a coupled vector [ocean (global, owned rows filled) | atmosphere]: on
        several ranks the ocean's owned rows summed over the ranks, the (replicated)
        atmosphere once."""
        oc = self.ocean
        if oc.layout()["nranks"] == 1:
            return float(np.linalg.norm(v))
        rows = oc.owned_rows()
        s = np.array([float(np.dot(v[rows], v[rows]))])
        check(lib().iemic_allreduce_sum(oc._h, ptr(s), 1), "iemic_allreduce_sum")
        va = v[oc.N:]
        return float(np.sqrt(s[0] + np.dot(va, va)))

    def solve(self, b: np.ndarray) -> np.ndarray:
        sp = self.solver_params
        opt = self.ocean._krylov()          # the ocean's block preconditioner settings
        opt.tol = float(sp["FGMRES tolerance"])
        opt.krylov_dim = int(sp["FGMRES iterations"])
        opt.max_restarts = int(sp["FGMRES restarts"])
        opt.prec = int(sp.get("Preconditioner", opt.prec))
        # "Solver": FGMRES (CoupledModel::FGMRESSolve) or IDR (config C4: IDR(4),
        # IDRSolver.H:109-340)
        opt.method = 1 if str(sp.get("Solver", "FGMRES")).upper() == "IDR" else 0
        opt.idr_s = int(sp.get("IDR s", 4))
        opt.idr_angle = float(sp.get("IDR angle", 0.7))
        opt.idr_replace = int(bool(sp.get("IDR replace residuals", False)))
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.zeros(self.N)
        info = _lib.SolveInfo()
        check(lib().iemic_coupled_solve(self._h, ptr(b), ptr(x), C.byref(opt), C.byref(info)),
              "iemic_coupled_solve")
        self.last_solve = info
        return x
