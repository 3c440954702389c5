"""Ocean-shaped host interface over the device library.

Mirrors the Model surface the reference's Continuation and transient Newton drive
(``src/ocean/Ocean.H``; calls listed in SURVEY.md §8b.1): ``computeRHS``,
``computeJacobian``, ``solve``, ``applyMatrix``, ``applyPrecon``, ``buildPreconditioner``,
``getState/getSolution/getRHS('C'|'V')``, ``setPar/getPar``, ``preProcess``,
``postProcess``.  Parameter names are THCM's (``THCM::par2int``, THCM.C:1754-1807) and
Belos settings keep Ocean's names ("FGMRES iterations", "FGMRES tolerance",
"FGMRES restarts"; defaults Ocean.C:2232-2237).

Everything computes on the GPU through the C ABI; the state, Jacobian, residual and
Krylov basis stay resident in HBM.  Errors raise ``IemicError`` (the reference throws).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import IemicError, check, lib, ptr
from .config import PAR_INDEX, THCMConfig, landmask

__all__ = ["Ocean", "IemicError", "DeviceVec", "DeviceOps"]


class DeviceVec:
    """One fp64 vector in HBM in the model's internal layout (iemic_layout: owned rows of
    this rank's subdomain), an Epetra_Vector of the solve map.  Buffers are recycled through
    the owning Ocean's pool, so the continuation's vector algebra allocates nothing per step."""
    __slots__ = ("oc", "p")

    def __init__(self, oc: "Ocean"):
        self.oc = oc
        self.p = oc._vec_take()

    def __del__(self):
        try:
            self.oc._vec_give(self.p)
        except Exception:
            pass


class DeviceOps:
    """Continuation.H's vector algebra on device vectors (Utils::dot / norm / update over the
    solve map; collective over the Ocean's ranks).  The functional forms mirror the host ops
    of iemic.continuation, so the continuation code is the same for both."""

    def __init__(self, oc: "Ocean"):
        self.oc = oc

    def _h(self):
        return self.oc._h

    def lincomb(self, a, x, b=0.0, y=None) -> DeviceVec:
        z = DeviceVec(self.oc)
        check(lib().iemic_vec_update(self._h(), float(a), x.p, float(b), y.p if y is not None else None,
                                     0.0, z.p), "iemic_vec_update")
        return z

    def copy(self, x) -> DeviceVec:
        return self.lincomb(1.0, x)

    def dot(self, x, y) -> float:
        v = C.c_double()
        check(lib().iemic_vec_dot(self._h(), x.p, y.p, C.byref(v)), "iemic_vec_dot")
        return v.value

    def norm(self, x) -> float:
        import math
        return math.sqrt(self.dot(x, x))

    def norm_inf(self, x) -> float:
        v = C.c_double()
        check(lib().iemic_vec_norm_inf(self._h(), x.p, C.byref(v)), "iemic_vec_norm_inf")
        return v.value

    # model side: state, residual, solve without host copies
    def state(self) -> DeviceVec:
        v = DeviceVec(self.oc)
        check(lib().iemic_state_vec(self._h(), v.p, 0), "iemic_state_vec")
        return v

    def set_state(self, v) -> None:
        check(lib().iemic_state_vec(self._h(), v.p, 1), "iemic_state_vec")

    def rhs(self) -> DeviceVec:
        """F(state) (Ocean::computeRHS + getRHS('C'))."""
        v = DeviceVec(self.oc)
        check(lib().iemic_rhs_vec(self._h(), v.p), "iemic_rhs_vec")
        return v

    def solve(self, b) -> DeviceVec:
        """J x = b (Ocean::solve on the device; the preconditioner is built once per Jacobian)."""
        oc = self.oc
        oc.buildPreconditioner()
        x = DeviceVec(oc)
        k = oc._krylov()
        info = _lib.SolveInfo()
        check(lib().iemic_solve_dev(self._h(), b.p, x.p, C.byref(k), C.byref(info)), "iemic_solve_dev")
        oc.last_solve = info
        if oc.solve_hook is not None:
            oc.solve_hook(info)
        return x

    def to_host(self, v) -> np.ndarray:
        """global reference-ordered host vector (this rank's rows; 0 elsewhere)"""
        out = np.zeros(self.oc.N)
        check(lib().iemic_vec_to_ref(self._h(), v.p, ptr(out)), "iemic_vec_to_ref")
        return out

    def from_host(self, x: np.ndarray) -> DeviceVec:
        v = DeviceVec(self.oc)
        x = np.ascontiguousarray(x, dtype=np.float64)
        check(lib().iemic_vec_from_ref(self._h(), ptr(x), v.p), "iemic_vec_from_ref")
        return v


class Ocean:
    """One THCM ocean model instance on one GPU (Ocean.C:63-213)."""

    def __init__(self, cfg: THCMConfig, landm: Optional[np.ndarray] = None, device: int = 0,
                 analyze_jacobian: bool = True, solver_params: Optional[dict] = None,
                 rank: int = 0, nranks: int = 1, comm_id: Optional[bytes] = None,
                 local_group=None, npx: Optional[int] = None, transport=None):
        """rank/nranks: the Decomp2D subdomain of this rank (one Ocean per GPU); comm_id is
        the RCCL unique id of rank 0 (Ocean.unique_id()), shared by the caller; transport:
        a host transport instead of RCCL (iemic.transport.GlooTransport); local_group: the
        in-process test facility.  npx: x parts (0: the reference's Decomp2D factorisation,
        1: latitude bands, the default on every transport: x cuts through the zonal flow cost
        FGMRES steps)."""
        cfg.validate()
        self.cfg = cfg
        L = landmask(cfg) if landm is None else landm
        L = np.ascontiguousarray(L, dtype=np.int32).reshape(-1)
        self._grid = _lib.grid_from_config(cfg, device=device, analyze_jacobian=analyze_jacobian)
        h = C.c_void_p()
        self._transport = transport
        if local_group is not None:
            rc = lib().iemic_create_local_2d(C.byref(h), C.byref(self._grid), ptr(L, C.c_int),
                                             local_group, rank, nranks, 1 if npx is None else npx)
        elif transport is not None:
            rc = lib().iemic_create_transport(C.byref(h), C.byref(self._grid), ptr(L, C.c_int), rank,
                                              nranks, 1 if npx is None else npx, C.byref(transport.c))
        elif nranks > 1:
            d = _lib.Dist(rank, nranks)
            d.npx = 1 if npx is None else npx
            C.memmove(d.id, comm_id, 128)
            rc = lib().iemic_create_dist(C.byref(h), C.byref(self._grid), ptr(L, C.c_int),
                                         C.byref(d))
        else:
            rc = lib().iemic_create(C.byref(h), C.byref(self._grid), ptr(L, C.c_int))
        check(rc, "iemic_create")
        self._vlive = 0                 # DeviceVecs handed out and not yet given back
        self._closing = False
        self._h = h
        self.N = lib().iemic_nrows(h)
        # Belos solver parameters (Ocean::getDefaultInitParameters, Ocean.C:2232-2237)
        sp = {"FGMRES iterations": 500, "FGMRES tolerance": 1e-8, "FGMRES restarts": 0,
              "Preconditioner": 2, "TS sweeps": 12, "Orthogonalization": "DCGS2",
              "Dyn iterations": 4, "Dyn damping": 0.95, "Dyn minimal residual": False, "TS multigrid cycles": 1,
              "Solver": "FGMRES", "IDR s": 4, "IDR angle": 0.7, "IDR replace residuals": False,
              "Multigrid sweeps": 1, "TS after dyn pass": 0,
              "Schur passes": 2}
        if solver_params:
            sp.update(solver_params)
        self.solver_params = sp
        self._recomp_prec = True
        for idx, v in cfg.par_list():
            self.setPar(idx, v)
        self._x = np.zeros(self.N)
        self._F = np.zeros(self.N)
        self._sol = np.zeros(self.N)
        self.last_solve = None
        self.solve_hook = None          # called with the iemic_solve_info of every solve
        self._vpool = []                # free device vectors (DeviceVec buffers)

    @staticmethod
    def unique_id() -> bytes:
        """RCCL unique id for a multi-GPU Ocean (call on rank 0, broadcast the bytes)."""
        buf = (C.c_ubyte * 128)()
        check(lib().iemic_comm_unique_id(buf), "iemic_comm_unique_id")
        return bytes(buf)

    def layout(self) -> dict:
        out = np.zeros(12, dtype=np.int64)
        check(lib().iemic_layout(self._h, ptr(out, C.c_int64)), "iemic_layout")
        return dict(ext_rows=int(out[0]), own_first=int(out[1]), own_rows=int(out[2]),
                    jb0=int(out[3]), jb1=int(out[4]), rank=int(out[5]), nranks=int(out[6]),
                    ib0=int(out[7]), ib1=int(out[8]), npx=int(out[9]), npy=int(out[10]),
                    hx=int(out[11]))

    # ---- device vectors (DeviceOps) ---------------------------------------------------
    def vec_ops(self) -> DeviceOps:
        """The device vector algebra a continuation driver uses on this model."""
        return DeviceOps(self)

    def _vec_take(self) -> C.c_void_p:
        if self._closing:
            raise IemicError("Ocean is closed")
        self._vlive += 1
        if self._vpool:
            return self._vpool.pop()
        p = C.c_void_p()
        rc = lib().iemic_vec_alloc(self._h, C.byref(p))
        if rc:
            self._vlive -= 1
        check(rc, "iemic_vec_alloc")
        return p

    def _vec_give(self, p) -> None:
        """a DeviceVec's buffer back: into the pool, or freed when the Ocean was closed (the
        context then lives until the last vector is gone)"""
        if not getattr(self, "_h", None):
            return
        self._vlive -= 1
        if self._closing:
            lib().iemic_vec_free(self._h, p)
            if self._vlive <= 0:
                self._destroy()
        else:
            self._vpool.append(p)

    # ---- lifecycle -----------------------------------------------------------------
    def close(self):
        """Frees the pooled vectors and the context; a context with DeviceVecs still alive
        (a continuation's saved state, say) is destroyed when the last of them is released."""
        if getattr(self, "_h", None) and not self._closing:
            for p in self._vpool:
                lib().iemic_vec_free(self._h, p)
            self._vpool = []
            self._closing = True
            if self._vlive <= 0:
                self._destroy()

    def _destroy(self):
        if getattr(self, "_h", None):
            lib().iemic_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- parameters (THCM::setParameter / getParameter) ------------------------------
    def setPar(self, par, value: float) -> None:
        idx = PAR_INDEX[par] if isinstance(par, str) else int(par)
        check(lib().iemic_set_par(self._h, idx, float(value)), "iemic_set_par")

    def getPar(self, par) -> float:
        idx = PAR_INDEX[par] if isinstance(par, str) else int(par)
        v = C.c_double()
        check(lib().iemic_get_par(self._h, idx, C.byref(v)), "iemic_get_par")
        return v.value

    # ---- coupled atmosphere (Ocean::synchronize(atmos), Ocean.C:1443-1472) -------------
    def setAtmosphere(self, t, q, a, p, commpars) -> None:
        """THCM::setAtmosphereT/Q/A/P + set_atmos_parameters (n*m surface fields, the 18
        AtmosLocal::CommPars); the context must be created with coupled_t = 1."""
        arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (t, q, a, p, commpars)]
        check(lib().iemic_set_atmosphere(self._h, *[ptr(v) for v in arrs]), "iemic_set_atmosphere")

    def getDeps(self) -> np.ndarray:
        """getdeps (usrc.F90:201-219): Ooa, Os, nus, eta, lvsc, qdim, pQSnd."""
        out = np.zeros(7)
        check(lib().iemic_get_deps(self._h, ptr(out)), "iemic_get_deps")
        return out

    def getSunO(self) -> np.ndarray:
        out = np.zeros(self.cfg.n * self.cfg.m)
        check(lib().iemic_get_suno(self._h, ptr(out)), "iemic_get_suno")
        return out

    def setIntCondCorrection(self, x: Optional[np.ndarray] = None) -> float:
        """THCM::setIntCondCorrection (THCM.C:2020-2038): the integral-condition entry of F
        becomes intSign (coeff . x - coeff . x0) with x0 = x (default: the current state),
        as Ocean does for a loaded SRES = 0 state (Ocean.C:144-148).  Returns it."""
        xp = None
        if x is not None:
            x = np.ascontiguousarray(x, dtype=np.float64)
            xp = ptr(x)
        check(lib().iemic_set_intcond_correction(self._h, xp), "iemic_set_intcond_correction")
        v = C.c_double()
        check(lib().iemic_get_intcond_correction(self._h, C.byref(v)), "iemic_get_intcond_correction")
        return v.value

    # ---- state files (Model::saveStateToFile / loadStateFromFile, Model.H:149-330) -----
    def saveStateToFile(self, filename: str) -> None:
        """HDF5 file in the reference's layout (EpetraExt::HDF5 conventions): State
        (an Epetra_MultiVector: Values, GlobalLength, NumVectors, __type__), Parameters (one
        scalar per continuation parameter, THCM::int2par names), Grid (n, m, l, nun, aux,
        bounds in radians, hdim, the uniform horizontal coordinates) and Ocean's MaskGlobal
        (Ocean.C:1904-2113).  Written by iemic.h5 (no libhdf5 in this build)."""
        import math
        from . import h5
        c = self.cfg
        x = self.getState()
        pars = {}
        for name in PAR_INDEX:
            pars[name] = np.array(self.getPar(name), dtype=np.float64)
        xmin, xmax = math.radians(c.xmin), math.radians(c.xmax)
        ymin, ymax = math.radians(c.ymin), math.radians(c.ymax)
        dx, dy = (xmax - xmin) / c.n, (ymax - ymin) / c.m
        L = self.landmask().astype(np.int32)
        tree = {
            "State": {"Values": x.reshape(1, -1), "GlobalLength": np.array(len(x), dtype=np.int32),
                      "NumVectors": np.array(1, dtype=np.int32),
                      "__type__": np.array([b"Epetra_MultiVector"], dtype="S19")},
            "Parameters": pars,
            "Grid": {"n": np.array(c.n, dtype=np.int32), "m": np.array(c.m, dtype=np.int32),
                     "l": np.array(c.l, dtype=np.int32), "nun": np.array(6, dtype=np.int32),
                     "aux": np.array(0, dtype=np.int32), "xmin": np.array(xmin), "xmax": np.array(xmax),
                     "ymin": np.array(ymin), "ymax": np.array(ymax), "hdim": np.array(float(c.hdim)),
                     "x": xmin + dx * (np.arange(c.n) + 0.5), "y": ymin + dy * (np.arange(c.m) + 0.5),
                     "xu": xmin + dx * np.arange(1, c.n + 1), "yv": ymin + dy * np.arange(1, c.m + 1)},
            "MaskGlobal": {"Global": L, "GlobalSize": np.array(L.size, dtype=np.int32),
                           "Label": np.array([b"current"], dtype="S8")},
        }
        h5.write(filename, tree)

    def loadStateFromFile(self, filename: str) -> int:
        """Model::loadStateFromFile: the state (global length must match), every parameter
        the file holds under a THCM name (unknown names are skipped, as the reference's
        try/catch does; the older label FPER is read as Flux Perturbation), and for an
        SRES = 0 grid the integral-condition correction of the loaded state (Ocean.C:144-148).
        Returns 1 (state untouched) if the file does not exist, 0 otherwise."""
        import os
        from . import h5
        if not os.path.exists(filename):
            return 1
        t = h5.read(filename)
        if "/State/Values" not in t:
            raise IemicError(f"The group <State> is not contained in hdf5 {filename}")
        x = np.asarray(t["/State/Values"][0], dtype=np.float64).reshape(-1)
        if x.size != self.N:
            raise IemicError(f"{filename}: state of length {x.size}, this model has {self.N}")
        self.setState(x)
        alias = {"FPER": "Flux Perturbation"}
        for path, (v, _) in t.items():
            if not path.startswith("/Parameters/"):
                continue
            name = alias.get(path.split("/", 2)[2], path.split("/", 2)[2])
            if name in PAR_INDEX:
                self.setPar(name, float(np.asarray(v).reshape(-1)[0]))
        if self.rowintcon >= 0:
            self.setIntCondCorrection()
        return 0

    # ---- state --------------------------------------------------------------------
    def setState(self, x: np.ndarray) -> None:
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert x.shape == (self.N,)
        check(lib().iemic_set_state(self._h, ptr(x)), "iemic_set_state")
        self._x = x.copy()

    def getState(self, mode: str = "C") -> np.ndarray:
        x = np.zeros(self.N)
        check(lib().iemic_get_state(self._h, ptr(x)), "iemic_get_state")
        return x

    def getRHS(self, mode: str = "C") -> np.ndarray:
        return self._F.copy() if mode == "C" else self._F

    def getSolution(self, mode: str = "C") -> np.ndarray:
        return self._sol.copy() if mode == "C" else self._sol

    # ---- Model API -----------------------------------------------------------------
    def computeRHS(self) -> np.ndarray:
        """F(state) (Ocean::computeRHS, Ocean.C:1267-1274)."""
        check(lib().iemic_rhs(self._h, ptr(self._F)), "iemic_rhs")
        return self._F

    def computeJacobian(self) -> None:
        """J(state) + diag(B) (Ocean::computeJacobian, Ocean.C:1287-1299)."""
        check(lib().iemic_jacobian(self._h), "iemic_jacobian")

    def applyMatrix(self, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.N) if y is None else y
        check(lib().iemic_spmv(self._h, ptr(x), ptr(y)), "iemic_spmv")
        return y

    def diagB(self) -> np.ndarray:
        B = np.zeros(self.N)
        check(lib().iemic_diag_b(self._h, ptr(B)), "iemic_diag_b")
        return B

    def _krylov(self) -> _lib.Krylov:
        sp = self.solver_params
        return _lib.Krylov(float(sp["FGMRES tolerance"]), int(sp["FGMRES iterations"]),
                           int(sp["FGMRES restarts"]), int(sp["Preconditioner"]),
                           int(sp["TS sweeps"]), 1 if sp["Orthogonalization"] == "DGKS" else 0,
                           int(sp["Dyn iterations"]), 1 if str(sp["Solver"]).upper() == "IDR" else 0,
                           int(sp["TS multigrid cycles"]), int(sp["Multigrid sweeps"]),
                           float(sp["Dyn damping"]), int(bool(sp["Dyn minimal residual"])),
                           int(sp["IDR s"]), float(sp["IDR angle"]),
                           int(bool(sp["IDR replace residuals"])), int(sp["TS after dyn pass"]),
                           int(sp["Schur passes"]))

    def buildPreconditioner(self, force: bool = False) -> None:
        """Ocean::buildPreconditioner (Ocean.C:1360-1374): recompute only when flagged."""
        if self._recomp_prec or force:
            k = self._krylov()
            check(lib().iemic_prec_compute(self._h, C.byref(k)), "iemic_prec_compute")
            self._recomp_prec = False

    def applyPrecon(self, r: np.ndarray) -> np.ndarray:
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros(self.N)
        check(lib().iemic_prec_apply(self._h, ptr(r), ptr(z)), "iemic_prec_apply")
        return z

    def solve(self, rhs: np.ndarray) -> np.ndarray:
        """J x = rhs with FGMRES (Ocean::solve, Ocean.C:1060-1137)."""
        self.buildPreconditioner()
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        k = self._krylov()
        info = _lib.SolveInfo()
        check(lib().iemic_solve(self._h, ptr(rhs), ptr(self._sol), C.byref(k), C.byref(info)),
              "iemic_solve")
        self.last_solve = info
        if self.solve_hook is not None:
            self.solve_hook(info)
        return self._sol

    def preProcess(self) -> None:
        """Ocean::preProcess (Ocean.C:790-801): refactor the preconditioner next solve."""
        self._recomp_prec = True

    def postProcess(self) -> None:
        pass

    # ---- diagnostics (Ocean.C; host side as in the reference) ---------------------------
    def getIntCondCoeff(self) -> np.ndarray:
        """THCM::getIntCondCoeff (THCM.C:2549-2577), reference row order."""
        out = np.zeros(self.N)
        check(lib().iemic_get_intcond_coeff(self._h, ptr(out)), "iemic_get_intcond_coeff")
        return out

    def getPsiM(self, field: bool = False):
        """Ocean::getPsiM (Ocean.C:872-886): (psiMin, psiMax) of the meridional overturning
        streamfunction of the current state in Sv; with field=True also PsiM(0:m, 0:l) as
        an (l+1, m+1) array."""
        mn, mx = C.c_double(), C.c_double()
        ps = np.zeros((self.cfg.m + 1) * (self.cfg.l + 1))
        check(lib().iemic_psim(self._h, C.byref(mn), C.byref(mx), ptr(ps)), "iemic_psim")
        if field:
            return mn.value, mx.value, ps.reshape(self.cfg.l + 1, self.cfg.m + 1)
        return mn.value, mx.value

    def integralChecks(self):
        """Ocean::integralChecks (Ocean.C:1841-1848): (salt_advection, salt_diffusion)."""
        a, d = C.c_double(), C.c_double()
        check(lib().iemic_integral_checks(self._h, C.byref(a), C.byref(d)), "iemic_integral_checks")
        return a.value, d.value

    def getMassMat(self) -> np.ndarray:
        """Ocean::getMassMat: the diagonal mass matrix B (fillcolB; state independent, so
        a Jacobian is assembled first when none is current)."""
        try:
            return self.diagB()
        except _lib.IemicError:
            self.computeJacobian()
            return self.diagB()

    def applyMassMat(self, v: np.ndarray) -> np.ndarray:
        """Ocean::applyMassMat: B v (B diagonal)."""
        return self.getMassMat() * np.asarray(v, dtype=np.float64)

    def getColumnIntegral(self, use_sres: bool = True) -> np.ndarray:
        """Ocean::getColumnIntegral (Ocean.C:1851-1895): for every S column of the last
        Jacobian the integral-condition-weighted column sum sum_r coeff_r J[r, c] (the
        intcond row's own coefficient dropped when SRES = 0 and use_sres), 0 elsewhere.
        Host side, from the exported CSR, as the reference's Epetra computation; on several
        ranks each sums its owned rows and the sums are added over the ranks (collective)."""
        rowptr, col, val = self.exportCSR()
        coef = self.getIntCondCoeff()
        ri = self.rowintcon
        if use_sres and ri >= 0:
            coef[ri] = 0.0
        rows = self.owned_rows()
        nown = len(rows)
        grow = np.repeat(rows, np.diff(rowptr[:nown + 1]))
        sums = np.zeros(self.N)
        np.add.at(sums, col[:len(grow)], coef[grow] * val[:len(grow)])
        if self.layout()["nranks"] > 1:
            check(lib().iemic_allreduce_sum(self._h, ptr(sums), self.N), "iemic_allreduce_sum")
        sel = np.zeros(self.N)
        sel[5::6] = 1.0
        return sums * sel

    def owned_rows(self) -> np.ndarray:
        """Global (reference-order) rows of this rank, in the order exportCSR lists them:
        levels, then latitudes, then longitudes of the subdomain, six unknowns per cell."""
        lay, c = self.layout(), self.cfg
        k = np.arange(c.l)[:, None, None, None]
        j = np.arange(lay["jb0"], lay["jb1"])[None, :, None, None]
        i = np.arange(lay["ib0"], lay["ib1"])[None, None, :, None]
        v = np.arange(6)[None, None, None, :]
        return (6 * ((k * c.m + j) * c.n + i) + v).reshape(-1)

    def comm_size(self):
        """(ranks the communicator reports -- ncclCommCount under RCCL --, transport name)."""
        n, kind = C.c_int(), C.c_int()
        check(lib().iemic_comm_size(self._h, C.byref(n), C.byref(kind)), "iemic_comm_size")
        return n.value, {0: "none", 1: "rccl", 2: "local", 3: "host"}[kind.value]

    def active_cells(self) -> int:
        """Cells with a non-identity row (iemic_active_cells; 0 before a preconditioner set-up)."""
        v = C.c_int64()
        check(lib().iemic_active_cells(self._h, C.byref(v)), "iemic_active_cells")
        return v.value

    def comm_stats(self) -> dict:
        """Communication counters since the previous call (then reset)."""
        out = np.zeros(4, dtype=np.int64)
        check(lib().iemic_comm_stats(self._h, ptr(out, C.c_int64)), "iemic_comm_stats")
        return dict(batches=int(out[0]), messages=int(out[1]), bytes=int(out[2]), allreduces=int(out[3]))

    # ---- fused device-resident Newton step -------------------------------------------
    def newtonStep(self, allow_unconverged: bool = False) -> _lib.NewtonInfo:
        """F, J, preconditioner, J dx = -F, x += dx, F (transient/Newton.H:92-99).  The
        update is applied either way (as Newton.H does); a solve that missed its tolerance
        raises IemicError unless allow_unconverged."""
        k = self._krylov()
        info = _lib.NewtonInfo()
        rc = lib().iemic_newton_step(self._h, C.byref(k), C.byref(info))
        if rc == _lib.IEMIC_ENOCONV and allow_unconverged:
            rc = 0
        if rc == _lib.IEMIC_ENOCONV:
            method = f"IDR({k.idr_s})" if k.method == 1 else "FGMRES"
            raise _lib.IemicError(
                f"iemic_newton_step: {method} did not converge ({info.solve.iters} steps, "
                f"relative residual {info.solve.explicit_rel_res:.3e})")
        check(rc, "iemic_newton_step")
        return info

    # ---- inspection -----------------------------------------------------------------
    def exportCSR(self):
        nnz = lib().iemic_graph_nnz(self._h)
        rowptr = np.zeros(self.N + 1, dtype=np.int64)
        col = np.zeros(nnz, dtype=np.int32)
        val = np.zeros(nnz)
        check(lib().iemic_export_csr(self._h, ptr(rowptr, C.c_int64), ptr(col, C.c_int), ptr(val)),
              "iemic_export_csr")
        return rowptr, col, val

    def landmask(self) -> np.ndarray:
        c = self.cfg
        out = np.zeros((c.l + 2) * (c.m + 2) * (c.n + 2), dtype=np.int32)
        check(lib().iemic_landm(self._h, ptr(out, C.c_int)), "iemic_landm")
        return out

    @property
    def rowintcon(self) -> int:
        return lib().iemic_rowintcon(self._h)

    def time_spmv(self, nrep: int = 20) -> float:
        ms = C.c_double()
        check(lib().iemic_time_spmv(self._h, int(nrep), C.byref(ms)), "iemic_time_spmv")
        return ms.value

    def time_prec(self, nrep: int = 20):
        """(GPU ms, host enqueue ms) per preconditioner apply, nrep applies back to back."""
        ms, hms = C.c_double(), C.c_double()
        self.buildPreconditioner()
        check(lib().iemic_time_prec(self._h, int(nrep), C.byref(ms), C.byref(hms)), "iemic_time_prec")
        return ms.value, hms.value

    def time_prec_parts(self, nrep: int = 50) -> dict:
        """GPU microseconds of the block GS apply's parts (iemic_time_prec_parts)."""
        self.buildPreconditioner()
        us = np.zeros(4)
        check(lib().iemic_time_prec_parts(self._h, int(nrep), ptr(us)), "iemic_time_prec_parts")
        return dict(schur_solve_us=us[0], ts_solve_us=us[1], dyn_pass_us=us[2], dyn_defect_us=us[3])

    def time_spmv_cold(self, flush_ptr: int, flush_bytes: int, nrep: int = 10) -> float:
        """Mean SpMV kernel ms with the Infinity Cache flushed (device memset of a caller
        buffer) before each launch -- the in-solve, cold-cache rate."""
        ms = C.c_double()
        check(lib().iemic_time_spmv_cold(self._h, int(nrep), C.c_void_p(flush_ptr),
                                         int(flush_bytes), C.byref(ms)), "iemic_time_spmv_cold")
        return ms.value
