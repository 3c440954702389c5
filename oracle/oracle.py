"""TEST INFRASTRUCTURE ONLY -- ctypes front-ends of the two CPU checkers.

* ``Oracle``: the C restatement (oracle/thcm_oracle.c -> oracle/_build/liboracle.so).
* ``run_reference``: the reference's own THCM Fortran (compiled in place by
  oracle/ref/Makefile into oracle/_ref/libthcm_ref.so), driven in a fresh subprocess
  per configuration because THCM keeps global Fortran module state (a singleton,
  src/ocean/THCM.H:76-84).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product (i-emic_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_ORACLE = os.path.join(HERE, "_build", "liboracle.so")
LIB_REF = os.path.join(HERE, "_ref", "libthcm_ref.so")


def build(ref: bool = True) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference/src/ocean"):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "ref")], check=True)


class _Cfg(C.Structure):
    _fields_ = [("n", C.c_int), ("m", C.c_int), ("l", C.c_int),
                ("xmin_deg", C.c_double), ("xmax_deg", C.c_double),
                ("ymin_deg", C.c_double), ("ymax_deg", C.c_double),
                ("periodic", C.c_int), ("hdim", C.c_double), ("qz", C.c_double),
                ("tres", C.c_int), ("sres", C.c_int), ("ite", C.c_int), ("its", C.c_int),
                ("iza", C.c_int), ("forcing_type", C.c_int), ("ih", C.c_int),
                ("vmix", C.c_int), ("coriolis_on", C.c_int), ("alphaT", C.c_double),
                ("alphaS", C.c_double), ("int_sign", C.c_int), ("nic", C.c_int),
                ("mic", C.c_int), ("rho_mixing", C.c_int), ("coupled_t", C.c_int),
                ("coupled_s", C.c_int)]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_ORACLE):
            build(ref=False)
        lib = C.CDLL(LIB_ORACLE)
        lib.orc_create.restype = C.c_void_p
        lib.orc_create.argtypes = [C.POINTER(_Cfg), C.POINTER(C.c_int), C.POINTER(C.c_double)]
        lib.orc_set_atmos.argtypes = [C.c_void_p] + [C.POINTER(C.c_double)] * 5
        lib.orc_get_deps.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        lib.orc_destroy.argtypes = [C.c_void_p]
        lib.orc_set_par.argtypes = [C.c_void_p, C.c_int, C.c_double]
        lib.orc_get_par.argtypes = [C.c_void_p, C.c_int]
        lib.orc_get_par.restype = C.c_double
        lib.orc_nrows.argtypes = [C.c_void_p]
        lib.orc_rowintcon.argtypes = [C.c_void_p]
        lib.orc_graph_nnz.argtypes = [C.c_void_p]
        lib.orc_graph_nnz.restype = C.c_int64
        lib.orc_graph.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int)]
        lib.orc_fortran_matrix.restype = C.c_int64
        lib.orc_fortran_matrix.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int),
                                           C.POINTER(C.c_int), C.POINTER(C.c_double),
                                           C.POINTER(C.c_double)]
        lib.orc_fortran_rhs.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        lib.orc_jacobian.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_double)]
        lib.orc_rhs.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        lib.orc_intcond_coeff.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        lib.orc_csr_spmv.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int),
                                     C.POINTER(C.c_double), C.POINTER(C.c_double),
                                     C.POINTER(C.c_double)]
        _lib = lib
    return _lib


def cfg_struct(d: dict) -> _Cfg:
    return _Cfg(d["n"], d["m"], d["l"], d["xmin_deg"], d["xmax_deg"], d["ymin_deg"],
                d["ymax_deg"], d["periodic"], d["hdim"], d["qz"], d["tres"], d["sres"],
                d["ite"], d["its"], d["iza"], d["forcing_type"], d["ih"], d["vmix"],
                d["coriolis_on"], d["alphaT"], d["alphaS"], d["int_sign"], d["nic"], d["mic"],
                d["rho_mixing"], int(d.get("coupled_T", 0)), int(d.get("coupled_S", 0)))


class Oracle:
    """C restatement of the THCM hot path (see oracle/thcm_oracle.c)."""

    def __init__(self, cfgdict: dict, landm: np.ndarray, pars=(), spert=None):
        lib = _load()
        self.lib = lib
        self.d = dict(cfgdict)
        self._cfg = cfg_struct(cfgdict)
        lm = np.ascontiguousarray(landm, dtype=np.int32)
        n, m = cfgdict["n"], cfgdict["m"]
        sp = np.full(n * m, float(cfgdict["sres"])) if spert is None else np.ascontiguousarray(spert, dtype=np.float64)
        self.h = lib.orc_create(C.byref(self._cfg), _p(lm, C.c_int), _p(sp, C.c_double))
        if not self.h:
            raise RuntimeError("orc_create failed")
        for idx, v in pars:
            lib.orc_set_par(self.h, int(idx), float(v))
        self.N = lib.orc_nrows(self.h)
        self.rowintcon = lib.orc_rowintcon(self.h)
        nnz = lib.orc_graph_nnz(self.h)
        self.rowptr = np.zeros(self.N + 1, dtype=np.int64)
        self.col = np.zeros(nnz, dtype=np.int32)
        lib.orc_graph(self.h, _p(self.rowptr, C.c_int64), _p(self.col, C.c_int))

    def __del__(self):
        try:
            self.lib.orc_destroy(self.h)
        except Exception:
            pass

    def set_atmos(self, t, q, a, pars, p=None):
        """Ocean::synchronize(atmos) on the restatement (coupled_T / coupled_S configs)"""
        arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (t, q, a)]
        pa = np.ascontiguousarray(pars, dtype=np.float64)
        pp = None if p is None else np.ascontiguousarray(p, dtype=np.float64)
        self._atm = (arrs, pa, pp)
        self.lib.orc_set_atmos(self.h, *[_p(v, C.c_double) for v in arrs],
                               None if pp is None else _p(pp, C.c_double), _p(pa, C.c_double))

    def get_deps(self) -> np.ndarray:
        out = np.zeros(7)
        self.lib.orc_get_deps(self.h, _p(out, C.c_double))
        return out

    def set_par(self, idx, v):
        self.lib.orc_set_par(self.h, int(idx), float(v))

    def get_par(self, idx):
        return self.lib.orc_get_par(self.h, int(idx))

    def jacobian(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        val = np.zeros(len(self.col))
        B = np.zeros(self.N)
        self.lib.orc_jacobian(self.h, _p(x, C.c_double), _p(val, C.c_double), _p(B, C.c_double))
        return val, B

    def rhs(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        F = np.zeros(self.N)
        self.lib.orc_rhs(self.h, _p(x, C.c_double), _p(F, C.c_double))
        return F

    def fortran_rhs(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        B = np.zeros(self.N)
        self.lib.orc_fortran_rhs(self.h, _p(x, C.c_double), _p(B, C.c_double))
        return B

    def fortran_matrix(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        nnz = self.lib.orc_fortran_matrix(self.h, _p(x, C.c_double), None, None, None, None)
        beg = np.zeros(self.N + 1, dtype=np.int32)
        jco = np.zeros(nnz, dtype=np.int32)
        co = np.zeros(nnz)
        coB = np.zeros(self.N)
        self.lib.orc_fortran_matrix(self.h, _p(x, C.c_double), _p(beg, C.c_int),
                                    _p(jco, C.c_int), _p(co, C.c_double), _p(coB, C.c_double))
        return beg, jco, co, coB

    def intcond_coeff(self):
        c = np.zeros(self.N)
        self.lib.orc_intcond_coeff(self.h, _p(c, C.c_double))
        return c

    def spmv(self, val, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.N)
        self.lib.orc_csr_spmv(self.N, _p(self.rowptr, C.c_int64), _p(self.col, C.c_int),
                              _p(val, C.c_double), _p(x, C.c_double), _p(y, C.c_double))
        return y


# ------------------------------------------------------------------------------------
# reference (Fortran) runner: one subprocess per configuration

_REF_SCRIPT = r'''
import ctypes as C, sys, numpy as np
lib = C.CDLL(sys.argv[1])
d = np.load(sys.argv[2], allow_pickle=False)
class Cfg(C.Structure):
    _fields_ = [(k, t) for k, t in [("n",C.c_int),("m",C.c_int),("l",C.c_int),
        ("xmin_deg",C.c_double),("xmax_deg",C.c_double),("ymin_deg",C.c_double),("ymax_deg",C.c_double),
        ("periodic",C.c_int),("hdim",C.c_double),("qz",C.c_double),("itopo",C.c_int),("flat",C.c_int),
        ("rd_mask",C.c_int),("tres",C.c_int),("sres",C.c_int),("iza",C.c_int),("ite",C.c_int),
        ("its",C.c_int),("rd_spertm",C.c_int),("coupled_T",C.c_int),("coupled_S",C.c_int),
        ("forcing_type",C.c_int),("ih",C.c_int),("vmix",C.c_int),("tap",C.c_int),
        ("rho_mixing",C.c_int),("coriolis_on",C.c_int),("alphaT",C.c_double),("alphaS",C.c_double),
        ("maskfile",C.c_char*256),("spertfile",C.c_char*256)]]
cfg = Cfg()
ints = d["cfg_int"]; dbls = d["cfg_dbl"]
names_i = ["n","m","l","periodic","itopo","flat","rd_mask","tres","sres","iza","ite","its",
           "rd_spertm","coupled_T","coupled_S","forcing_type","ih","vmix","tap","rho_mixing","coriolis_on"]
names_d = ["xmin_deg","xmax_deg","ymin_deg","ymax_deg","hdim","qz","alphaT","alphaS"]
for k, v in zip(names_i, ints): setattr(cfg, k, int(v))
for k, v in zip(names_d, dbls): setattr(cfg, k, float(v))
cfg.maskfile = bytes(d["maskfile"]).rstrip(b"\0")
cfg.spertfile = b"no_mask_specified"
landm = np.ascontiguousarray(d["landm"], dtype=np.int32)
use_landm = bool(d["use_landm"])
lib.thcmref_init.argtypes = [C.POINTER(Cfg), C.c_void_p]
rc = lib.thcmref_init(C.byref(cfg), landm.ctypes.data if use_landm else None)
assert rc == 0, rc
lib.thcmref_set_par.argtypes = [C.c_int, C.c_double]
for idx, v in d["pars"]:
    lib.thcmref_set_par(int(idx), float(v))
if "atm_t" in d.files:
    atm = [np.ascontiguousarray(d["atm_" + k], dtype=np.float64) for k in "tqap"]
    apars = np.ascontiguousarray(d["atm_pars"], dtype=np.float64)
    lib.thcmref_set_atmos.argtypes = [C.c_void_p] * 5
    lib.thcmref_set_atmos(*[a.ctypes.data for a in atm], apars.ctypes.data)
deps = np.zeros(7)
lib.thcmref_getdeps.argtypes = [C.c_void_p]
lib.thcmref_getdeps(deps.ctypes.data)
nrows = C.c_int(); cap = C.c_int()
lib.thcmref_sizes(C.byref(nrows), C.byref(cap))
N = nrows.value
out = {}
L = np.zeros(landm.size, dtype=np.int32)
lib.thcmref_landm(L.ctypes.data_as(C.c_void_p))
out["landm_local"] = L
iv = np.zeros(N, dtype=np.float64); ii = np.zeros(N, dtype=np.int32)
lib.thcmref_intcond.argtypes = [C.c_void_p, C.c_void_p]
ln = lib.thcmref_intcond(iv.ctypes.data, ii.ctypes.data)
out["intcond_val"] = iv[:ln]; out["intcond_ind"] = ii[:ln]
lib.thcmref_matrix.argtypes = [C.c_void_p] * 5
lib.thcmref_rhs.argtypes = [C.c_void_p] * 2
pidx = np.arange(31)
out["par"] = np.array([0.0] + [0.0]*30)
lib.thcmref_get_par.restype = C.c_double
lib.thcmref_get_par.argtypes = [C.c_int]
for p in range(1, 31):
    out["par"][p] = lib.thcmref_get_par(p)
out["deps"] = deps
for s in range(int(d["nstates"])):
    x = np.ascontiguousarray(d["x%d" % s])
    beg = np.zeros(N + 1, dtype=np.int32); jco = np.zeros(cap.value, dtype=np.int32)
    co = np.zeros(cap.value); coB = np.zeros(N)
    nnz = lib.thcmref_matrix(x.ctypes.data, beg.ctypes.data, jco.ctypes.data, co.ctypes.data, coB.ctypes.data)
    B = np.zeros(N)
    lib.thcmref_rhs(x.ctypes.data, B.ctypes.data)
    out["beg%d" % s] = beg; out["jco%d" % s] = jco[:nnz]; out["co%d" % s] = co[:nnz]
    out["coB%d" % s] = coB; out["B%d" % s] = B
np.savez(sys.argv[3], **out)
'''


def reference_available() -> bool:
    return os.path.exists(LIB_REF)


def run_reference(cfgdict: dict, landm, pars, states, use_landm: bool = True,
                  timeout: float = 600.0, atmos: dict | None = None) -> dict:
    """Run the reference THCM Fortran (init, setparcs, matrix, rhs) in a fresh process.

    Returns dict with per-state Fortran CSR (beg/jco/co, 1-based), coB, rhs B, the local
    land mask after init, intcond scaling and par(1..30)."""
    if not reference_available():
        raise RuntimeError("reference library not built (make -C oracle ref)")
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.npz")
        outp = os.path.join(td, "out.npz")
        ints = [cfgdict[k] for k in ["n", "m", "l", "periodic", "itopo", "flat", "rd_mask", "tres",
                                     "sres", "iza", "ite", "its", "rd_spertm", "coupled_T",
                                     "coupled_S", "forcing_type", "ih", "vmix", "tap",
                                     "rho_mixing", "coriolis_on"]]
        dbls = [cfgdict[k] for k in ["xmin_deg", "xmax_deg", "ymin_deg", "ymax_deg", "hdim",
                                     "qz", "alphaT", "alphaS"]]
        mf = np.frombuffer(cfgdict["maskfile"].encode().ljust(256, b"\0"), dtype=np.uint8)
        arrs = dict(cfg_int=np.array(ints, dtype=np.int64), cfg_dbl=np.array(dbls),
                    maskfile=mf, landm=np.ascontiguousarray(landm, dtype=np.int32).reshape(-1),
                    use_landm=np.array(int(use_landm)),
                    pars=np.array(list(pars), dtype=np.float64).reshape(-1, 2),
                    nstates=np.array(len(states)))
        for s, x in enumerate(states):
            arrs["x%d" % s] = np.ascontiguousarray(x, dtype=np.float64)
        if atmos is not None:
            # coupled ocean (coupled_T = 1): atmosphere fields t, q, a, p (n*m each) and the
            # 18 AtmosLocal::CommPars, inserted through Ocean::synchronize's Fortran calls
            for k in "tqap":
                arrs["atm_" + k] = np.ascontiguousarray(atmos[k], dtype=np.float64)
            arrs["atm_pars"] = np.ascontiguousarray(atmos["pars"], dtype=np.float64)
        np.savez(inp, **arrs)
        script = os.path.join(td, "run.py")
        with open(script, "w") as f:
            f.write(_REF_SCRIPT)
        subprocess.run([sys.executable, script, LIB_REF, inp, outp], check=True, cwd=td,
                       timeout=timeout, stdout=subprocess.DEVNULL)
        with np.load(outp, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}


def fortran_to_graph(rowptr, col, beg, jco, co, rowintcon=-1):
    """Restates THCM.C:1074-1155: place the 1-based Fortran CSR rows into the maximal
    graph (rows sorted by column); unfilled slots stay explicit zeros."""
    N = len(rowptr) - 1
    val = np.zeros(len(col))
    for r in range(N):
        if r == rowintcon:
            continue
        b, e = int(rowptr[r]), int(rowptr[r + 1])
        cols = col[b:e]
        fb, fe = int(beg[r]) - 1, int(beg[r + 1]) - 1
        fc = jco[fb:fe] - 1
        pos = np.searchsorted(cols, fc)
        if np.any(pos >= len(cols)) or np.any(cols[np.minimum(pos, len(cols) - 1)] != fc):
            raise AssertionError(f"row {r}: Fortran entry outside maximal graph")
        val[b + pos] = co[fb:fe]
    return val


def graph_to_fortran(n, m, l, periodic, rowptr, col, val, rowintcon=-1, chunk=16384):
    """The inverse of fortran_to_graph: the Fortran CSR (beg, jco, co; 1-based, int32 /
    float64) that assemble.F90's fillcolA (assemble.F90:57-139) writes for the same
    coefficients -- per row the 27 stencil positions kk outer (kk 1..9 at level k, 10..18
    at k-1, 19..27 at k+1; within a level (i-1+(kk-1)//3, j-1+(kk+2)%3), shift's periodic
    wrap in i, assemble.F90:142-179), the 6 unknowns inner, entries with |v| > 1e-10 only.
    The integral-condition row (SRES = 0) is not a Fortran row (assemble.F90:198-199)."""
    N = len(rowptr) - 1
    di = np.empty(27, np.int64)
    dj = np.empty(27, np.int64)
    dk = np.empty(27, np.int64)
    for kk in range(1, 28):
        q = (kk - 1) % 9 + 1
        di[kk - 1] = (q - 1) // 3 - 1
        dj[kk - 1] = (q + 2) % 3 - 1
        dk[kk - 1] = 0 if kk <= 9 else (-1 if kk <= 18 else 1)
    rows_of = np.repeat(np.arange(N, dtype=np.int64), np.diff(rowptr))
    gkey = rows_of * N + np.asarray(col, dtype=np.int64)          # sorted (rows, then cols)
    val = np.asarray(val)
    begs, jcos, cos = [np.zeros(1, np.int64)], [], []
    for r0 in range(0, N, chunk):
        r = np.arange(r0, min(N, r0 + chunk), dtype=np.int64)
        cell = r // 6
        i, j, k = cell % n, (cell // n) % m, cell // (n * m)
        ii = i[:, None, None] + di[None, :, None]
        jj = j[:, None, None] + dj[None, :, None]
        kc = k[:, None, None] + dk[None, :, None]
        if periodic:
            ii = np.where(ii < 0, ii + n, np.where(ii >= n, ii - n, ii))
        inside = np.broadcast_to((ii >= 0) & (ii < n) & (jj >= 0) & (jj < m) & (kc >= 0) & (kc < l),
                                 (len(r), 27, 6))
        cc = 6 * ((kc * m + jj) * n + ii) + np.arange(6)[None, None, :]
        cc = np.where(inside, cc, 0).reshape(len(r), 162)
        key = r[:, None] * N + cc
        pos = np.minimum(np.searchsorted(gkey, key), len(gkey) - 1)
        hit = (gkey[pos] == key) & inside.reshape(len(r), 162)
        v = np.where(hit, val[pos], 0.0)
        keep = np.abs(v) > 1e-10
        if rowintcon >= 0:
            keep[r == rowintcon] = False
        cnt = keep.sum(axis=1)
        begs.append(np.cumsum(cnt))
        jcos.append(cc[keep])
        cos.append(v[keep])
    bl = [begs[0]]
    off = 0
    for b in begs[1:]:
        bl.append(b + off)
        off += b[-1] if len(b) else 0
    beg = np.concatenate(bl).astype(np.int32) + 1
    return beg, (np.concatenate(jcos) + 1).astype(np.int32), np.concatenate(cos).astype(np.float64)


# ------------------------------------------------------------------------------------
# CPU linear solve (krylov_oracle.c)

def _load_krylov():
    lib = _load()
    if not hasattr(lib, "_krylov_ready"):
        P64, PI, PD = C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_double)
        lib.orc_bcsr_build.restype = C.c_int64
        lib.orc_bcsr_build.argtypes = [C.c_int, P64, PI, PD, P64, PI, PD, C.c_int64]
        lib.orc_bilu0_factor.argtypes = [C.c_int, P64, PI, PD, PI, PI, PD]
        lib.orc_bilu0_apply.argtypes = [C.c_int, P64, PI, PD, PI, PI, PD, PD, PD]
        lib.orc_fgmres.argtypes = [C.c_int, P64, PI, PD, P64, PI, PD, PI, PI, PD, PD, PD,
                                   C.c_double, C.c_int, C.c_int, PD, PD]
        lib._krylov_ready = True
    return lib


def cell_orders(n, m, l, kind="natural"):
    """Cell elimination orders: 'natural' (FIND_ROW2 order) or 'color8'
    ((i%2, j%2, k%2) colour classes, natural order inside each)."""
    ncell = n * m * l
    c = np.arange(ncell)
    if kind == "natural":
        order = c
    elif kind == "color8":
        i, j, k = c % n, (c // n) % m, c // (n * m)
        col = (i % 2) + 2 * (j % 2) + 4 * (k % 2)
        order = np.lexsort((c, col))
    else:
        raise KeyError(kind)
    order = np.ascontiguousarray(order, dtype=np.int32)
    rank = np.empty(ncell, dtype=np.int32)
    rank[order] = np.arange(ncell, dtype=np.int32)
    return order, rank


class BILU0:
    def __init__(self, rowptr, col, val, ncell, order, rank):
        lib = _load_krylov()
        self.lib = lib
        self.ncell = ncell
        nb = lib.orc_bcsr_build(ncell, _p(rowptr, C.c_int64), _p(col, C.c_int), _p(val, C.c_double),
                                None, None, None, 0)
        self.bptr = np.zeros(ncell + 1, dtype=np.int64)
        self.bcol = np.zeros(nb, dtype=np.int32)
        self.bval = np.zeros(nb * 36)
        lib.orc_bcsr_build(ncell, _p(rowptr, C.c_int64), _p(col, C.c_int), _p(val, C.c_double),
                           _p(self.bptr, C.c_int64), _p(self.bcol, C.c_int),
                           _p(self.bval, C.c_double), nb)
        self.order, self.rank = order, rank
        self.dinv = np.zeros(ncell * 36)
        rc = lib.orc_bilu0_factor(ncell, _p(self.bptr, C.c_int64), _p(self.bcol, C.c_int),
                                  _p(self.bval, C.c_double), _p(order, C.c_int), _p(rank, C.c_int),
                                  _p(self.dinv, C.c_double))
        if rc:
            raise RuntimeError(f"BILU0: singular pivot at cell {rc - 1}")

    def apply(self, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros_like(r)
        self.lib.orc_bilu0_apply(self.ncell, _p(self.bptr, C.c_int64), _p(self.bcol, C.c_int),
                                 _p(self.bval, C.c_double), _p(self.order, C.c_int),
                                 _p(self.rank, C.c_int), _p(self.dinv, C.c_double),
                                 _p(r, C.c_double), _p(z, C.c_double))
        return z


def fgmres(rowptr, col, val, b, prec=None, tol=1e-8, m=500, maxit=500):
    lib = _load_krylov()
    N = len(rowptr) - 1
    x = np.zeros(N)
    rel = C.c_double()
    hist = np.zeros(maxit + 1)
    b = np.ascontiguousarray(b, dtype=np.float64)
    if prec is None:
        it = lib.orc_fgmres(N // 6, _p(rowptr, C.c_int64), _p(col, C.c_int), _p(val, C.c_double),
                            None, None, None, None, None, None, _p(b, C.c_double),
                            _p(x, C.c_double), tol, m, maxit, C.byref(rel), _p(hist, C.c_double))
    else:
        it = lib.orc_fgmres(N // 6, _p(rowptr, C.c_int64), _p(col, C.c_int), _p(val, C.c_double),
                            _p(prec.bptr, C.c_int64), _p(prec.bcol, C.c_int),
                            _p(prec.bval, C.c_double), _p(prec.order, C.c_int),
                            _p(prec.rank, C.c_int), _p(prec.dinv, C.c_double),
                            _p(b, C.c_double), _p(x, C.c_double), tol, m, maxit, C.byref(rel),
                            _p(hist, C.c_double))
    return x, it, rel.value, hist[:it]


# ------------------------------------------------------------------------------------
# block Gauss-Seidel preconditioner (prec_oracle.c) -- CPU twin of prec_gs.hip

def _load_gs():
    lib = _load_krylov()
    if not hasattr(lib, "_gs_ready"):
        P64, PI, PD = C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_double)
        lib.orc_gs_create.restype = C.c_void_p
        lib.orc_gs_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, P64, PI, PD, C.c_int64,
                                      C.c_int, PD, C.c_int]
        lib.orc_gs_destroy.argtypes = [C.c_void_p]
        lib.orc_gs_apply.argtypes = [C.c_void_p, PD, PD]
        lib.orc_gs_ncol.argtypes = [C.c_void_p]
        lib.orc_gs_band.argtypes = [C.c_void_p]
        lib.orc_gs_schur.argtypes = [C.c_void_p, PD, PI, C.POINTER(C.c_uint8)]
        lib.orc_gs_config.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_int]
        lib.orc_gs_ts_at.argtypes = [C.c_void_p, C.c_int]
        lib.orc_gs_dyn_krylov.argtypes = [C.c_void_p, C.c_int]
        lib.orc_gs_schur_passes.argtypes = [C.c_void_p, C.c_int]
        lib.orc_gs_schur_mask.argtypes = [C.c_void_p, C.c_int]
        lib.orc_fgmres_gs.argtypes = [C.c_int, P64, PI, PD, C.c_void_p, PD, PD, C.c_double,
                                      C.c_int, C.c_int, PD, PD]
        lib._gs_ready = True
    return lib


class BlockGS:
    """CPU block Gauss-Seidel preconditioner on the oracle's CSR Jacobian."""

    def __init__(self, o: "Oracle", val, ts_sweeps: int = 3, dyn_iters: int = 1,
                 dyn_omega: float = 1.0, ts_mg: int = 0, ts_at: int = 0, dyn_krylov: int = 0,
                 schur_passes: int = 0, schur_mask: int = 0):
        """ts_sweeps plain T/S sweeps, or (ts_mg > 0) the GPU's default variant: dyn_iters
        defect-correction passes of step dyn_omega on the dynamics block and ts_mg
        aggregation-multigrid V-cycles with z-line smoothing on the T/S block; the T/S
        right-hand side is formed after ts_at dynamics passes (0: after the last)."""
        lib = _load_gs()
        self.lib = lib
        d = o.d
        self.o = o
        self.val = np.ascontiguousarray(val, dtype=np.float64)
        self.intc = np.ascontiguousarray(o.intcond_coeff())
        self.h = lib.orc_gs_create(d["n"], d["m"], d["l"], d["periodic"],
                                   _p(o.rowptr, C.c_int64), _p(o.col, C.c_int),
                                   _p(self.val, C.c_double), o.rowintcon, d["int_sign"],
                                   _p(self.intc, C.c_double), ts_sweeps)
        if not self.h:
            raise RuntimeError("BlockGS: singular Schur complement")
        if lib.orc_gs_config(self.h, dyn_iters, dyn_omega, ts_mg) != 0:
            raise RuntimeError("BlockGS: the T/S multigrid needs a coarse level")
        lib.orc_gs_ts_at(self.h, ts_at)
        lib.orc_gs_dyn_krylov(self.h, dyn_krylov)
        lib.orc_gs_schur_passes(self.h, schur_passes)
        lib.orc_gs_schur_mask(self.h, schur_mask)   # study: which correction passes solve it
        self.ncol = lib.orc_gs_ncol(self.h)
        self.band = lib.orc_gs_band(self.h)

    def schur(self):
        """the pinned 2-D Schur matrix (scipy CSR over the water columns in band order),
        the (j*n+i) position and the pin flag of every column"""
        import scipy.sparse as sp
        ncol, bl = self.ncol, self.band
        W = 3 * bl + 1
        band = np.zeros(ncol * W)
        ij = np.zeros(ncol, dtype=np.int32)
        pin = np.zeros(ncol, dtype=np.uint8)
        self.lib.orc_gs_schur(self.h, _p(band, C.c_double), _p(ij, C.c_int),
                              _p(pin, C.c_uint8))
        band = band.reshape(ncol, W)
        r, d = np.nonzero(band)
        S = sp.csr_matrix((band[r, d], (r, r + d - bl)), shape=(ncol, ncol))
        return S, ij, pin.astype(bool)

    def __del__(self):
        try:
            self.lib.orc_gs_destroy(self.h)
        except Exception:
            pass

    def apply(self, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros_like(r)
        self.lib.orc_gs_apply(self.h, _p(r, C.c_double), _p(z, C.c_double))
        return z

    def fgmres(self, b, tol=1e-8, m=500, maxit=500):
        o = self.o
        N = len(o.rowptr) - 1
        x = np.zeros(N)
        rel = C.c_double()
        hist = np.zeros(maxit + 1)
        b = np.ascontiguousarray(b, dtype=np.float64)
        it = self.lib.orc_fgmres_gs(N // 6, _p(o.rowptr, C.c_int64), _p(o.col, C.c_int),
                                    _p(self.val, C.c_double), self.h, _p(b, C.c_double),
                                    _p(x, C.c_double), tol, m, maxit, C.byref(rel),
                                    _p(hist, C.c_double))
        return x, it, rel.value, hist[:it]


# ------------------------------------------------------------------------------------
# block ILU(0) (ilu_oracle.c) -- CPU twin of ilu.hip (the MRILU seam)

class BlockILU:
    """CPU block ILU(0) of a 0-based CSR matrix (int64 row pointers), block size bs."""

    def __init__(self, rowptr, col, val, bs: int = 6):
        lib = _load_krylov()
        if not hasattr(lib, "_ilu_ready"):
            lib.orc_ilu_create.restype = C.c_void_p
            lib.orc_ilu_create.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int),
                                           C.POINTER(C.c_double), C.c_int]
            lib.orc_ilu_apply.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
            lib.orc_ilu_destroy.argtypes = [C.c_void_p]
            lib.orc_ilu_perturbed.argtypes = [C.c_void_p]
            lib._ilu_ready = True
        self.lib = lib
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.val = np.ascontiguousarray(val, dtype=np.float64)
        self.n = len(self.rowptr) - 1
        self.h = lib.orc_ilu_create(self.n, _p(self.rowptr, C.c_int64), _p(self.col, C.c_int),
                                    _p(self.val, C.c_double), bs)
        if not self.h:
            raise RuntimeError("BlockILU: bad block size")
        self.perturbed = lib.orc_ilu_perturbed(self.h)

    def apply(self, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros_like(r)
        self.lib.orc_ilu_apply(self.h, _p(r, C.c_double), _p(z, C.c_double))
        return z

    def __del__(self):
        try:
            self.lib.orc_ilu_destroy(self.h)
        except Exception:
            pass


# ------------------------------------------------------------------------------------
# coupled ocean + atmosphere Newton step on the CPU (CoupledModel.C, bench cpu_baseline)

def coupled_newton_step(cfg, landm, xo, xa, comb, atm_params, ts_sweeps=12, dyn_iters=4,
                        dyn_omega=0.95, ts_mg=1, tol=1e-8, m=100, maxit=600, schur_passes=0):
    """One Newton step of CoupledModel (solving scheme 'C', preconditioning 'F') on the CPU
    restatements: synchronize (Ocean::synchronize(atmos): T, q, A, dimensional P over water,
    CommPars; Atmosphere: SST), F and J of the ocean (thcm_oracle.c in coupled mode) and of
    the atmosphere (atmos_oracle.py), the coupling blocks (Ocean::getBlock /
    Atmosphere::getBlock), FGMRES(m) on [ocean | atmosphere] with the forward block
    Gauss-Seidel preconditioner (ocean: prec_oracle.c block GS; atmosphere: sparse LU
    with r_a - C_ao z_o), x += dx, F(x + dx).  Returns timings and norms."""
    import time
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    from . import atmos_oracle as ao
    t_all = time.perf_counter()
    n, mm, l = cfg.n, cfg.m, cfg.l
    o = Oracle(cfg.ref_dict(), landm, cfg.par_list())
    o.set_par(19, comb)
    surf = (landm[l, 1:mm + 1, 1:n + 1] != 0).astype(int)
    deps0 = o.get_deps()
    at = ao.AtmosOracle(n, mm, cfg.xmin, cfg.xmax, cfg.ymin, cfg.ymax, cfg.periodic, surf,
                        Ooa=deps0[0], Os=deps0[1], params={**atm_params, "Combined Forcing": comb})
    No = 6 * n * mm * l
    top = 6 * (((l - 1) * mm) * n + np.arange(n * mm)) + 4     # surface T rows

    def sync(xo_, xa_):
        T, Q, A = xa_[0:3 * n * mm:3], xa_[1:3 * n * mm:3], xa_[2:3 * n * mm:3]
        P = at.P
        pf = np.where(surf.reshape(-1) == 0, at.pdist * (P.Eo0 + P.eta * P.qdim * xa_[at.rowP]), 0.0)
        o.set_atmos(T, Q, A, at.P.commpars(), p=pf if cfg.coupled_s else None)
        return xo_[top]

    def rhs(xo_, xa_):
        sst = sync(xo_, xa_)
        return np.concatenate([o.rhs(xo_), at.rhs(xa_, sst)])

    t = time.perf_counter()
    F0 = rhs(xo, xa)
    t_rhs = time.perf_counter() - t
    t = time.perf_counter()
    val, _ = o.jacobian(xo)
    Jo = sp.csr_matrix((val, o.col, o.rowptr), shape=(No, No))
    Ja = at.jacobian(xa).tocsc()
    Cao = at.block_from_ocean(l).tocsr()
    Coa = at.block_to_ocean(l, surf, o.get_deps(), comb, o.get_par(10), coupled_s=bool(cfg.coupled_s),
                            rowintcon=o.rowintcon).tocsr()
    A = sp.bmat([[Jo, Coa], [Cao, Ja]]).tocsr()
    t_jac = time.perf_counter() - t
    t = time.perf_counter()
    G = BlockGS(o, val, ts_sweeps, dyn_iters=dyn_iters, dyn_omega=dyn_omega, ts_mg=ts_mg,
                schur_passes=schur_passes)
    lu = spla.splu(Ja)
    t_prec = time.perf_counter() - t

    def prec(r):
        zo = G.apply(r[:No])
        return np.concatenate([zo, lu.solve(r[No:] - Cao @ zo)])

    t = time.perf_counter()
    b = -F0
    nb = np.linalg.norm(b)
    x = np.zeros_like(b)
    its = 0
    rel = 1.0
    V = np.zeros((m + 1, len(b)))
    Z = np.zeros((m, len(b)))
    while its < maxit and rel > tol:                       # FGMRES(m), x0 = 0, restarts
        r = b - A @ x
        beta = np.linalg.norm(r)
        V[0] = r / beta
        H = np.zeros((m + 1, m))
        g = np.zeros(m + 1)
        g[0] = beta
        for k in range(m):
            Z[k] = prec(V[k])
            w = A @ Z[k]
            for rep in range(2):                            # CGS2
                h = V[:k + 1] @ w
                w -= h @ V[:k + 1]
                H[:k + 1, k] += h
            H[k + 1, k] = np.linalg.norm(w)
            V[k + 1] = w / H[k + 1, k]
            its += 1
            y = np.linalg.lstsq(H[:k + 2, :k + 1], g[:k + 2], rcond=None)[0]
            rel = np.linalg.norm(H[:k + 2, :k + 1] @ y - g[:k + 2]) / nb
            if rel <= tol or its >= maxit:
                break
        x = x + y @ Z[:len(y)]
        rel = np.linalg.norm(b - A @ x) / nb
    t_solve = time.perf_counter() - t
    F1 = rhs(xo + x[:No], xa + x[No:])
    total = time.perf_counter() - t_all
    return dict(total=total, t_rhs=t_rhs, t_jac=t_jac, t_prec=t_prec, t_solve=t_solve, iters=its,
                rel=rel, norm_f0=float(np.linalg.norm(F0)), norm_f1=float(np.linalg.norm(F1)))
