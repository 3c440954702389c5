"""Test helpers: golden fixtures, mask fix-up, the CPU emulation harness wrapper."""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np

from iemic import _lib
from iemic import config as cf

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
EMUL_LIB = os.path.join(HERE, "_build", "libstencil_emul.so")
P = C.POINTER


def manifest() -> dict:
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_landm(name: str) -> np.ndarray:
    c = cf.preset(name, mixing=0)
    g = golden(name)
    return g["landm_local"].astype(np.int32).reshape(c.l + 2, c.m + 2, c.n + 2)


def state(cfg, landm, kind: str, g: dict | None = None) -> np.ndarray:
    if kind == "zero":
        return np.zeros(cfg.nrows)
    if kind == "synthetic":
        return cf.synthetic_state(cfg, landm)
    return g[f"{kind}_x"]


def mask_fix(orc, cfg, L, max_fix: int = 5):
    """Ocean::analyzeJacobian1 (Ocean.C:1877-1938) restated on the oracle: pressure rows
    with at most two entries |v| > 1e-10 at the zero state become land."""
    L = L.copy()
    for _ in range(max_fix):
        o = orc.Oracle(cfg.ref_dict(), L, cfg.par_list())
        val, _ = o.jacobian(np.zeros(o.N))
        bad = []
        for cell in range(cfg.ncell):
            row = 6 * cell + 3
            v = val[o.rowptr[row]:o.rowptr[row + 1]]
            i, j, k = cell % cfg.n, (cell // cfg.n) % cfg.m, cell // (cfg.n * cfg.m)
            if v.sum() == 1:
                continue
            if np.sum(np.abs(v) > 1e-10) <= 2:
                bad.append((i, j, k))
        if not bad:
            return L
        for i, j, k in bad:
            L[k + 1, j + 1, i + 1] = 1
    return L


def emul_lib():
    """the CPU emulation library of the device assembly (tests/emul)"""
    return C.CDLL(EMUL_LIB)


class Emul:
    """ctypes wrapper of tests/emul/stencil_emul.cpp: one latitude band (default: all), or
    with sub=(rank, nranks, npx) the library's Decomp2D subdomain of that rank."""

    def __init__(self, cfg, landm, jb0: int = 0, jb1: int = -1, sub=None):
        lib = C.CDLL(EMUL_LIB)
        vp = C.c_void_p
        lib.emul_create_band.restype = vp
        lib.emul_create_band.argtypes = [P(_lib.Grid), P(C.c_int), C.c_int, C.c_int]
        lib.emul_create_sub.restype = vp
        lib.emul_create_sub.argtypes = [P(_lib.Grid), P(C.c_int), C.c_int, C.c_int, C.c_int]
        lib.emul_sub_info.argtypes = [vp, P(C.c_int)]
        lib.emul_plan.restype = C.c_int
        lib.emul_plan.argtypes = [vp, C.c_int, C.c_int, C.c_int, P(C.c_int64), C.c_int]
        lib.emul_destroy.argtypes = [vp]
        lib.emul_set_par.argtypes = [vp, C.c_int, C.c_double]
        lib.emul_ext_rows.restype = C.c_int64
        lib.emul_ext_rows.argtypes = [vp]
        lib.emul_jacobian_ext.argtypes = [vp, P(C.c_double), P(C.c_double)]
        lib.emul_rhs_ext.argtypes = [vp, P(C.c_double), P(C.c_double), P(C.c_double)]
        lib.emul_to_csr.restype = C.c_int64
        lib.emul_to_csr.argtypes = [vp, P(C.c_int64), P(C.c_int), P(C.c_double)]
        lib.emul_ref_to_ext.argtypes = [vp, P(C.c_double), P(C.c_double)]
        lib.emul_ext_to_ref.argtypes = [vp, P(C.c_double), P(C.c_double)]
        self.lib = lib
        self.cfg = cfg
        g = _lib.grid_from_config(cfg, analyze_jacobian=False)
        L = np.ascontiguousarray(landm.reshape(-1), dtype=np.int32)
        if sub is None:
            self.h = lib.emul_create_band(C.byref(g), _lib.ptr(L, C.c_int), jb0, jb1)
            self.ib0, self.ib1, self.jb0, self.jb1 = 0, cfg.n, jb0, cfg.m if jb1 < 0 else jb1
            self.nb = [-1, -1, -1, -1]
        else:
            self.h = lib.emul_create_sub(C.byref(g), _lib.ptr(L, C.c_int), *sub)
            if not self.h:
                raise ValueError(f"decomposition {sub} refused")
            info = (C.c_int * 10)()
            lib.emul_sub_info(self.h, info)
            self.ib0, self.ib1, self.jb0, self.jb1, self.npx, self.npy = info[:6]
            self.nb = list(info[6:10])
        for idx, v in cfg.par_list():
            lib.emul_set_par(self.h, idx, v)
        self.ext_rows = lib.emul_ext_rows(self.h)

    def plan(self, width: int, depth: int, phase: int):
        """the library's halo-exchange plan: [(send, peer, off, nblk, len, stride)]"""
        out = np.zeros(6 * 64, dtype=np.int64)
        k = self.lib.emul_plan(self.h, width, depth, phase, _lib.ptr(out, C.c_int64), 64)
        return [tuple(int(v) for v in out[6 * q:6 * q + 6]) for q in range(k)]

    def __del__(self):
        try:
            self.lib.emul_destroy(self.h)
        except Exception:
            pass

    # layout -------------------------------------------------------------------------
    def to_ext(self, x_ref, ext=None):
        ext = np.zeros(self.ext_rows) if ext is None else ext
        self.lib.emul_ref_to_ext(self.h, _lib.ptr(np.ascontiguousarray(x_ref, dtype=np.float64)),
                                 _lib.ptr(ext))
        return ext

    def to_ref(self, ext, ref=None):
        ref = np.zeros(self.cfg.nrows) if ref is None else ref
        self.lib.emul_ext_to_ref(self.h, _lib.ptr(ext), _lib.ptr(ref))
        return ref

    # band-level (ext) calls -----------------------------------------------------------
    def jacobian_ext(self, xe):
        Be = np.zeros(self.ext_rows)
        self.lib.emul_jacobian_ext(self.h, _lib.ptr(xe), _lib.ptr(Be))
        return Be

    def csr(self):
        nnz = self.lib.emul_to_csr(self.h, None, None, None)
        nrow = 6 * (self.ib1 - self.ib0) * self.cfg.l * (self.jb1 - self.jb0)
        rowptr = np.zeros(nrow + 1, dtype=np.int64)
        col = np.zeros(nnz, dtype=np.int32)
        val = np.zeros(nnz)
        self.lib.emul_to_csr(self.h, _lib.ptr(rowptr, C.c_int64), _lib.ptr(col, C.c_int),
                             _lib.ptr(val))
        return rowptr, col, val

    def rhs_ext(self, xe):
        Fe = np.zeros(self.ext_rows)
        part = C.c_double()
        self.lib.emul_rhs_ext(self.h, _lib.ptr(xe), _lib.ptr(Fe), C.byref(part))
        return Fe, part.value

    # whole-grid convenience (reference order in and out) -------------------------------
    def jacobian_csr(self, x):
        xe = self.to_ext(x)
        Be = self.jacobian_ext(xe)
        rowptr, col, val = self.csr()
        return rowptr, col, val, self.to_ref(Be)

    def rhs(self, x):
        Fe, _ = self.rhs_ext(self.to_ext(x))
        return self.to_ref(Fe)


def emul_set_atmosphere(e: "Emul", t, q, a, pars, p=None) -> None:
    """iemic_set_atmosphere on the CPU emulation of the device assembly."""
    lib = e.lib
    lib.emul_set_atmosphere.argtypes = [C.c_void_p] + [P(C.c_double)] * 5
    p = np.zeros_like(np.asarray(t, dtype=np.float64)) if p is None else p
    arrs = [np.ascontiguousarray(v, dtype=np.float64) for v in (t, q, a, p, pars)]
    lib.emul_set_atmosphere(e.h, *[_lib.ptr(v) for v in arrs])


def emul_get_deps(e: "Emul") -> np.ndarray:
    out = np.zeros(7)
    e.lib.emul_get_deps.argtypes = [C.c_void_p, P(C.c_double)]
    e.lib.emul_get_deps(e.h, _lib.ptr(out))
    return out


def free_port() -> int:
    """A TCP port nothing listens on now (for gloo rendezvous on 127.0.0.1): fixed ports
    collide when several test workers (pytest -n) start process groups at once."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]
