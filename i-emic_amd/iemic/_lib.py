"""ctypes binding of the device library's C ABI (include/iemic.h).

The library is built in-tree (``make -C i-emic_amd``) into ``i-emic_amd/lib/libiemic_amd.so``.
There is no CPU fallback: if the library or a GPU is missing, every call fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# IEMIC_LIB names another build of the library under lib/ (kernel A/B measurements of
# scripts/ab_probe.py run every variant on the same box); the default is the in-tree build
LIB_PATH = os.path.join(PKG_DIR, "lib", os.environ.get("IEMIC_LIB", "libiemic_amd.so"))

IEMIC_ENODEV = -19
ABI_VERSION = 6             # IEMIC_ABI_VERSION of include/iemic.h this binding mirrors
IEMIC_ENOCONV = 1           # iemic_newton_step: applied, but the solve missed its tolerance


class Grid(C.Structure):
    """iemic_grid (include/iemic.h)."""
    _fields_ = [("n", C.c_int), ("m", C.c_int), ("l", C.c_int),
                ("xmin", C.c_double), ("xmax", C.c_double), ("ymin", C.c_double),
                ("ymax", C.c_double), ("periodic", C.c_int), ("hdim", C.c_double),
                ("qz", C.c_double), ("tres", C.c_int), ("sres", C.c_int),
                ("forcing_type", C.c_int), ("ih", C.c_int), ("vmix", C.c_int),
                ("coriolis_on", C.c_int), ("alpha_t", C.c_double), ("alpha_s", C.c_double),
                ("int_sign", C.c_int), ("int_i", C.c_int), ("int_j", C.c_int),
                ("analyze_jacobian", C.c_int), ("max_mask_fixes", C.c_int),
                ("device", C.c_int), ("rho_mixing", C.c_int), ("coupled_t", C.c_int),
                ("coupled_s", C.c_int)]


class Dist(C.Structure):
    """iemic_dist: Decomp2D decomposition over nranks GPUs (RCCL unique id; npx x parts,
    0: the reference's factorisation, 1: latitude bands)."""
    _fields_ = [("rank", C.c_int), ("nranks", C.c_int), ("id", C.c_ubyte * 128), ("npx", C.c_int)]


SEND_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_int64)
RECV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_int64)
WAIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p)
ALLRED_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)


class Transport(C.Structure):
    """iemic_transport: the caller's host point-to-point and all-reduce."""
    _fields_ = [("user", C.c_void_p), ("send", SEND_FN), ("recv", RECV_FN), ("wait", WAIT_FN),
                ("allreduce_sum", ALLRED_FN)]


class Krylov(C.Structure):
    _fields_ = [("tol", C.c_double), ("krylov_dim", C.c_int), ("max_restarts", C.c_int),
                ("prec", C.c_int), ("ts_sweeps", C.c_int), ("orth", C.c_int),
                ("dyn_iters", C.c_int), ("method", C.c_int), ("ts_mg", C.c_int),
                ("mg_sweeps", C.c_int), ("dyn_omega", C.c_double), ("dyn_mr", C.c_int),
                ("idr_s", C.c_int), ("idr_angle", C.c_double), ("idr_replace", C.c_int),
                ("ts_at", C.c_int), ("schur_passes", C.c_int)]


class SolveInfo(C.Structure):
    _fields_ = [("iters", C.c_int), ("converged", C.c_int),
                ("implicit_rel_res", C.c_double), ("explicit_rel_res", C.c_double),
                ("t_prec_ms", C.c_double), ("t_spmv_ms", C.c_double),
                ("t_orth_ms", C.c_double), ("t_total_ms", C.c_double), ("reorth", C.c_int),
                ("n_spmv", C.c_int), ("safeguard", C.c_int)]


class AtmosParams(C.Structure):
    """iemic_atmos_params (include/iemic.h; AtmosLocal::setParameters names in order)."""
    NAMES = ["rhoa", "rhoo", "hdima", "hdimq", "cpa", "D0", "kappa", "arad", "brad", "sun0", "c0",
             "ce", "ch", "uw", "t0a", "t0o", "t0i", "tdim", "q0", "qdim", "lv", "udim", "r0dim",
             "a0", "da", "tauf_days", "tauc_days", "Tm", "Tr", "Pa", "epm", "epr", "epa"]
    _fields_ = [(k, C.c_double) for k in NAMES] + [("par", C.c_double * 7)]


class NewtonInfo(C.Structure):
    _fields_ = [("norm_f0", C.c_double), ("norm_f1", C.c_double), ("solve", SolveInfo),
                ("t_jac_ms", C.c_double), ("t_rhs_ms", C.c_double), ("t_prec_ms", C.c_double),
                ("t_solve_ms", C.c_double), ("t_total_ms", C.c_double)]


def grid_from_config(cfg, device: int = 0, analyze_jacobian: bool = True) -> Grid:
    return Grid(cfg.n, cfg.m, cfg.l, cfg.xmin, cfg.xmax, cfg.ymin, cfg.ymax, int(cfg.periodic),
                cfg.hdim, cfg.qz, cfg.tres, cfg.sres, cfg.forcing_type,
                cfg.inhomogeneous_mixing, cfg.mixing, cfg.coriolis, cfg.alpha_t, cfg.alpha_s,
                cfg.int_sign, cfg.integral_i, cfg.integral_j, int(analyze_jacobian), 5, device,
                int(cfg.rho_mixing), int(getattr(cfg, "coupled_t", 0)),
                int(getattr(cfg, "coupled_s", 0)))


_lib = None

P = C.POINTER
PD, PI, P64 = P(C.c_double), P(C.c_int), P(C.c_int64)


def ptr(a, t=C.c_double):
    return a.ctypes.data_as(P(t))


def lib():
    """Load the in-tree device library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"device library not built: {LIB_PATH} (run make -C i-emic_amd)")
    L = C.CDLL(LIB_PATH)
    if not os.environ.get("IEMIC_LIB"):
        # the structs below mirror one header version: a stale library must not be driven
        L.iemic_abi_version.restype = C.c_int
        got = L.iemic_abi_version() if hasattr(L, "iemic_abi_version") else None
        if got != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH}: ABI version {got}, this binding expects {ABI_VERSION} "
                               "(rebuild with make -C i-emic_amd)")
    vp = C.c_void_p
    sig = {
        "iemic_abi_version": (C.c_int, []),
        "iemic_create": (C.c_int, [P(vp), P(Grid), PI]),
        "iemic_create_dist": (C.c_int, [P(vp), P(Grid), PI, P(Dist)]),
        "iemic_comm_unique_id": (C.c_int, [P(C.c_ubyte)]),
        "iemic_layout": (C.c_int, [vp, P64]),
        "iemic_comm_stats": (C.c_int, [vp, P64]),
        "iemic_active_cells": (C.c_int, [vp, P64]),
        "iemic_comm_size": (C.c_int, [vp, PI, PI]),
        "iemic_allreduce_sum": (C.c_int, [vp, PD, C.c_int64]),
        "iemic_set_comm_timeout": (C.c_int, [vp, C.c_double]),
        "iemic_local_group_new": (vp, [C.c_int]),
        "iemic_local_group_free": (None, [vp]),
        "iemic_create_local": (C.c_int, [P(vp), P(Grid), PI, vp, C.c_int, C.c_int]),
        "iemic_create_local_2d": (C.c_int, [P(vp), P(Grid), PI, vp, C.c_int, C.c_int, C.c_int]),
        "iemic_create_transport": (C.c_int, [P(vp), P(Grid), PI, C.c_int, C.c_int, C.c_int, P(Transport)]),
        "iemic_decomp2d": (C.c_int, [C.c_int, C.c_int, C.c_int, PI, PI]),
        "iemic_destroy": (None, [vp]),
        "iemic_device_count": (C.c_int, []),
        "iemic_last_error": (C.c_char_p, []),
        "iemic_set_par": (C.c_int, [vp, C.c_int, C.c_double]),
        "iemic_get_par": (C.c_int, [vp, C.c_int, PD]),
        "iemic_nrows": (C.c_int, [vp]),
        "iemic_graph_nnz": (C.c_int64, [vp]),
        "iemic_rowintcon": (C.c_int, [vp]),
        "iemic_landm": (C.c_int, [vp, PI]),
        "iemic_set_state": (C.c_int, [vp, PD]),
        "iemic_get_state": (C.c_int, [vp, PD]),
        "iemic_set_state_dev": (C.c_int, [vp, vp]),
        "iemic_jacobian": (C.c_int, [vp]),
        "iemic_rhs": (C.c_int, [vp, PD]),
        "iemic_diag_b": (C.c_int, [vp, PD]),
        "iemic_export_csr": (C.c_int, [vp, P64, PI, PD]),
        "iemic_spmv": (C.c_int, [vp, PD, PD]),
        "iemic_spmv_dev": (C.c_int, [vp, vp, vp, vp]),
        "iemic_prec_compute": (C.c_int, [vp, P(Krylov)]),
        "iemic_prec_apply": (C.c_int, [vp, PD, PD]),
        "iemic_solve": (C.c_int, [vp, PD, PD, P(Krylov), P(SolveInfo)]),
        "iemic_solve_dev": (C.c_int, [vp, vp, vp, P(Krylov), P(SolveInfo)]),
        "iemic_newton_step": (C.c_int, [vp, P(Krylov), P(NewtonInfo)]),
        "iemic_vec_alloc": (C.c_int, [vp, P(vp)]),
        "iemic_vec_free": (C.c_int, [vp, vp]),
        "iemic_vec_update": (C.c_int, [vp, C.c_double, vp, C.c_double, vp, C.c_double, vp]),
        "iemic_vec_dot": (C.c_int, [vp, vp, vp, PD]),
        "iemic_vec_norm_inf": (C.c_int, [vp, vp, PD]),
        "iemic_vec_from_ref": (C.c_int, [vp, PD, vp]),
        "iemic_vec_to_ref": (C.c_int, [vp, vp, PD]),
        "iemic_state_vec": (C.c_int, [vp, vp, C.c_int]),
        "iemic_rhs_vec": (C.c_int, [vp, vp]),
        "iemic_time_spmv": (C.c_int, [vp, C.c_int, PD]),
        "iemic_time_prec": (C.c_int, [vp, C.c_int, PD, PD]),
        "iemic_time_prec_parts": (C.c_int, [vp, C.c_int, PD]),
        "iemic_time_spmv_cold": (C.c_int, [vp, C.c_int, vp, C.c_int64, PD]),
        "iemic_set_intcond_correction": (C.c_int, [vp, PD]),
        "iemic_get_intcond_correction": (C.c_int, [vp, PD]),
        "iemic_get_intcond_coeff": (C.c_int, [vp, PD]),
        "iemic_psim": (C.c_int, [vp, PD, PD, PD]),
        "iemic_integral_checks": (C.c_int, [vp, PD, PD]),
        "iemic_ilu_create": (C.c_int, [P(vp), C.c_int, C.c_int, C.c_int64, P64, PI, PD, C.c_int]),
        "iemic_ilu_compute": (C.c_int, [vp]),
        "iemic_ilu_apply": (C.c_int, [vp, PD, PD]),
        "iemic_ilu_apply_dev": (C.c_int, [vp, vp, vp]),
        "iemic_ilu_stats": (C.c_int, [vp, PI, PI, PI]),
        "iemic_ilu_destroy": (None, [vp]),
        "iemic_set_atmosphere": (C.c_int, [vp, PD, PD, PD, PD, PD]),
        "iemic_get_deps": (C.c_int, [vp, PD]),
        "iemic_get_suno": (C.c_int, [vp, PD]),
        "iemic_atmos_default_params": (C.c_int, [P(AtmosParams)]),
        "iemic_atmos_create": (C.c_int, [P(vp), vp, P(AtmosParams)]),
        "iemic_atmos_destroy": (None, [vp]),
        "iemic_atmos_dim": (C.c_int, [vp]),
        "iemic_atmos_set_par": (C.c_int, [vp, C.c_int, C.c_double]),
        "iemic_atmos_set_state": (C.c_int, [vp, PD]),
        "iemic_atmos_get_state": (C.c_int, [vp, PD]),
        "iemic_atmos_set_sst": (C.c_int, [vp, PD]),
        "iemic_atmos_rhs": (C.c_int, [vp, PD]),
        "iemic_atmos_jacobian": (C.c_int, [vp]),
        "iemic_atmos_spmv": (C.c_int, [vp, PD, PD]),
        "iemic_atmos_prec_apply": (C.c_int, [vp, PD, PD]),
        "iemic_atmos_export_ell": (C.c_int, [vp, PD, PI]),
        "iemic_atmos_integral_coeff": (C.c_int, [vp, PD, PD, PI, PI]),
        "iemic_atmos_commpars": (C.c_int, [vp, PD]),
        "iemic_atmos_pdist": (C.c_int, [vp, PD]),
        "iemic_coupled_create": (C.c_int, [P(vp), vp, vp]),
        "iemic_coupled_destroy": (None, [vp]),
        "iemic_coupled_synchronize": (C.c_int, [vp]),
        "iemic_coupled_rhs": (C.c_int, [vp, PD, PD]),
        "iemic_coupled_jacobian": (C.c_int, [vp]),
        "iemic_coupled_spmv": (C.c_int, [vp, PD, PD]),
        "iemic_coupled_solve": (C.c_int, [vp, PD, PD, P(Krylov), P(SolveInfo)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("IEMIC_LIB") and not hasattr(L, name):
            continue                  # an older build under A/B measurement lacks newer entry points
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


EXPORTED = ("iemic_abi_version", "iemic_create", "iemic_create_dist", "iemic_comm_unique_id", "iemic_layout",
            "iemic_comm_stats", "iemic_active_cells",
            "iemic_comm_size", "iemic_allreduce_sum", "iemic_set_comm_timeout",
            "iemic_local_group_new", "iemic_local_group_free", "iemic_create_local",
            "iemic_create_local_2d", "iemic_create_transport", "iemic_decomp2d",
            "iemic_destroy", "iemic_device_count", "iemic_last_error",
            "iemic_set_par", "iemic_get_par", "iemic_set_intcond_correction",
            "iemic_get_intcond_correction", "iemic_get_intcond_coeff", "iemic_psim",
            "iemic_integral_checks", "iemic_nrows", "iemic_graph_nnz",
            "iemic_rowintcon", "iemic_landm", "iemic_set_state", "iemic_get_state",
            "iemic_set_state_dev",
            "iemic_jacobian", "iemic_rhs", "iemic_diag_b", "iemic_export_csr", "iemic_spmv",
            "iemic_spmv_dev", "iemic_prec_compute", "iemic_prec_apply", "iemic_solve",
            "iemic_solve_dev", "iemic_newton_step", "iemic_vec_alloc", "iemic_vec_free",
            "iemic_vec_update", "iemic_vec_dot", "iemic_vec_norm_inf", "iemic_vec_from_ref",
            "iemic_vec_to_ref", "iemic_state_vec", "iemic_rhs_vec", "iemic_time_spmv", "iemic_time_spmv_cold", "iemic_time_prec",
            "iemic_time_prec_parts",
            "iemic_ilu_create", "iemic_ilu_compute", "iemic_ilu_apply", "iemic_ilu_apply_dev",
            "iemic_ilu_stats", "iemic_ilu_destroy",
            "iemic_set_atmosphere", "iemic_get_deps", "iemic_get_suno",
            "iemic_atmos_default_params", "iemic_atmos_create", "iemic_atmos_destroy",
            "iemic_atmos_dim", "iemic_atmos_set_par", "iemic_atmos_set_state",
            "iemic_atmos_get_state", "iemic_atmos_set_sst", "iemic_atmos_rhs",
            "iemic_atmos_jacobian", "iemic_atmos_spmv", "iemic_atmos_prec_apply",
            "iemic_atmos_export_ell", "iemic_atmos_integral_coeff", "iemic_atmos_commpars",
            "iemic_atmos_pdist", "iemic_coupled_create", "iemic_coupled_destroy",
            "iemic_coupled_synchronize", "iemic_coupled_rhs", "iemic_coupled_jacobian",
            "iemic_coupled_spmv", "iemic_coupled_solve")


def src_digest() -> str:
    """SHA-256 over the device library's sources (csrc/ and include/iemic.h, sorted by path):
    the key under which measured per-kernel tables (bench_data/pmc_*.json) apply."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*")))
    files.append(os.path.join(os.path.dirname(PKG_DIR), "include", "iemic.h"))
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


class IemicError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().iemic_last_error()
        raise IemicError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")
