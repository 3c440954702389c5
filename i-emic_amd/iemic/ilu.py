"""Block ILU(0) factor handles on the GPU (include/iemic.h iemic_ilu_*): the build's
replacement for the reference's MRILU seam (src/mrilucpp/Ifpack_MRILU.cpp:22-39,
mrilucpp_create / compute / apply / destroy on a rank-local 0-based CSR)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, ptr


class BlockILU:
    """``mrilucpp_create(id, n, nnz, beg, jco, co)`` + ``mrilucpp_compute(id)``: the CSR is
    copied to the device as bs x bs blocks and factorised by block ILU(0)."""

    def __init__(self, rowptr, col, val, bs: int = 6, device: int = 0):
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = np.ascontiguousarray(val, dtype=np.float64)
        self.n = len(rowptr) - 1
        h = C.c_void_p()
        check(lib().iemic_ilu_create(C.byref(h), device, self.n, C.c_int64(int(rowptr[-1])),
                                     ptr(rowptr, C.c_int64), ptr(col, C.c_int), ptr(val), bs),
              "iemic_ilu_create")
        self._h = h
        check(lib().iemic_ilu_compute(h), "iemic_ilu_compute")

    def apply(self, r: np.ndarray) -> np.ndarray:
        """``mrilucpp_apply(id, n, rhs, sol)``"""
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros_like(r)
        check(lib().iemic_ilu_apply(self._h, ptr(r), ptr(z)), "iemic_ilu_apply")
        return z

    def stats(self):
        """(levels of the lower solve, of the upper solve, unit-completed pivot columns)"""
        lo, up, pt = C.c_int(), C.c_int(), C.c_int()
        check(lib().iemic_ilu_stats(self._h, C.byref(lo), C.byref(up), C.byref(pt)), "iemic_ilu_stats")
        return lo.value, up.value, pt.value

    def close(self):
        if getattr(self, "_h", None):
            lib().iemic_ilu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
