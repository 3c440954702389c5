"""Preconditioner study on the CPU (scipy): FGMRES iteration counts of block variants
on the oracle's Jacobian.  Development tool, not part of the product or the tests.

usage: python tools/prec_study.py [global4] [amp_ts]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd"), os.path.join(ROOT, "tests")]
from iemic import config as cf  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from helpers import mask_fix  # noqa: E402


def gmres(A, b, M, tol=1e-8, m=500):
    """right-preconditioned GMRES (== FGMRES for a fixed M), x0 = 0; returns its, relres"""
    n = len(b)
    beta = np.linalg.norm(b)
    V = np.zeros((m + 1, n)); Z = np.zeros((m, n)); H = np.zeros((m + 1, m))
    V[0] = b / beta
    g = np.zeros(m + 1); g[0] = beta
    cs = np.zeros(m); sn = np.zeros(m)
    for j in range(m):
        Z[j] = M(V[j])
        w = A @ Z[j]
        for _ in range(2):
            h = V[:j + 1] @ w
            w -= h @ V[:j + 1]
            H[:j + 1, j] += h
        H[j + 1, j] = np.linalg.norm(w)
        V[j + 1] = w / H[j + 1, j]
        for i in range(j):
            t = cs[i] * H[i, j] + sn[i] * H[i + 1, j]
            H[i + 1, j] = -sn[i] * H[i, j] + cs[i] * H[i + 1, j]
            H[i, j] = t
        r = np.hypot(H[j, j], H[j + 1, j])
        cs[j], sn[j] = H[j, j] / r, H[j + 1, j] / r
        H[j, j] = r; H[j + 1, j] = 0
        g[j + 1] = -sn[j] * g[j]; g[j] *= cs[j]
        if abs(g[j + 1]) <= tol * beta:
            return j + 1, abs(g[j + 1]) / beta
    return m, abs(g[m]) / beta


def setup(name, amp_ts):
    c = cf.preset(name, mixing=0)
    L0 = cf.landmask(c)
    L = mask_fix(orc, c, L0)
    o = orc.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=amp_ts)
    val, _ = o.jacobian(x)
    F = o.rhs(x)
    N = c.nrows
    A = sp.csr_matrix((val, o.col, o.rowptr), shape=(N, N))
    return c, L, o, x, val, F, A


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "global4"
    amp = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    c, L, o, x, val, F, A = setup(name, amp)
    N = c.nrows
    b = -F
    # identity rows
    d = A.diagonal()
    nnzr = np.diff(A.indptr)
    rowabs = np.asarray(abs(A).sum(axis=1)).ravel()
    known = (d == 1.0) & (rowabs == 1.0)
    if o.rowintcon >= 0:
        known[o.rowintcon] = False
    var = np.arange(N) % 6
    dyn = (~known) & (var <= 3)
    ts = (~known) & (var >= 4)
    print(f"{name}: N={N} known={known.sum()} dyn={dyn.sum()} ts={ts.sum()}")
    iK, iD, iT = [np.flatnonzero(s) for s in (known, dyn, ts)]
    Add = A[iD][:, iD].tocsc(); Atd = A[iT][:, iD]; Att = A[iT][:, iT].tocsc()
    t = time.time(); luD = spla.splu(Add); luT = spla.splu(Att)
    print(f"  exact LU of dyn/ts blocks: {time.time()-t:.1f}s")

    def ideal(r):
        z = np.zeros(N)
        z[iK] = r[iK]
        rd = r[iD] - A[iD][:, iK] @ z[iK]
        z[iD] = luD.solve(rd)
        rt = r[iT] - A[iT][:, iK] @ z[iK] - Atd @ z[iD]
        z[iT] = luT.solve(rt)
        return z
    its, rr = gmres(A, b, ideal)
    print(f"  ideal block-LT (exact dyn, exact ts): its={its} rel={rr:.2e}")
    P = orc.BlockGS(o, val, 12)
    its, rr = gmres(A, b, P.apply)
    print(f"  BlockGS(12 sweeps) : its={its} rel={rr:.2e}")

    # BlockGS dyn part + exact ts
    def gs_dyn_exact_ts(r):
        z = P.apply(r)
        rt = r[iT] - A[iT][:, iK] @ z[iK] - Atd @ z[iD]
        z[iT] = luT.solve(rt)
        return z
    its, rr = gmres(A, b, gs_dyn_exact_ts)
    print(f"  BlockGS dyn + exact ts: its={its} rel={rr:.2e}")

    def exact_dyn_gs_ts(r):
        z = P.apply(r)       # approximate dyn + ts
        z2 = np.zeros(N); z2[iK] = r[iK]
        z2[iD] = luD.solve(r[iD] - A[iD][:, iK] @ z2[iK])
        # re-run ts with GS on the corrected rhs: emulate via P on a masked residual
        rr_ = r.copy()
        rr_[iD] = 0; rr_[iK] = 0
        rr_[iT] = r[iT] - A[iT][:, iK] @ z2[iK] - Atd @ z2[iD]
        z3 = P.apply(rr_)
        z2[iT] = z3[iT]
        return z2
    its, rr = gmres(A, b, exact_dyn_gs_ts)
    print(f"  exact dyn + GS ts : its={its} rel={rr:.2e}")


if __name__ == "__main__":
    main()
