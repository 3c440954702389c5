"""Preconditioner study (CPU, scipy; development tool, not product or test): see DESIGN.md §4.

usage: python tools/dyn_study.py [global4]
"""
import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import numpy as np, scipy.sparse.linalg as spla
from prec_study import gmres, setup, orc
name = sys.argv[1] if len(sys.argv) > 1 else "global4"
c, L, o, x, val, F, A = setup(name, 1e-3)
N = c.nrows; b = -F
d = A.diagonal(); rowabs = np.asarray(abs(A).sum(axis=1)).ravel()
known = (d == 1.0) & (rowabs == 1.0)
if o.rowintcon >= 0: known[o.rowintcon] = False
var = np.arange(N) % 6
dyn = (~known) & (var <= 3); ts = (~known) & (var >= 4)
iK, iD, iT = [np.flatnonzero(s) for s in (known, dyn, ts)]
A = A.tocsr()
Add = A[iD][:, iD]; Adk = A[iD][:, iK]; Atd = A[iT][:, iD]; Atk = A[iT][:, iK]; Att = A[iT][:, iT].tocsc()
luT = spla.splu(Att)
P = orc.BlockGS(o, val, 12)
def PD(rd):
    r = np.zeros(N); r[iD] = rd
    return P.apply(r)[iD]
def make(k, exact_ts=True):
    def M(r):
        z = P.apply(r)
        rrD = r[iD] - Adk @ z[iK]
        zD = z[iD]
        for _ in range(k - 1):
            zD = zD + PD(rrD - Add @ zD)
        z[iD] = zD
        rt = r[iT] - Atk @ z[iK] - Atd @ zD
        if exact_ts:
            z[iT] = luT.solve(rt)
        else:
            rr = np.zeros(N); rr[iT] = rt
            # dyn part of rr is zero -> ts sweeps get rhs rt exactly (dyn z = 0)
            z[iT] = P.apply(rr)[iT]
        return z
    return M
for k in map(int, sys.argv[2:] or ["1", "2", "3", "4"]):
    for ex in (True, False):
        t = time.time(); its, rr = gmres(A, b, make(k, ex))
        print(f"dyn richardson k={k} exact_ts={ex}: its={its} rel={rr:.2e} ({time.time()-t:.0f}s)", flush=True)
