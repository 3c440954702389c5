"""Preconditioner study (CPU, scipy; development tool, not product or test): see DESIGN.md §4.

usage: python tools/mg_outer.py [global4]
"""
import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__))); 
import numpy as np, scipy.sparse.linalg as spla
import mg_study as M   # builds Att, levels helpers at import (global4)
from prec_study import gmres
o, val, A, F, N = M.o, M.val, M.A, M.F, M.N
import oracle.oracle as orc
d = A.diagonal(); rowabs = np.asarray(abs(A).sum(axis=1)).ravel()
known = (d == 1.0) & (rowabs == 1.0)
if o.rowintcon >= 0: known[o.rowintcon] = False
var = np.arange(N) % 6
iK, iD, iT = [np.flatnonzero(s) for s in (known, (~known) & (var <= 3), (~known) & (var >= 4))]
Add = A[iD][:, iD]; Adk = A[iD][:, iK]; Atd = A[iT][:, iD]; Atk = A[iT][:, iK]
P = orc.BlockGS(o, val, 12)
def PD(rd):
    r = np.zeros(N); r[iD] = rd
    return P.apply(r)[iD]
levels = M.build_levels(M.Att, M.i, M.j, M.k, M.vv, M.n, M.m, M.l, agg=(2, 2, 1))
def make(tsmode):
    def M_(r):
        z = P.apply(r)
        rrD = r[iD] - Adk @ z[iK]
        zD = z[iD] + PD(rrD - Add @ z[iD])
        z[iD] = zD
        rt = r[iT] - Atk @ z[iK] - Atd @ zD
        if tsmode == "exact": z[iT] = M.lu.solve(rt)
        else:
            nu, alpha, cyc = tsmode
            z[iT] = M.vcycle(levels, 0, rt, nu, alpha, cyc)
        return z
    return M_
for mode in [(1, 1.0, "V"), (2, 1.0, "V"), (3, 1.0, "V"), (1, 1.5, "W")]:
    t = time.time(); its, rr = gmres(A, -F, make(mode))
    print(mode, its, f"{rr:.2e}", f"{time.time()-t:.0f}s", flush=True)
