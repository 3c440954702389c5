"""Preconditioner study (CPU, scipy; development tool, not product or test): see DESIGN.md §4.

usage: python tools/ts_study.py [global4]
"""
import sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import numpy as np, scipy.sparse as sp, scipy.sparse.linalg as spla
from prec_study import setup
name = sys.argv[1] if len(sys.argv) > 1 else "global4"
c, L, o, x, val, F, A = setup(name, 1e-3)
N = c.nrows; n, m, l = c.n, c.m, c.l
d = A.diagonal(); rowabs = np.asarray(abs(A).sum(axis=1)).ravel()
known = (d == 1.0) & (rowabs == 1.0)
if o.rowintcon >= 0: known[o.rowintcon] = False
var = np.arange(N) % 6
iT = np.flatnonzero((~known) & (var >= 4))
A = A.tocsr(); Att = A[iT][:, iT].tocsr()
cell = iT // 6; i = cell % n; j = (cell // n) % m; k = cell // (n * m)
# magnitude of couplings by direction
coo = Att.tocoo(); ci = cell[coo.row]; cj = cell[coo.col]
dk = (cj // (n*m)) - (ci // (n*m)); dj = ((cj // n) % m) - ((ci // n) % m); di = (cj % n) - (ci % n)
same = cj == ci
for lab, msk in (("diag-cell", same), ("vertical", (dk != 0) & (dj == 0) & (di == 0)), ("horizontal", (dk == 0) & ~same)):
    print(lab, np.abs(coo.data[msk]).sum() / len(iT))
lu = spla.splu(Att.tocsc())
rng = np.random.default_rng(1)
b = rng.standard_normal(len(iT)); xe = lu.solve(b)
def err(z): return np.linalg.norm(z - xe) / np.linalg.norm(xe)
# point GS (cell 2x2 blocks), red-black on (i+j+k)
def blocks(colour_of):
    cols = colour_of
    res = []
    for q in range(cols.max() + 1):
        idx = np.flatnonzero(cols == q)
        res.append((idx, spla.splu(Att[idx][:, idx].tocsc())))
    return res
pt = blocks((i + j + k) % 2 + 2 * ((i == n - 1) & (n % 2 == 1)))
ln = blocks((i + j) % 2 + 2 * ((i == n - 1) & (n % 2 == 1)))
def gs(bl, sweeps):
    z = np.zeros(len(iT))
    seq = list(range(len(bl))) + list(range(len(bl)))[::-1]
    for _ in range(sweeps):
        for q in seq:
            idx, f = bl[q]
            r = b - Att @ z
            z[idx] += f.solve(r[idx])
    return z
for s in (1, 2, 4, 8, 12, 20):
    print(f"sweeps {s}: point {err(gs(pt, s)):.3e}  zline {err(gs(ln, s)):.3e}", flush=True)
