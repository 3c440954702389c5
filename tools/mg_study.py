"""Preconditioner study (CPU, scipy; development tool, not product or test): see DESIGN.md §4.

usage: python tools/mg_study.py [global4]
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
cell = iT // 6; vv = iT % 6
i = cell % n; j = (cell // n) % m; k = cell // (n * m)
lu = spla.splu(Att.tocsc())
rng = np.random.default_rng(1)
b = rng.standard_normal(len(iT)); xe = lu.solve(b)
def err(z): return np.linalg.norm(z - xe) / np.linalg.norm(xe)

def build_levels(A, i, j, k, vv, n, m, l, agg=(2,2,2), nlev=6):
    levels = []
    for lev in range(nlev):
        # smoother blocks: colours by parity (+ extra for odd periodic)
        col = (i + j + k) % 2 + 2 * ((i == n - 1) & (n % 2 == 1))
        cellid = (k * m + j) * n + i
        bl = []
        for q in range(col.max() + 1):
            idx = np.flatnonzero(col == q)
            bl.append((idx, spla.splu(A[idx][:, idx].tocsc())))
        levels.append(dict(A=A, bl=bl))
        if len(vv) < 100 or lev == nlev - 1:
            levels[-1]["lu"] = spla.splu(A.tocsc())
            break
        ai, aj, ak = agg
        nc, mc, lc = (n + ai - 1) // ai, (m + aj - 1) // aj, (l + ak - 1) // ak
        ci, cj, ck = i // ai, j // aj, k // ak
        key = ((ck * mc + cj) * nc + ci) * 2 + (vv - 4)
        uk, inv = np.unique(key, return_inverse=True)
        P = sp.csr_matrix((np.ones(len(vv)), (np.arange(len(vv)), inv)), shape=(len(vv), len(uk)))
        levels[-1]["P"] = P
        A = (P.T @ A @ P).tocsr()
        cc = uk // 2; vv = uk % 2 + 4
        i, j, k = cc % nc, (cc // nc) % mc, cc // (nc * mc)
        n, m, l = nc, mc, lc
    return levels

def smooth(lv, bb, z, sweeps):
    A = lv["A"]; bl = lv["bl"]
    seq = list(range(len(bl))) + list(range(len(bl)))[::-1]
    for _ in range(sweeps):
        for q in seq:
            idx, f = bl[q]
            r = bb - A @ z
            z[idx] += f.solve(r[idx])
    return z

def vcycle(levels, lev, bb, nu, alpha, cyc="V"):
    lv = levels[lev]
    if "lu" in lv and lev == len(levels) - 1:
        return lv["lu"].solve(bb)
    z = smooth(lv, bb, np.zeros_like(bb), nu)
    r = bb - lv["A"] @ z
    rc = lv["P"].T @ r
    ec = vcycle(levels, lev + 1, rc, nu, alpha, cyc)
    if cyc == "W":
        rc2 = rc - levels[lev+1]["A"] @ ec
        ec = ec + vcycle(levels, lev + 1, rc2, nu, alpha, cyc)
    z += alpha * (lv["P"] @ ec)
    z = smooth(lv, bb, z, nu)
    return z

if __name__ == "__main__":
    for agg in ((2,2,1),(2,2,2)):
      levels = build_levels(Att, i, j, k, vv, n, m, l, agg=agg)
      print("agg", agg, "levels", [lv["A"].shape[0] for lv in levels])
      for nu in (1, 2):
          for alpha in (1.0, 1.5):
              for cyc in ("V", "W"):
                  z = vcycle(levels, 0, b, nu, alpha, cyc)
                  # 2 cycles as stationary iteration
                  z2 = z + vcycle(levels, 0, b - Att @ z, nu, alpha, cyc)
                  print(f"  nu={nu} alpha={alpha} {cyc}: 1 cycle err {err(z):.3e}, 2 cycles {err(z2):.3e}", flush=True)
