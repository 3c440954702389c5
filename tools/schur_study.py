"""Barotropic (2-D Schur) solve study on the CPU (scipy): outer FGMRES iterations of the
SIMPLE dynamics pass when the pinned Schur solve S pbar = b is exact vs approximated by
colour-separated aggregation multigrid.  Development tool, not product or test.

usage: python tools/schur_study.py [global4] [amp_ts]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.csgraph as csg
import scipy.sparse.linalg as spla

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import simple_study  # noqa: E402
from prec_study import gmres, setup  # noqa: E402


class Dyn(simple_study.Dyn):
    def schur_pinv(self, Xinv):      # skip the dense pseudo-inverses of the parent
        return None


def schur_parts(dy, c):
    S = (dy.Mz2 @ dy.Apu @ dy.Dinv @ dy.Aup @ dy.E).tocsr()
    S.eliminate_zeros()
    # column (i, j) of each Schur unknown
    cp = (dy.iP // 6)
    ij = np.unique(cp % (c.n * c.m))
    ci, cj = ij % c.n, ij // c.n
    # null space: connected components of same-colour (diagonal) couplings
    co = S.tocoo()
    di = ci[co.col] - ci[co.row]
    di = np.where(di > 1, di - c.n, np.where(di < -1, di + c.n, di))
    dj = cj[co.col] - cj[co.row]
    diag = (di != 0) & (dj != 0)
    G = sp.csr_matrix((np.ones(diag.sum()), (co.row[diag], co.col[diag])), shape=S.shape)
    ncomp, lab = csg.connected_components(G, directed=False)
    pin = np.zeros(S.shape[0], bool)
    # pin the first unknown of each component in the GPU's band order (i folded, j fastest)
    n = c.n
    ipos = np.empty(n, int)
    a, b, q = 0, n - 1, 0
    while a <= b:
        ipos[a] = q; q += 1
        if a != b:
            ipos[b] = q; q += 1
        a += 1; b -= 1
    key = ipos[ci] * c.m + cj
    for comp in range(ncomp):
        idx = np.flatnonzero(lab == comp)
        pin[idx[np.argmin(key[idx])]] = True
    return S, ci, cj, pin


def pinned_matrix(S, pin):
    D = sp.diags((~pin).astype(float))
    Sp = (D @ S @ D).tolil()
    for q in np.flatnonzero(pin):
        Sp[q, q] = 1.0
    return Sp.tocsr()


class AggMG:
    """colour-separated pairwise/quad aggregation multigrid on the pinned Schur matrix"""

    def __init__(self, A, ci, cj, n, periodic, smoother="gs", nu=1, omega=0.8, coarse=200,
                 scheme="quad", alpha=1.0, cycle="V"):
        self.levels = []
        self.nu, self.omega, self.smoother, self.alpha, self.cycle = nu, omega, smoother, alpha, cycle
        colour = (ci + cj) % 2
        I, J = ci.copy(), cj.copy()
        lev = 0
        while True:
            lv = {"A": A.tocsr(), "d": A.diagonal().copy()}
            lv["dinv"] = np.where(lv["d"] != 0, 1.0 / np.where(lv["d"] != 0, lv["d"], 1), 0.0)
            # GS colouring for the smoother: 4 colours by (i%2, j%2)
            lv["col"] = (I % 2) + 2 * (J % 2)
            if A.shape[0] <= coarse:
                lv["lu"] = spla.splu(A.tocsc())
                self.levels.append(lv)
                break
            if lev == 0 and scheme in ("quad", "pair"):
                # red/black lattices: the 2x2 block (I//2, J//2) holds one aggregate per colour
                key = ((J // 2) * ((n + 1) // 2) + (I // 2)) * 2 + colour
                nI, nJ = I // 2, J // 2
                ncol_ = colour
            else:
                key = ((J // 2) * ((n + 1) // 2) + (I // 2)) * 2 + colour
                nI, nJ = I // 2, J // 2
                ncol_ = colour
            uk, inv = np.unique(key, return_inverse=True)
            P = sp.csr_matrix((np.ones(len(key)), (np.arange(len(key)), inv)), shape=(len(key), len(uk)))
            lv["P"] = P
            self.levels.append(lv)
            A = (P.T @ A @ P).tocsr()
            # coarse coordinates
            I = np.zeros(len(uk), int); J = np.zeros(len(uk), int); colour = np.zeros(len(uk), int)
            I[inv] = nI; J[inv] = nJ; colour[inv] = ncol_
            n = (n + 1) // 2
            lev += 1

    def smooth(self, lv, b, x, post):
        A = lv["A"]
        for _ in range(self.nu):
            if self.smoother == "jacobi":
                x = x + self.omega * lv["dinv"] * (b - A @ x)
            else:
                seq = [0, 1, 2, 3] if not post else [3, 2, 1, 0]
                for q in seq:
                    idx = np.flatnonzero(lv["col"] == q)
                    r = b[idx] - A[idx] @ x
                    x[idx] += lv["dinv"][idx] * r
        return x

    def cyc(self, q, b):
        lv = self.levels[q]
        if "lu" in lv:
            return lv["lu"].solve(b)
        x = self.smooth(lv, b, np.zeros_like(b), False)
        r = b - lv["A"] @ x
        rc = lv["P"].T @ r
        ec = self.cyc(q + 1, rc)
        if self.cycle == "W" and "lu" not in self.levels[q + 1]:
            ec = ec + self.cyc(q + 1, rc - self.levels[q + 1]["A"] @ ec)
        x = x + self.alpha * (lv["P"] @ ec)
        return self.smooth(lv, b, x, True)

    def solve(self, b, ncyc=1):
        x = np.zeros_like(b)
        for _ in range(ncyc):
            x = x + self.cyc(0, b - self.levels[0]["A"] @ x)
        return x


def inner_gmres(A, b, M, its):
    """fixed number of right-preconditioned GMRES steps (nonlinear in b; FGMRES outside)"""
    n = len(b)
    beta = np.linalg.norm(b)
    if beta == 0:
        return np.zeros(n)
    V = np.zeros((its + 1, n)); Z = np.zeros((its, n)); H = np.zeros((its + 1, its))
    V[0] = b / beta
    k = its
    for j in range(its):
        Z[j] = M(V[j])
        w = A @ Z[j]
        h = V[:j + 1] @ w
        w -= h @ V[:j + 1]
        H[:j + 1, j] = h
        H[j + 1, j] = np.linalg.norm(w)
        if H[j + 1, j] < 1e-14 * beta:
            k = j + 1
            break
        V[j + 1] = w / H[j + 1, j]
    e = np.zeros(k + 1); e[0] = beta
    y = np.linalg.lstsq(H[:k + 1, :k], e, rcond=None)[0]
    return y @ Z[:k]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "global4"
    amp = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    c, L, o, x, val, F, A = setup(name, amp)
    N = c.nrows
    b = -F
    t = time.time()
    dy = Dyn(c, o, A, val)
    S, ci, cj, pin = schur_parts(dy, c)
    Sp = pinned_matrix(S, pin)
    print(f"{name}: ncol={S.shape[0]} nnz(S)={S.nnz} pins={pin.sum()} ({time.time()-t:.1f}s)", flush=True)
    Sd = abs(Sp.diagonal())
    offs = np.asarray(abs(Sp).sum(axis=1)).ravel() - Sd
    print(f"  diag dominance: min d/off={np.min(Sd/np.maximum(offs,1e-300)):.3f} "
          f"median={np.median(Sd/np.maximum(offs,1e-300)):.3f}; "
          f"asym |S-S^T|/|S| = {spla.norm(Sp-Sp.T)/spla.norm(Sp):.3f}")
    lu = spla.splu(Sp.tocsc())
    free = ~pin

    def exact(rhs):
        rr = rhs.copy(); rr[pin] = 0
        return lu.solve(rr)

    rng = np.random.default_rng(3)
    bt = rng.standard_normal(S.shape[0]); bt[pin] = 0
    xt = exact(bt)

    Att = None
    iT = dy.iT
    Atd = A.tocsr()[iT][:, dy.iD]
    Atk = A.tocsr()[iT][:, dy.iK]
    Add = A.tocsr()[dy.iD][:, dy.iD]
    luT = spla.splu(A.tocsr()[iT][:, iT].tocsc())

    def outer(schur_solve, npass=4, omega=0.95):
        dy.Spinv["Z"] = None

        def dsolve(rd):
            nU, nW = len(dy.iU), len(dy.iW)
            ru, rw, rp = rd[:nU], rd[nU:nU + nW], rd[nU + nW:]
            ptil = np.zeros(len(dy.iP))
            ptil[dy.pfree] = dy.Awp_lu.solve(rw)
            us = dy.Dinv @ (ru - dy.Aup @ ptil)
            pbar = schur_solve(dy.Mz2 @ (dy.Apu @ us - rp))
            u = us - dy.Dinv @ (dy.Aup @ (dy.E @ pbar))
            p = ptil + dy.E @ pbar
            w = dy.Apw_lu.solve((rp - dy.Apu @ u)[dy.ptop_rows])
            return np.concatenate([u, w, p])

        def M(r):
            z = np.zeros(N)
            z[dy.iK] = r[dy.iK]
            rd = r[dy.iD] - dy.Adk @ z[dy.iK]
            zd = dsolve(rd)
            for _ in range(npass - 1):
                zd = zd + omega * dsolve(rd - Add @ zd)
            z[dy.iD] = zd
            rt = r[iT] - Atk @ z[dy.iK] - Atd @ zd
            z[iT] = luT.solve(rt)
            return z
        t = time.time()
        its, rr = gmres(A, b, M)
        return its, rr, time.time() - t

    its, rr, tt = outer(exact)
    print(f"  exact Schur: outer its={its} rel={rr:.2e} ({tt:.0f}s)", flush=True)
    variants = [
        dict(smoother="gs", nu=1), dict(smoother="gs", nu=2), dict(smoother="jacobi", nu=2, omega=0.7),
        dict(smoother="gs", nu=1, cycle="W"), dict(smoother="gs", nu=2, cycle="W"),
    ]
    for kw in variants:
        mg = AggMG(Sp, ci, cj, c.n, c.periodic, **kw)
        sizes = [lv["A"].shape[0] for lv in mg.levels]
        # standalone convergence
        res = []
        xx = np.zeros_like(bt)
        for k in range(10):
            xx = xx + mg.cyc(0, bt - Sp @ xx)
            res.append(np.linalg.norm(xx - xt) / np.linalg.norm(xt))
        rate = (res[-1] / res[2]) ** (1 / 7)
        print(f"  MG {kw} levels={sizes}: err after 1,2,5,10 cycles "
              f"{res[0]:.2e} {res[1]:.2e} {res[4]:.2e} {res[9]:.2e} rate {rate:.3f}", flush=True)
        for nin in (2, 4, 8):
            def ss(rhs, mg=mg, nin=nin):
                rr_ = rhs.copy(); rr_[pin] = 0
                return inner_gmres(Sp, rr_, lambda v: mg.cyc(0, v), nin)
            e = np.linalg.norm(ss(bt) - xt) / np.linalg.norm(xt)
            its, rr, tt = outer(ss)
            print(f"     MG-GMRES({nin}) err {e:.2e}: outer its={its} rel={rr:.2e} ({tt:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
