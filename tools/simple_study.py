"""SIMPLE-type dynamics solve variants (CPU/scipy prototype of the block-GS preconditioner's
U/V/W/P part).  Development tool: measures outer FGMRES iterations for A_uu approximations.

usage: python tools/simple_study.py [global4] [amp_ts]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prec_study import gmres, orc, setup  # noqa: E402


class Dyn:
    def __init__(self, c, o, A, val):
        self.c, self.o = c, o
        N = c.nrows
        n, m, l = c.n, c.m, c.l
        A = A.tocsr()
        self.A = A
        d = A.diagonal()
        rowabs = np.asarray(abs(A).sum(axis=1)).ravel()
        known = (d == 1.0) & (rowabs == 1.0)
        if o.rowintcon >= 0:
            known[o.rowintcon] = False
        self.known = known
        var = np.arange(N) % 6
        cell = np.arange(N) // 6
        self.iK = np.flatnonzero(known)
        self.iU = np.flatnonzero(~known & (var <= 1))
        self.iW = np.flatnonzero(~known & (var == 2))
        self.iP = np.flatnonzero(~known & (var == 3))
        self.iT = np.flatnonzero(~known & (var >= 4))
        self.iD = np.concatenate([self.iU, self.iW, self.iP])
        sub = lambda r, cc: A[r][:, cc].tocsr()
        self.Auu = sub(self.iU, self.iU)
        self.Auw = sub(self.iU, self.iW)
        self.Aup = sub(self.iU, self.iP)
        self.Awp = sub(self.iW, self.iP)
        self.Apu = sub(self.iP, self.iU)
        self.Apw = sub(self.iP, self.iW)
        self.Adk = sub(self.iD, self.iK)
        self.Atk = sub(self.iT, self.iK)
        self.Atd = sub(self.iT, self.iD)
        # 2x2 point blocks of A_uu (U,V of the same cell)
        cu = cell[self.iU]
        same = (cu[self.Auu.tocoo().row] == cu[self.Auu.tocoo().col])
        co = self.Auu.tocoo()
        Dm = sp.csr_matrix((co.data[same], (co.row[same], co.col[same])), shape=self.Auu.shape)
        self.Dinv = sp.csr_matrix(spla.inv(Dm.tocsc()))
        # colours (i+j+k) parity
        ci = cu % n; cj = (cu // n) % m; ck = cu // (n * m)
        par = (ci + cj + ck) % 2
        if c.periodic and n % 2:
            par = par + 2 * (ci == n - 1)
        self.colours = [np.flatnonzero(par == q) for q in range(par.max() + 1)]
        self.uu_lu = None
        # columns: P cells grouped by (i,j)
        cp = cell[self.iP]
        ij = cp % (n * m)
        cols, colidx = np.unique(ij, return_inverse=True)
        self.ncol = len(cols)
        E = sp.csr_matrix((np.ones(len(cp)), (np.arange(len(cp)), colidx)), shape=(len(cp), self.ncol))
        # depth weights: 1 / A_pw[k, W(k)] (or -1/A_pw[k, W(k-1)])
        wcell = {cc: q for q, cc in enumerate(cell[self.iW])}
        pw = np.zeros(len(cp))
        Apw = self.Apw.tolil()
        for q, cc in enumerate(cp):
            row = dict(zip(Apw.rows[q], Apw.data[q]))
            if cc in wcell and row.get(wcell[cc], 0.0) != 0.0:
                pw[q] = 1.0 / row[wcell[cc]]
            elif (cc - n * m) in wcell and row.get(wcell[cc - n * m], 0.0) != 0.0:
                pw[q] = -1.0 / row[wcell[cc - n * m]]
        self.E = E
        self.Mz2 = (E.T @ sp.diags(pw)).tocsr()
        self.Spinv = {"D": self.schur_pinv(self.Dinv)}
        # SIMPLEC-style lumped 2x2 blocks: row sums of the U-U, U-V, V-U, V-V couplings
        vu = (np.arange(N) % 6)[self.iU]
        cu_row = cu[co.row]
        key_r = vu[co.row]; key_c = vu[co.col]
        # map each entry to the 2x2 block of its row cell
        pos = {cc: q for q, cc in enumerate(cu)}  # last index per cell (U or V)
        lr, lc_, lv = [], [], []
        uidx = {}
        for q, (cc, vv) in enumerate(zip(cu, vu)):
            uidx[(cc, vv)] = q
        for r_, c_, v_ in zip(co.row, co.col, co.data):
            tgt = uidx.get((cu[r_], vu[c_]))
            if tgt is None:
                continue
            lr.append(r_); lc_.append(tgt); lv.append(v_)
        Dl = sp.csr_matrix((lv, (lr, lc_)), shape=self.Auu.shape)
        self.Dlinv = sp.csr_matrix(spla.inv(Dl.tocsc()))
        self.Spinv["L"] = self.schur_pinv(self.Dlinv)
        # ptil: pin the top P cell of each column
        kp = cp // (n * m)
        top = np.zeros(len(cp), bool)
        for q in range(self.ncol):
            pass
        order = np.lexsort((-kp, colidx))
        first = np.r_[True, colidx[order][1:] != colidx[order][:-1]]
        top[order[first]] = True
        self.pfree = np.flatnonzero(~top)
        self.Awp_lu = spla.splu(self.Awp[:, self.pfree].tocsc())
        # w: drop the top P row of each column
        self.Apw_lu = spla.splu(self.Apw[np.flatnonzero(~top)].tocsc())
        self.ptop_rows = np.flatnonzero(~top)

    def schur_pinv(self, Xinv):
        S = (self.Mz2 @ self.Apu @ Xinv @ self.Aup @ self.E)
        S = S.toarray() if sp.issparse(S) else S
        return np.linalg.pinv(S, rcond=1e-12)

    def exact_schur(self):
        lu = spla.splu(self.Auu.tocsc())
        X = lu.solve((self.Aup @ self.E).toarray())
        S = self.Mz2 @ self.Apu @ X
        self.Spinv["X"] = np.linalg.pinv(S, rcond=1e-12)

    def uu_solve(self, rhs, mode, k=0, u0=None):
        if mode == "D":
            return self.Dinv @ rhs
        if mode == "exact":
            if self.uu_lu is None:
                self.uu_lu = spla.splu(self.Auu.tocsc())
            return self.uu_lu.solve(rhs)
        # symmetric 2x2-block coloured GS, k sweeps from u0 (default D^-1 rhs)
        u = self.Dinv @ rhs if u0 is None else u0.copy()
        seq = list(range(len(self.colours))) + list(range(len(self.colours)))[::-1]
        for _ in range(k):
            for q in seq:
                C = self.colours[q]
                res = rhs - self.Auu @ u
                u[C] += (self.Dinv[C][:, C] @ res[C])
        return u

    def solve(self, rd, mode, k=0, schur="D"):
        nU, nW = len(self.iU), len(self.iW)
        ru, rw, rp = rd[:nU], rd[nU:nU + nW], rd[nU + nW:]
        ptil = np.zeros(len(self.iP))
        ptil[self.pfree] = self.Awp_lu.solve(rw)
        us = self.uu_solve(ru - self.Aup @ ptil, mode, k)
        pbar = self.Spinv[schur] @ (self.Mz2 @ (self.Apu @ us - rp))
        u = us - self.uu_solve(self.Aup @ (self.E @ pbar), mode, k)
        p = ptil + self.E @ pbar
        w = self.Apw_lu.solve((rp - self.Apu @ u)[self.ptop_rows])
        return np.concatenate([u, w, p])


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "global4"
    amp = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    c, L, o, x, val, F, A = setup(name, amp)
    N = c.nrows
    b = -F
    dy = Dyn(c, o, A, val)
    print(f"ncol={dy.ncol} |U|={len(dy.iU)} colours={len(dy.colours)}")
    P = orc.BlockGS(o, val, 12)

    def make(mode, k, schur="D"):
        def M(r):
            z = np.zeros(N)
            z[dy.iK] = r[dy.iK]
            rd = r[dy.iD] - dy.Adk @ z[dy.iK]
            zd = dy.solve(rd, mode, k, schur)
            z[dy.iD] = zd
            rt = r[dy.iT] - dy.Atk @ z[dy.iK] - dy.Atd @ zd
            rr = np.zeros(N)
            rr[dy.iT] = rt
            z[dy.iT] = P.apply(rr)[dy.iT]
            return z
        return M

    dy.exact_schur()
    for schur in ("X", "L"):
        for mode, k in (("exact", 0), ("D", 0), ("gs", 2), ("gs", 4)):
            its, rr = gmres(A, b, make(mode, k, schur))
            print(f"schur={schur} uu={mode} k={k}: outer its={its} rel={rr:.2e}", flush=True)


if __name__ == "__main__":
    main()
