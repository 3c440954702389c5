"""Diagnostic: band operators (in-process group on one GPU) driven by a numpy FGMRES."""
import os
import sys
import threading
import queue

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd"), os.path.join(ROOT, "tests")]
from iemic import _lib, config as cf  # noqa
from iemic.ocean import Ocean  # noqa
from oracle import oracle as orc  # noqa
from helpers import golden_landm, mask_fix  # noqa

name, P, prec = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
c = cf.preset(name, mixing=0)
L0 = golden_landm(name)
L = mask_fix(orc, c, L0)
o = orc.Oracle(c.ref_dict(), L, c.par_list())
x = cf.synthetic_state(c, L, amp_ts=1e-3)
ov, _ = o.jacobian(x)
b = -o.rhs(x)
group = _lib.lib().iemic_local_group_new(P)
cmds = [queue.Queue() for _ in range(P)]
outs = [queue.Queue() for _ in range(P)]
rowsets = [None] * P


def work(r):
    oc = Ocean(c, landm=L0, local_group=group, rank=r, nranks=P,
               solver_params={"Preconditioner": prec, "FGMRES tolerance": 1e-10,
                              "FGMRES iterations": 300, "FGMRES restarts": 0})
    oc.setState(x)
    oc.computeJacobian()
    lay = oc.layout()
    rowsets[r] = np.array([6 * ((k * c.m + j) * c.n + i) + q for k in range(c.l)
                           for j in range(lay["jb0"], lay["jb1"]) for i in range(c.n) for q in range(6)])
    if prec:
        oc.buildPreconditioner()
    while True:
        cmd, v = cmds[r].get()
        if cmd == "quit":
            break
        if cmd == "A":
            outs[r].put(oc.applyMatrix(v).copy())
        elif cmd == "M":
            outs[r].put(oc.applyPrecon(v).copy() if prec else v.copy())
        elif cmd == "S":
            s = oc.solve(v).copy()
            inf = oc.last_solve
            outs[r].put((s, inf.iters, inf.implicit_rel_res, inf.explicit_rel_res))
    oc.close()


th = [threading.Thread(target=work, args=(r,)) for r in range(P)]
for t in th:
    t.start()


def op(cmd, v):
    for r in range(P):
        cmds[r].put((cmd, v))
    res = [outs[r].get() for r in range(P)]
    if cmd == "S":
        out = np.zeros(c.nrows)
        for r in range(P):
            out[rowsets[r]] = res[r][0][rowsets[r]]
        return out, [q[1:] for q in res]
    out = np.zeros(c.nrows)
    for r in range(P):
        out[rowsets[r]] = res[r][rowsets[r]]
    return out


v = cf.synthetic_vector(c)
print("spmv err", np.abs(op("A", v) - o.spmv(ov, v)).max())
z1 = op("M", v); z2 = op("M", 2 * v); z3 = op("M", v)
print("prec determinism", np.abs(z1 - z3).max(), "linearity", np.abs(z2 - 2 * z1).max(), "|z|", np.abs(z1).max(),
      "nan", np.isnan(z1).sum())
# numpy FGMRES with band operators
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prec_study import gmres  # noqa
import scipy.sparse as sp
A = sp.csr_matrix((ov, o.col, o.rowptr), shape=(c.nrows, c.nrows))
its, rr = gmres(A, b, lambda r: op("M", r), tol=1e-10, m=300)
print("numpy fgmres with band prec:", its, rr)
s, infos = op("S", b)
print("library solve infos (iters, implicit, explicit):", infos)
print("library solve true rel res:", np.linalg.norm(b - A @ s) / np.linalg.norm(b))
for r in range(P):
    cmds[r].put(("quit", None))
for t in th:
    t.join()
