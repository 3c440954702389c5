"""Diagnostics of the coupled solve (GPU): ocean-only and atmosphere-only preconditioned
iterations on the coupled4 Jacobian."""
import sys
import numpy as np
import scipy.sparse.linalg as sla
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "i-emic_amd")
from test_gpu_coupled import setup
from oracle import atmos_oracle as ao
from iemic import config as cf
from iemic.coupled import Atmosphere, CoupledModel

c, g, L, oc = setup("coupled4")
atm = Atmosphere(oc, {**ao.COUPLED_RUN_PARAMS, "Combined Forcing": c.start_params["Combined Forcing"]})
cm = CoupledModel(oc, atm, {"FGMRES iterations": 150, "FGMRES restarts": 2})
x = cf.synthetic_state(c, cf.landmask(c), amp_ts=1e-3)
oc.setState(x); atm.setState(g["xa"])
cm.computeJacobian()
F = cm.computeRHS()
Fo, Fa = F[:oc.N], F[oc.N:]
oc.solver_params.update({"FGMRES iterations": 300, "FGMRES restarts": 2})
dxo = oc.solve(-Fo)
print("ocean-only iters", oc.last_solve.iters, oc.last_solve.explicit_rel_res, flush=True)
n = atm.dim
A = sla.LinearOperator((n, n), matvec=atm.applyMatrix)
M = sla.LinearOperator((n, n), matvec=atm.applyPrecon)
its = []
z, info = sla.gmres(A, -Fa, M=M, rtol=1e-10, restart=200, maxiter=5, callback=lambda r: its.append(r),
                    callback_type="pr_norm")
print("atmos-only gmres iters", len(its), "info", info,
      "res", np.linalg.norm(atm.applyMatrix(z) + Fa) / np.linalg.norm(Fa), flush=True)
r = np.random.default_rng(1).standard_normal(n)
zz = atm.applyPrecon(r)
e = atm.applyMatrix(zz) - r
print("atmos prec one-shot residual", np.linalg.norm(e) / np.linalg.norm(r), flush=True)
for rr in (1, 2, n - 1):
    print("  row", rr, e[rr], flush=True)
cm.solver_params.update({"FGMRES iterations": 250, "FGMRES restarts": 0})
dx = cm.solve(-F)
print("coupled iters", cm.last_solve.iters, cm.last_solve.explicit_rel_res, flush=True)
