"""Preconditioner sweep on the CPU twin (oracle/prec_oracle.c, test infrastructure): FGMRES
steps of one Newton step from a bench state for block GS variants, to find which block's
inner solve limits the outer iteration (mesh robustness).
usage: python tests/prec_sweep_cpu.py <config> '<json list of {dyn_iters, dyn_omega, ts_mg}>'"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from iemic import config as cf  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from helpers import mask_fix  # noqa: E402


def main():
    name = sys.argv[1]
    variants = json.loads(sys.argv[2])
    c = cf.preset(name, mixing=1)
    L0 = cf.init_landmask(c, cf.landmask(c))
    L = mask_fix(orc, c, L0)
    o = orc.Oracle(c.ref_dict(), L, c.par_list())
    with np.load(os.path.join(ROOT, "bench_data", f"{name}_cf05.npz"), allow_pickle=False) as d:
        x = d["x"].astype(np.float64)
    F = o.rhs(x)
    val, _ = o.jacobian(x)
    for v in variants:
        t = time.perf_counter()
        P = orc.BlockGS(o, val, 12, dyn_iters=v.get("dyn_iters", 4), dyn_omega=v.get("dyn_omega", 0.95),
                        ts_mg=v.get("ts_mg", 1), dyn_krylov=v.get("dyn_krylov", 0),
                        schur_passes=v.get("schur_passes", 0), schur_mask=v.get("schur_mask", 0))
        dx, its, rel, _ = P.fgmres(np.ascontiguousarray(-F), tol=1e-8, m=90, maxit=90 * 21)
        print(json.dumps({"config": name, **v, "fgmres_steps": its, "rel": rel,
                          "s": round(time.perf_counter() - t, 1)}), flush=True)
        del P


if __name__ == "__main__":
    main()
