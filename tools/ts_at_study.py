"""FGMRES iterations of the CPU block GS (oracle/prec_oracle.c) against the dynamics pass
after which the T/S right-hand side is formed (ts_at): with ts_at < dyn_iters the T/S
multigrid V-cycle no longer depends on the last passes and can run beside them on a second
stream.  One Newton-step linear system at the benchmark's branch state.

usage: python tools/ts_at_study.py [config] [ts_at ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]


def main():
    from iemic import config as cf
    from oracle import oracle as orc
    name = sys.argv[1] if len(sys.argv) > 1 else "global4"
    ats = [int(a) for a in sys.argv[2:]] or [0, 3, 2, 1]
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import mask_fix
    cfg = cf.preset(name, mixing=1)
    L = mask_fix(orc, cfg, cf.landmask(cfg))
    fix = os.path.join(ROOT, "bench_data", f"{name}_cf05.npz")
    if os.path.exists(fix):
        with np.load(fix, allow_pickle=False) as d:
            x = d["x"].astype(np.float64)
    else:
        x = cf.synthetic_state(cfg, L, amp_ts=1e-3)
    o = orc.Oracle(cfg.ref_dict(), L, cfg.par_list())
    F = o.rhs(x)
    val, _ = o.jacobian(x)
    for a in ats:
        P = orc.BlockGS(o, val, 12, dyn_iters=4, dyn_omega=0.95, ts_mg=1, ts_at=a)
        t = time.perf_counter()
        _, its, rel, _ = P.fgmres(np.ascontiguousarray(-F), tol=1e-8, m=100, maxit=2100)
        print(f"{name} ts_at={a}: {its} iterations, rel {rel:.2e}, {time.perf_counter() - t:.1f} s", flush=True)


if __name__ == "__main__":
    main()
