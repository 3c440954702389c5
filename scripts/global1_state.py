"""The 1-degree near-solution state (development tool and config C5's set-up): prolong the
2-degree branch state (bench_data/global2_cf05.npz, Combined Forcing 0.5) to the 1-degree
grid (iemic.config.prolong_state) and run Newton corrector steps at Combined Forcing 0.5
on the GPU until ||F|| stops dropping; prints the residual sequence.

usage: python scripts/global1_state.py [newton_steps] [fgmres_tol] [out.npz]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
from iemic import config as cf  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402


def near_solution(oc, cfg, steps: int, log=print, ts_only: bool = False):
    """prolonged 2-degree branch state (ts_only: T and S only, u, v, w, p = 0) -> Newton at
    the config's Combined Forcing; returns the list of (||F0||, ||F1||, FGMRES its)"""
    c2 = cf.preset("global2", mixing=1)
    with np.load(os.path.join(ROOT, "bench_data", "global2_cf05.npz"), allow_pickle=False) as d:
        x2 = d["x"].astype(np.float64)
    L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
    x = cf.prolong_state(c2, x2, cfg, L)
    if ts_only:
        x.reshape(-1, 6)[:, :4] = 0.0
    oc.setState(x)
    seq = []
    for it in range(steps):
        t = time.time()
        info = oc.newtonStep(allow_unconverged=True)
        seq.append((info.norm_f0, info.norm_f1, info.solve.iters))
        log(f"newton {it}: |F| {info.norm_f0:.4e} -> {info.norm_f1:.4e}, {info.solve.iters} its "
            f"(conv {info.solve.converged}, rel {info.solve.explicit_rel_res:.1e}), {time.time() - t:.1f}s")
        if info.norm_f1 > info.norm_f0:
            break
    return seq


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    tol = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-8
    cfg = cf.preset("global1", mixing=1)
    oc = Ocean(cfg, solver_params={"FGMRES tolerance": tol, "FGMRES iterations": 90, "FGMRES restarts": 20})
    near_solution(oc, cfg, steps, log=lambda s: print(s, flush=True),
                  ts_only=os.environ.get("TS_ONLY", "0") == "1")
    if len(sys.argv) > 3:
        np.savez_compressed(sys.argv[3], x=oc.getState().astype(np.float32), par=0.5)


if __name__ == "__main__":
    main()
