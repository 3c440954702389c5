"""FGMRES steps of the bench's Newton step when the grid is split into N latitude bands
(in-process group on one GPU) at the bench's branch state (STATE=synthetic: the synthetic
state): the step count is what the multi-GPU bench pays per band.
usage: python scripts/band_iters.py ['{"solver param": value}'] [1,2,4,8]"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
import numpy as np  # noqa: E402

from iemic import _lib, config as cf  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402


def run(nranks, c, L0, x):
    group = _lib.lib().iemic_local_group_new(nranks) if nranks > 1 else None
    out = [None] * nranks

    def work(r):
        kw = dict(local_group=group, rank=r, nranks=nranks) if nranks > 1 else {}
        sp = {"FGMRES iterations": 100, "FGMRES restarts": 20}
        sp.update(EXTRA)
        oc = Ocean(c, landm=L0, solver_params=sp, **kw)
        oc.setState(x)
        info = oc.newtonStep()
        out[r] = (info.solve.iters, info.solve.converged, info.norm_f1)
        oc.close()

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if group:
        _lib.lib().iemic_local_group_free(group)
    return out[0]


EXTRA = {}


def main():
    import json
    if len(sys.argv) > 1:
        EXTRA.update(json.loads(sys.argv[1]))
    ns = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8]
    c = cf.preset("global2", mixing=1)
    L0 = cf.init_landmask(c, cf.landmask(c))
    fix = os.path.join(ROOT, "bench_data", "global2_cf05.npz")
    if os.path.exists(fix) and os.environ.get("STATE", "branch") == "branch":
        with np.load(fix, allow_pickle=False) as d:
            x = d["x"].astype(np.float64)
    else:
        x = cf.synthetic_state(c, L0, amp_ts=1e-3)
    for n in ns:
        print(n, run(n, c, L0, x), flush=True)


if __name__ == "__main__":
    main()
