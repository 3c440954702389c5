"""FGMRES steps and communication of the bench's Newton step when the grid is split into
N subdomains (in-process group on one GPU; "N" = the Decomp2D rule, "N:npx" = npx x parts,
"N:1" latitude bands) at the bench's branch state (STATE=synthetic: the synthetic state):
the step count and the exchange batches / all-reduces per FGMRES step are what the
multi-GPU bench pays per rank.
usage: python scripts/band_iters.py ['{"solver param": value}'] [1,2:1,4,8:1,8]"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
import numpy as np  # noqa: E402

from iemic import _lib, config as cf  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402


def run(nranks, npx, c, L0, x):
    group = _lib.lib().iemic_local_group_new(nranks) if nranks > 1 else None
    out = [None] * nranks

    def work(r):
        kw = dict(local_group=group, rank=r, nranks=nranks, npx=npx) if nranks > 1 else {}
        sp = {"FGMRES iterations": 100, "FGMRES restarts": 20}
        sp.update(EXTRA)
        oc = Ocean(c, landm=L0, solver_params=sp, **kw)
        oc.setState(x)
        st = np.zeros(4, dtype=np.int64)
        _lib.lib().iemic_comm_stats(oc._h, _lib.ptr(st, _lib.C.c_int64))
        info = oc.newtonStep()
        _lib.lib().iemic_comm_stats(oc._h, _lib.ptr(st, _lib.C.c_int64))
        lay = oc.layout()
        it = max(1, info.solve.iters)
        out[r] = dict(iters=info.solve.iters, converged=info.solve.converged, norm_f1=info.norm_f1,
                      grid=f"{lay['npx']}x{lay['npy']}", batches_per_iter=round(st[0] / it, 1),
                      kbytes_per_iter=round(st[2] / it / 1e3, 1), allreduce_per_iter=round(st[3] / it, 1))
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
    ns = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2:1", "4:1", "4", "8:1", "8"]
    name = os.environ.get("CONFIG", "global2")
    c = cf.preset(name, mixing=1 if name.startswith("global") else 0)
    L0 = cf.init_landmask(c, cf.landmask(c))
    fix = os.path.join(ROOT, "bench_data", f"{name}_cf05.npz")
    if os.path.exists(fix) and os.environ.get("STATE", "branch") == "branch":
        with np.load(fix, allow_pickle=False) as d:
            x = d["x"].astype(np.float64)
    else:
        x = cf.synthetic_state(c, L0, amp_ts=1e-3)
    for spec in ns:
        n, npx = (int(spec.split(":")[0]), int(spec.split(":")[1])) if ":" in spec else (int(spec), 0)
        print(spec, run(n, npx, c, L0, x), flush=True)


if __name__ == "__main__":
    main()
