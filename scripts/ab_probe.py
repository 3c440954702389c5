"""A/B kernel measurement on one box: the 2-degree bench state with one build of the device
library (IEMIC_LIB, scripts/ab_build.sh): preconditioner apply, its parts, SpMV and a full
Newton step, GPU-timed; run once per variant (the library is loaded once per process).

usage: IEMIC_LIB=libiemic_amd_<v>.so python scripts/ab_probe.py <v> [newton steps (0: none)]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]

import numpy as np  # noqa: E402


def main():
    import torch
    from iemic import _lib
    from iemic import config as cf
    from iemic.ocean import Ocean
    name = sys.argv[1] if len(sys.argv) > 1 else "base"
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = cf.preset("global2", mixing=1)
    with np.load(os.path.join(ROOT, "bench_data", "global2_cf05.npz"), allow_pickle=False) as d:
        x = d["x"].astype(np.float64)
    oc = Ocean(cfg, device=0, solver_params={"FGMRES iterations": 90, "FGMRES restarts": 20})
    oc.setState(x)
    oc.computeJacobian()
    out = {"variant": name, "lib": os.path.basename(_lib.LIB_PATH)}
    ms, _ = oc.time_prec(100)
    out["apply_us"] = round(ms * 1e3, 2)
    if hasattr(_lib.lib(), "iemic_time_prec_parts"):
        out.update({k: round(v, 2) for k, v in oc.time_prec_parts(100).items()})
    out["spmv_us"] = round(oc.time_spmv(50) * 1e3, 2)
    if nsteps == 0:                      # apply and SpMV timings only
        print(json.dumps(out), flush=True)
        return
    x0 = torch.from_numpy(x).cuda()
    L_ = _lib.lib()
    times, iters, prec, f1, sp = [], [], [], None, []
    for q in range(nsteps + 1):
        _lib.check(L_.iemic_set_state_dev(oc._h, x0.data_ptr()), "set_state_dev")
        torch.cuda.synchronize()
        t = time.perf_counter()
        info = oc.newtonStep()
        torch.cuda.synchronize()
        if q:
            times.append((time.perf_counter() - t) * 1e3)
            iters.append(info.solve.iters)
            prec.append(info.t_prec_ms)
            if info.solve.n_spmv:
                sp.append(info.solve.t_spmv_ms * 1e3 / info.solve.n_spmv)
            f1 = info.norm_f1
    out["newton_ms"] = round(float(np.median(times)), 2)
    out["newton_ms_all"] = [round(t, 2) for t in times]
    out["fgmres_iters"] = iters
    out["prec_setup_ms"] = round(float(np.median(prec)), 3)
    out["norm_f1"] = repr(f1)
    out["spmv_insolve_us"] = round(float(np.median(sp)), 2) if sp else None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
