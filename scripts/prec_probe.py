"""Preconditioner apply timing at the benchmark state: GPU ms and host enqueue ms per apply
(iemic_time_prec), for the solver-parameter variants given as KEY=VALUE,... arguments.

usage: python scripts/prec_probe.py [config] ["TS after dyn pass=2" ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]


def main():
    from iemic import config as cf
    from iemic.ocean import Ocean
    name = sys.argv[1] if len(sys.argv) > 1 else "global2"
    variants = sys.argv[2:] or [""]
    cfg = cf.preset(name, mixing=1)
    fix = os.path.join(ROOT, "bench_data", f"{name}_cf05.npz")
    for v in variants:
        sp = {"Preconditioner": 2}
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=")
            sp[k.strip()] = type(Ocean.default_solver_params()[k.strip()])(val) if hasattr(Ocean, "default_solver_params") else int(val)
        oc = Ocean(cfg, device=0, solver_params=sp)
        L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
        if os.path.exists(fix):
            with np.load(fix, allow_pickle=False) as d:
                x = d["x"].astype(np.float64)
        else:
            x = cf.synthetic_state(cfg, L, amp_ts=1e-3)
        oc.setState(x)
        oc.computeJacobian()
        ms, hms = oc.time_prec(50)
        parts = {k: round(u, 2) for k, u in oc.time_prec_parts(50).items()}
        print(json.dumps({"config": name, "variant": v, "gpu_us": round(ms * 1e3, 1),
                          "host_us": round(hms * 1e3, 1), **parts}), flush=True)
        del oc


if __name__ == "__main__":
    main()
