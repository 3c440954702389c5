"""SpMV probe for the PMC passes: builds the 2-degree Jacobian on the GPU and launches
k_spmv `reps` times, each after an Infinity Cache flush (the in-solve, cold-cache
condition), timed with HIP events on the library stream.  Run under rocprofv3 --pmc
(scripts/gpu_pmc.sh); tools/pmc_report.py turns the counters into bytes per launch.

usage: python scripts/spmv_probe.py [config] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]


def main():
    import torch
    from iemic import config as cf
    from iemic.ocean import Ocean
    name = sys.argv[1] if len(sys.argv) > 1 else "global2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = cf.preset(name, mixing=0)
    oc = Ocean(cfg, device=0)
    L = oc.landmask().reshape(cfg.l + 2, cfg.m + 2, cfg.n + 2)
    oc.setState(cf.synthetic_state(cfg, L, amp_ts=1e-3))
    oc.computeJacobian()
    fl = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    ms = oc.time_spmv_cold(fl.data_ptr(), fl.numel(), reps)
    print(json.dumps({"config": name, "reps": reps, "cold_us": round(ms * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
