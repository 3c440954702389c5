"""Continue the coupled ocean + atmosphere model (config C4) on the GPU from rest in
Combined Forcing with the reference's run/coupled continuation settings
(continuation_params.xml: ds0 1e-2, Newton tolerance 1e-4, destination tolerance 1e-7;
CoupledModel's FGMRES from run/coupled/solver_params.xml) and store the branch state of
both models (development tool: the coupled benchmark's near-solution state,
bench.py --config coupled4).

usage: python scripts/coupled_branch_state.py <destination> <out.npz> [max_steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
from iemic import config as cf  # noqa: E402
from iemic.continuation import Continuation  # noqa: E402
from iemic.coupled import RUN_COUPLED_ATMOS, Atmosphere, CoupledModel  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402

RUN_COUPLED = {                     # run/coupled/continuation_params.xml
    "continuation parameter": "Combined Forcing", "initial step size": 1.0e-2,
    "minimum step size": 1.0e-12, "maximum step size": 1.0e3, "Newton tolerance": 1.0e-4,
    "destination tolerance": 1.0e-7, "post processing": "never"}


def main():
    dest, out = float(sys.argv[1]), sys.argv[2]
    maxs = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    cfg = cf.preset("coupled4")
    oc = Ocean(cfg)
    atm = Atmosphere(oc, {**RUN_COUPLED_ATMOS, "Combined Forcing": 0.0})
    cm = CoupledModel(oc, atm, {"FGMRES tolerance": 1e-8, "FGMRES iterations": 150,
                                "FGMRES restarts": 6})
    cm.setState(np.zeros(cm.N))
    cm.setPar("Combined Forcing", 0.0)
    p = dict(RUN_COUPLED)
    p["destination 0"] = dest
    p["maximum number of steps"] = maxs
    cont = Continuation(cm, p)
    orig_step = cont.step

    def step():
        t = time.time()
        rc = orig_step()
        print(f"step {len(cont.history)}: rc {rc} par {cm.getPar('Combined Forcing'):.5f} "
              f"ds {cont.ds:.3e} newton {cont.newtonIter} ({time.time() - t:.1f}s)", flush=True)
        if rc == 0:
            np.savez_compressed(out, x=oc.getState("C"), xa=atm.getState(),
                                par=cm.getPar("Combined Forcing"))
        return rc
    cont.step = step
    rc = cont.run()
    print("run rc", rc, "par", cm.getPar("Combined Forcing"), flush=True)


if __name__ == "__main__":
    main()
