"""Continue a global ocean on the GPU from rest in Combined Forcing with the reference's
run/ocean settings (continuation_params.xml: ds0 1e-3, Newton tolerance 1e-2; solver
FGMRES tolerance 1e-4) and store the branch states (development tool: generates the
benchmark's near-solution state, see bench.py --state branch).

usage: python scripts/branch_state.py <preset> <destination> <out.npz> [max_steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
from iemic import config as cf  # noqa: E402
from iemic.continuation import Continuation  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402

RUN_OCEAN = {                       # run/ocean/continuation_params.xml
    "continuation parameter": "Combined Forcing", "initial step size": 1.0e-3,
    "minimum step size": 1.0e-8, "maximum step size": 1.0, "Newton tolerance": 1.0e-2,
    "destination tolerance": 1.0e-4, "epsilon increment": 1.0e-5, "normalize strategy": "N",
    "corrector residual test": "D", "state tangent scaling": 1.0,
    "enable Newton Chord hybrid solve": False, "predictor bound": 3000.0,
    "post processing": "never"}


class Logged(Ocean):
    def solve(self, b):
        t = time.time()
        x = super().solve(b)
        s = self.last_solve
        print(f"      solve: {s.iters} its, rel {s.explicit_rel_res:.2e}, conv {s.converged}, "
              f"{time.time() - t:.2f}s", flush=True)
        return x


def main():
    name, dest, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    maxs = int(sys.argv[4]) if len(sys.argv) > 4 else 60
    c = cf.preset(name, mixing=1)
    c.start_params["Combined Forcing"] = 0.0
    oc = Logged(c, solver_params={"FGMRES tolerance": 1e-4, "FGMRES iterations": 250,
                                  "FGMRES restarts": 4})
    p = dict(RUN_OCEAN)
    p["destination 0"] = dest
    p["maximum number of steps"] = maxs
    cont = Continuation(oc, p)
    states, pars = [], []
    orig_step = cont.step

    def step():
        t = time.time()
        rc = orig_step()
        print(f"step {len(cont.history)}: rc {rc} par {oc.getPar('Combined Forcing'):.5f} "
              f"ds {cont.ds:.3e} newton {cont.newtonIter} |F| {np.linalg.norm(oc.getRHS('V')):.3e} "
              f"({time.time() - t:.1f}s)", flush=True)
        if rc == 0:
            states.append(oc.getState("C").astype(np.float64))
            pars.append(oc.getPar("Combined Forcing"))
            np.savez_compressed(out, x=states[-1].astype(np.float32), par=pars[-1], n=len(pars),
                                ds=cont.ds)
        return rc
    cont.step = step
    rc = cont.run()
    print("run rc", rc, "par", oc.getPar("Combined Forcing"), flush=True)


if __name__ == "__main__":
    main()
