"""What a NaN state does to the device path (global4): NaN count in J, the preconditioner
set-up's return, the solve's info (the NaN reaches the solver through the integral-condition
correction computeRHS forms from the state; the presets' J does not depend on it).  usage: python scripts/nan_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "i-emic_amd")]
import numpy as np  # noqa: E402

from iemic import config as cf  # noqa: E402
from iemic.ocean import Ocean  # noqa: E402
from iemic._lib import IemicError  # noqa: E402


def main():
    c = cf.preset("global4")
    L = cf.init_landmask(c, cf.landmask(c))
    oc = Ocean(c, landm=L, analyze_jacobian=os.environ.get("AJ", "1") == "1", solver_params={"Preconditioner": 2})
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    b = cf.synthetic_vector(c, seed=5)
    oc.setState(x)
    oc.computeRHS()
    oc.computeJacobian()
    oc.solve(b)
    s0 = oc.last_solve
    print("before: iters", s0.iters, "converged", s0.converged, "explicit", s0.explicit_rel_res, flush=True)
    xn = x.copy()
    xn[::7] = np.nan
    oc.setState(xn)
    F = oc.computeRHS()
    print("F nan", int(np.isnan(F).sum()), "of", F.size, flush=True)
    oc.computeJacobian()
    _, _, val = oc.exportCSR()
    print("J nan", int(np.isnan(val).sum()), "of", val.size, flush=True)
    b = cf.synthetic_vector(c, seed=5)
    try:
        sol = oc.solve(b)
        s = oc.last_solve
        print("solve returned: iters", s.iters, "converged", s.converged, "explicit", s.explicit_rel_res,
              "sol nan", int(np.isnan(sol).sum()), flush=True)
    except IemicError as e:
        print("solve raised:", e, flush=True)
    oc.setState(x)
    oc.computeRHS()                      # the integral-condition correction from the state
    oc.computeJacobian()
    sol = oc.solve(b)
    s1 = oc.last_solve
    print("after: iters", s1.iters, "converged", s1.converged, "explicit", s1.explicit_rel_res,
          "finite", bool(np.all(np.isfinite(sol))), flush=True)


if __name__ == "__main__":
    main()
