"""Golden fixtures of the THCM hot path WITH vertical mixing (Mixing = 1 / 2), from the
reference itself (this container only; see make_golden.py for the mechanism).

The reference THCM Fortran (oracle/_ref/libthcm_ref.so, compiled from
/root/reference/src/ocean) runs init_ -> setparcs -> matrix_ (lin, nlin_jac, vmix_jac by
coloured forward differences, boundaries, fillcolA) / rhs_ (incl. vmix_fun) on each
state; the Fortran CSR (beg/jco/co), coB and rhs B are stored in full for the small
grids and as SHA-256 digests (+ norms) for the larger ones.  States: the seeded
synthetic state (T, S ~ U(+-0.1): about half of the vertical faces statically unstable,
so the convective mixing is active) and, on gateway16, the reference's own fixture state
test/ocean/ocean_reference.h5.  Mixing = 2 (gateway16) fixes the T/S mixing flags at the
first evaluation (mix_imp.f vmix_control); every state here has nonzero T and S.

Usage (this container only):  python tests/golden/make_golden_mix.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import OUT, h5_state, sha  # noqa: E402
from make_golden import cf, orc  # noqa: E402

MIX = {"test6x6x4": 1, "natl8": 1, "gateway16": 2, "global4": 1}
FULL = ["test6x6x4", "natl8"]


def main() -> None:
    orc.build(ref=True)
    if not orc.reference_available():
        raise SystemExit("reference library missing")
    manifest = {}
    for name, mix in MIX.items():
        c = cf.preset(name, mixing=mix)
        L = cf.landmask(c)
        states = {"synthetic": cf.synthetic_state(c, L)}
        if name == "gateway16":
            states["h5"] = h5_state()
        entry = {"mixing": mix, "n": c.n, "m": c.m, "l": c.l, "states": {}}
        arrays = {}
        for k, x in states.items():
            # one reference process per state: Mixing = 2 decides at the first evaluation
            r = orc.run_reference(c.ref_dict(), L, c.par_list(), [x], use_landm=False, timeout=3000)
            st = {"x_sha": sha(x), "nnz": int(len(r["co0"]))}
            for f in ("beg", "jco", "co", "coB", "B"):
                a = r[f"{f}0"]
                st[f + "_sha"] = sha(a)
                if a.dtype.kind == "f":
                    st[f + "_norm"] = float(np.linalg.norm(a))
                if name in FULL:
                    arrays[f"{k}_{f}"] = a
            entry["states"][k] = st
            entry["par"] = [float(v) for v in r["par"]]
            entry["landm_sha"] = sha(r["landm_local"].astype(np.int32))
            print(name, k, "nnz", st["nnz"], flush=True)
        if arrays:
            np.savez_compressed(os.path.join(OUT, f"mix_{name}.npz"), **arrays)
        manifest[name] = entry
    with open(os.path.join(OUT, "manifest_mix.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
