"""Generate the golden fixtures of the THCM hot path from the reference itself.

Runs the reference's own THCM Fortran (compiled from /root/reference/src/ocean/thcm by
oracle/ref/Makefile into oracle/_ref/libthcm_ref.so; this container only) through
init_ -> setparcs -> matrix_ / rhs_ (THCM.C:178-798, 949-1192) and stores, per
configuration and state:

* the local land mask after ``init_`` (global.F90 topofit/readmask + usrc.F90:83-107),
* the intcond coefficients (thcm_utils.F90:285-312), par(1..30) after ``stpnt``/setparcs,
* the Fortran CSR (beg/jco/co, 1-based, fillcolA order), diagonal coB and rhs B.

Small configurations keep the full arrays; larger ones keep SHA-256 digests of the
exact float64 bytes plus norms, which pins bit-exactness without megabytes of data.

The states are the zero state, the benchmark's seeded synthetic state
(iemic.config.synthetic_state) and, on 16x16x16, the state stored in the reference's
own fixture test/ocean/ocean_reference.h5 (/State/Values, contiguous float64 at byte
offset 2144, 24576 values) -- decoded as raw data, no HDF5 library.

Usage (this container only):  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "i-emic_amd"))

from iemic import config as cf  # noqa: E402
from oracle import oracle as orc  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
H5 = "/root/reference/test/ocean/ocean_reference.h5"

FULL = ["test6x6x4", "natl8", "2dmoc"]
HASHED = ["2dmoc_run", "gateway16", "global4"]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def h5_state() -> np.ndarray:
    with open(H5, "rb") as f:
        f.seek(2144)
        return np.frombuffer(f.read(24576 * 8), dtype="<f8").copy()


def main() -> None:
    orc.build(ref=True)
    if not orc.reference_available():
        raise SystemExit("reference library missing")
    manifest = {}
    for name in FULL + HASHED:
        c = cf.preset(name, mixing=0)
        L = cf.landmask(c)
        states = {"zero": np.zeros(c.nrows), "synthetic": cf.synthetic_state(c, L)}
        if name == "gateway16":
            states["h5"] = h5_state()
        keys = list(states)
        r = orc.run_reference(c.ref_dict(), L, c.par_list(), [states[k] for k in keys],
                              use_landm=False, timeout=1800)
        entry = {"n": c.n, "m": c.m, "l": c.l, "nrows": c.nrows, "states": {},
                 "landm_sha": sha(r["landm_local"].astype(np.int32)),
                 "par": [float(v) for v in r["par"]]}
        arrays = {"landm_local": r["landm_local"].astype(np.int8),
                  "intcond_val": r["intcond_val"], "intcond_ind": r["intcond_ind"]}
        for s, k in enumerate(keys):
            x = states[k]
            st = {"x_sha": sha(x)}
            for f in ("beg", "jco", "co", "coB", "B"):
                a = r[f"{f}{s}"]
                st[f + "_sha"] = sha(a)
                if a.dtype.kind == "f":
                    st[f + "_norm"] = float(np.linalg.norm(a))
            st["nnz"] = int(len(r[f"co{s}"]))
            entry["states"][k] = st
            if name in FULL or k == "h5":
                for f in ("beg", "jco", "co", "coB", "B"):
                    arrays[f"{k}_{f}"] = r[f"{f}{s}"]
                arrays[f"{k}_x"] = x
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrays)
        manifest[name] = entry
        print(name, "done", {k: v["nnz"] for k, v in entry["states"].items()}, flush=True)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
