"""Golden fixtures of the coupled ocean (config C4) from the reference.

Runs the reference's own THCM Fortran with "Coupled Temperature" = 1 (coupled_T, THCM.C:232;
run/coupled/ocean_params.xml), inserts atmosphere fields through the calls
Ocean::synchronize(atmos) makes (Ocean.C:1443-1472: insert_atmosphere_t/q/a/p,
inserts.F90:12-100, then set_atmos_parameters, usrc.F90:237-293, with the
AtmosLocal::CommPars of the atmosphere restatement oracle/atmos_oracle.py), and stores the
Fortran Jacobian and right-hand side (matrix_/rhs_, usrc.F90:432-586) plus getdeps
(usrc.F90:201-219: Ooa, Os, nus, eta, lvsc, qdim, pQSnd).

coupled_natl8 (and coupled_natl8s, with "Coupled Salinity" = 1 too) keep full arrays; coupled4 (96x38x12, the C4 ocean) keeps SHA-256 digests.
The atmosphere state and fields are regenerated from the seeds below by the tests.

Usage (this container only):  python tests/golden/make_golden_coupled.py
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
from oracle import atmos_oracle as ao  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
NAMES = ["coupled_natl8", "coupled_natl8s", "coupled4"]
SEED_ATM = 20261017


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def surface_mask(landm_local: np.ndarray, c) -> np.ndarray:
    """Ocean landm(0:n+1,0:m+1,0:l+1) -> atmosphere surface mask (j, i) at k = l
    (Ocean::getLandMask global_surface -> AtmosLocal::setSurfaceMask 1722-1756)."""
    L = landm_local.reshape(c.l + 2, c.m + 2, c.n + 2)
    return (L[c.l, 1:c.m + 1, 1:c.n + 1] != 0).astype(np.int32)


def atmos_params(c) -> dict:
    p = dict(ao.COUPLED_RUN_PARAMS)
    p["Combined Forcing"] = c.start_params["Combined Forcing"]
    return p


def atmos_state(at: ao.AtmosOracle, seed: int = SEED_ATM) -> np.ndarray:
    """A non-trivial atmosphere state: the idealized profile (AtmosLocal::idealized
    423-456) plus seeded perturbations."""
    rng = np.random.default_rng(seed)
    n, m = at.n, at.m
    x = np.zeros(at.dim)
    ymin, ymax = at.yc[0] + 0.5 * at.dy, at.yv[m]
    for j in range(m):
        v = np.cos(np.pi * (at.yc[j + 1] - ymin) / (ymax - ymin))
        for i in range(n):
            x[at.row(i, j, ao.TT)] = v + 0.1 * rng.uniform(-1, 1)
            x[at.row(i, j, ao.QQ)] = v * at.P.tdim * at.P.dqso / at.P.qdim + 0.1 * rng.uniform(-1, 1)
            x[at.row(i, j, ao.AA)] = at.P.a0 + 0.05 * rng.uniform(-1, 1)
    x[at.rowP] = 0.3
    return x


def make_atmos(c, landm_local, deps):
    at = ao.AtmosOracle(c.n, c.m, c.xmin, c.xmax, c.ymin, c.ymax, c.periodic,
                        surface_mask(landm_local, c), Ooa=float(deps[0]), Os=float(deps[1]),
                        params=atmos_params(c))
    xa = atmos_state(at)
    return at, xa


def atmos_fields(at: ao.AtmosOracle, xa: np.ndarray) -> dict:
    """Atmosphere::interfaceT/Q/A/P (449-493) as n*m surface vectors; P dimensional
    (getP 1160-1225)."""
    nm = at.n * at.m
    P = at.P
    p = np.where(at.surf.reshape(-1) == 0, at.pdist * (P.Eo0 + P.eta * P.qdim * xa[at.rowP]), 0.0)
    return dict(t=xa[0:3 * nm:3].copy(), q=xa[1:3 * nm:3].copy(), a=xa[2:3 * nm:3].copy(), p=p,
                pars=P.commpars())


def main() -> None:
    orc.build(ref=True)
    manifest = {}
    for name in NAMES:
        c = cf.preset(name)
        L = cf.landmask(c)
        r0 = orc.run_reference(c.ref_dict(), L, c.par_list(), [], use_landm=False, timeout=1800)
        at, xa = make_atmos(c, r0["landm_local"], r0["deps"])
        atm = atmos_fields(at, xa)
        states = {"zero": np.zeros(c.nrows), "synthetic": cf.synthetic_state(c, L)}
        keys = list(states)
        r = orc.run_reference(c.ref_dict(), L, c.par_list(), [states[k] for k in keys],
                              use_landm=False, timeout=1800, atmos=atm)
        entry = {"n": c.n, "m": c.m, "l": c.l, "deps": [float(v) for v in r["deps"]],
                 "deps_uncoupled": [float(v) for v in r0["deps"]],
                 "par": [float(v) for v in r["par"]], "states": {}}
        arrays = {"landm_local": r["landm_local"].astype(np.int8), "xa": xa,
                  "deps": r["deps"], **{"atm_" + k: v for k, v in atm.items()}}
        for s, k in enumerate(keys):
            st = {"x_sha": sha(states[k])}
            for f in ("beg", "jco", "co", "coB", "B"):
                a = r[f"{f}{s}"]
                st[f + "_sha"] = sha(a)
                if a.dtype.kind == "f":
                    st[f + "_norm"] = float(np.linalg.norm(a))
            entry["states"][k] = st
            if name.startswith("coupled_natl8"):
                for f in ("beg", "jco", "co", "coB", "B"):
                    arrays[f"{k}_{f}"] = r[f"{f}{s}"]
                arrays[f"{k}_x"] = states[k]
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrays)
        manifest[name] = entry
        print(name, "done", entry["deps"], flush=True)
    with open(os.path.join(OUT, "manifest_coupled.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
