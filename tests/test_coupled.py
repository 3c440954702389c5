"""Coupled ocean + atmosphere (BASELINE config C4).

* The ocean side in coupled mode ("Coupled Temperature" = 1, run/coupled/ocean_params.xml)
  against the reference's own THCM Fortran with the atmosphere fields inserted through
  Ocean::synchronize(atmos)'s calls (tests/golden/make_golden_coupled.py): Jacobian and
  residual bitwise, getdeps constants bitwise -- on the CPU emulation of the device
  assembly here, on the device in the -m gpu tests below.
* The atmosphere restatement (oracle/atmos_oracle.py): analytic Jacobian against finite
  differences of its residual (the reference's test_atmos.C / NumericalJacobian check),
  and its coupling block d F_atm / d SST against finite differences.
* The coupled operator and solve on the device against the oracle.
"""
import json
import math
import os

import numpy as np
import pytest
import scipy.sparse as sp

from helpers import GOLDEN, Emul, emul_get_deps, emul_set_atmosphere, golden
from iemic import config as cf
from oracle import atmos_oracle as ao


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def coupled_manifest():
    with open(os.path.join(GOLDEN, "manifest_coupled.json")) as f:
        return json.load(f)


def landm_of(name):
    c = cf.preset(name)
    return golden(name)["landm_local"].astype(np.int32).reshape(c.l + 2, c.m + 2, c.n + 2)


def atm_args(g):
    return g["atm_t"], g["atm_q"], g["atm_a"], g["atm_pars"]


def fortran_placed(oracle_lib, rowptr, col, g, kind):
    return oracle_lib.fortran_to_graph(rowptr, col, g[f"{kind}_beg"], g[f"{kind}_jco"],
                                       g[f"{kind}_co"], -1)


@pytest.mark.parametrize("name", ["coupled_natl8", "coupled_natl8s"])
@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_emulated_coupled_ocean_bitexact(oracle_lib, emul, name, kind):
    """coupled_natl8 (coupled T) and coupled_natl8s (coupled T and S): the device assembly
    code (CPU emulation) == reference Fortran, bitwise."""
    c = cf.preset(name)
    g = golden(name)
    e = Emul(c, landm_of(name))
    emul_set_atmosphere(e, *atm_args(g), p=g["atm_p"])
    np.testing.assert_array_equal(bits(emul_get_deps(e)), bits(g["deps"]))
    x = g[f"{kind}_x"]
    rowptr, col, val, B = e.jacobian_csr(x)
    ref = fortran_placed(oracle_lib, rowptr, col, g, kind)
    np.testing.assert_array_equal(val, ref)
    F = e.rhs(x)
    np.testing.assert_array_equal(bits(F), bits(-g[f"{kind}_B"]))


def test_emulated_coupled4_hashes(emul):
    """coupled4 (the C4 ocean, 96x38x12): residual and getdeps bitwise vs the Fortran."""
    import hashlib
    name = "coupled4"
    c = cf.preset(name)
    g = golden(name)
    man = coupled_manifest()[name]
    e = Emul(c, landm_of(name))
    emul_set_atmosphere(e, *atm_args(g))
    np.testing.assert_array_equal(bits(emul_get_deps(e)), bits(g["deps"]))
    L = cf.landmask(c)
    x = cf.synthetic_state(c, L)
    assert hashlib.sha256(x.tobytes()).hexdigest() == man["states"]["synthetic"]["x_sha"]
    F = e.rhs(x)
    B = -F
    assert hashlib.sha256(B.tobytes()).hexdigest() == man["states"]["synthetic"]["B_sha"]


def test_atmos_oracle_fd_jacobian():
    """AtmosLocal/Atmosphere restatement: J == FD of F (test_atmos.C's numerical Jacobian
    check), on a small periodic grid with land, albedo forcing switched on."""
    rng = np.random.default_rng(3)
    n, m = 8, 6
    surf = (rng.random((m, n)) < 0.3).astype(int)
    p = dict(ao.COUPLED_RUN_PARAMS)
    p["Albedo Forcing"] = 1.0
    p["Combined Forcing"] = 0.7
    for periodic in (True, False):
        at = ao.AtmosOracle(n, m, 0, 359.99, -85.5, 85.5, periodic, surf, Ooa=5.4, Os=120.0,
                            params=p)
        x = 0.1 * rng.standard_normal(at.dim)
        x[2:3 * n * m:3] = 0.3 + 0.1 * rng.standard_normal(n * m)
        sst = 0.1 * rng.standard_normal(n * m)
        J = at.jacobian(x).toarray()
        Jfd = ao.fd_jacobian(lambda y: at.rhs(y, sst), x, 1e-6)
        assert np.abs(J - Jfd).max() <= 1e-9 * np.abs(J).max()
        l = 3
        C = at.block_from_ocean(l).toarray()
        idx = [6 * (((l - 1) * m + j) * n + i) + 4 for j in range(m) for i in range(n)]
        Cfd = ao.fd_jacobian(lambda s: at.rhs(x, s), sst, 1e-6)
        assert np.abs(C[:, idx] - Cfd).max() <= 1e-7 * max(1.0, np.abs(C).max())
        # the block is zero outside the surface temperature columns
        mask = np.ones(C.shape[1], bool)
        mask[idx] = False
        assert not np.any(C[:, mask])


@pytest.mark.parametrize("name", ["coupled_natl8", "coupled_natl8s"])
def test_ocean_block_matches_fortran_fd(oracle_lib, name):
    """Ocean::getBlock(atmos) (Ocean.C:1538-1667) == the derivative of the reference
    Fortran's residual w.r.t. the inserted atmosphere T, q, albedo (and, with coupled S,
    P) fields (forcing.F90:75-94, 162-182 are linear in them: a unit perturbation gives
    the entry up to rounding)."""
    if not oracle_lib.reference_available():
        pytest.skip("reference Fortran library not built (this container only)")
    c = cf.preset(name)
    g = golden(name)
    L = cf.landmask(c)
    t, q, a, pars = atm_args(g)
    xa = g["xa"]
    at = ao.AtmosOracle(c.n, c.m, c.xmin, c.xmax, c.ymin, c.ymax, c.periodic,
                        (landm_of(name)[c.l, 1:c.m + 1, 1:c.n + 1] != 0).astype(int),
                        Ooa=g["deps"][0], Os=g["deps"][1],
                        params={**ao.COUPLED_RUN_PARAMS,
                                "Combined Forcing": c.start_params["Combined Forcing"]})
    at.suno_ocean = np.array(at.suno[1:])
    Cb = at.block_to_ocean(c.l, at.surf, g["deps"], c.start_params["Combined Forcing"],
                           c.start_params["Solar Forcing"], coupled_s=bool(c.coupled_s)).toarray()
    x = g["synthetic_x"]
    p0 = g["atm_p"]
    runs = {}
    h = 1.0
    sel = [(3, 2), (5, 4)]          # a few surface points (i, j), 0-based
    for (i, j) in sel:
        for fld in ("t", "q", "a"):
            f2 = dict(t=t.copy(), q=q.copy(), a=a.copy(), p=p0.copy(), pars=pars)
            f2[fld][j * c.n + i] += h
            runs[(i, j, fld)] = f2
    if c.coupled_s:
        # the P anomaly column: the dimensional field moves by Pdist * eta qdim per unit
        f2 = dict(t=t, q=q, a=a, p=p0 + at.pdist * at.P.eta * at.P.qdim, pars=pars)
        runs[(0, 0, "P")] = f2
    keys = list(runs)
    base = oracle_lib.run_reference(c.ref_dict(), L, c.par_list(), [x], use_landm=False,
                                    atmos=dict(t=t, q=q, a=a, p=p0, pars=pars))
    for k in keys:
        r = oracle_lib.run_reference(c.ref_dict(), L, c.par_list(), [x], use_landm=False,
                                     atmos=runs[k])
        dF = (-r["B0"]) - (-base["B0"])
        i, j, fld = k
        if fld == "P":
            col = at.rowP                   # the perturbation above is one unit of P
        else:
            col = at.row(i, j, {"t": ao.TT, "q": ao.QQ, "a": ao.AA}[fld])
        np.testing.assert_allclose(dF, Cb[:, col], rtol=1e-6, atol=1e-9 * np.abs(Cb).max())


@pytest.mark.parametrize("name", ["coupled_natl8", "coupled_natl8s"])
@pytest.mark.parametrize("kind", ["zero", "synthetic"])
def test_oracle_coupled_ocean_bitexact(oracle_lib, name, kind):
    """The oracle's C restatement in coupled mode (usrc.F90:724-766 lin, forcing.F90:75-94 /
    162-182, set_atmos_parameters) against the reference Fortran: J and F bitwise -- the
    checker behind the coupled CPU baseline."""
    c = cf.preset(name)
    g = golden(name)
    o = oracle_lib.Oracle(c.ref_dict(), landm_of(name), c.par_list())
    o.set_atmos(g["atm_t"], g["atm_q"], g["atm_a"], g["atm_pars"], p=g["atm_p"])
    x = g[f"{kind}_x"]
    val, _ = o.jacobian(x)
    ref = fortran_placed(oracle_lib, o.rowptr, o.col, g, kind)
    np.testing.assert_array_equal(val, ref)
    np.testing.assert_array_equal(bits(o.rhs(x)), bits(-g[f"{kind}_B"]))


def test_atmos_coefficients_hand_derived():
    """The atmosphere restatement's coefficients against numbers written out here straight
    from the reference's formulas (AtmosLocal::setup, AtmosLocal.C:174-245; discretize
    1141-1234; computeJacobian 585-700), independently of oracle/atmos_oracle.py's code:
    the setup() scalars with run/coupled's parameter values, and the T / q rows of one
    interior ocean cell and one interior land cell (no boundaries() change there)."""
    p = dict(ao.COUPLED_RUN_PARAMS)
    p["Combined Forcing"] = 0.7
    P = ao.AtmosParams(p, Ooa=5.4, Os=120.0)
    # setup(): rhoa 1.25, ch 0.94*1.3e-3, cpa 1000, uw 8.5, A 216, B 1.5, t0a 15, hdima 8400,
    # D0 3.4e6, r0 6.37e6, udim 0.1, sun0 1360, c0 0.43, rhoo 1024, ce 1.3e-3, hdimq 1800,
    # kappa 3.1e6, q0 8e-3, qdim 1e-3, t0o 15, t0i -5, lv 2.5e6
    muoa = 1.25 * (0.94 * 1.3e-3) * 1000.0 * 8.5
    eta = (1.25 / 1024.0) * 1.3e-3 * 8.5
    qso = 3.8e-3 * math.exp(17.67 * 15.0 / (15.0 + 243.5))
    qsi = 3.8e-3 * math.exp(21.87 * -5.0 / (-5.0 + 265.5))
    hand = {
        "muoa": muoa,
        "amua": (216.0 + 1.5 * 15.0) / muoa,
        "bmua": 1.5 / muoa,
        "Ai": 1.25 * 8400.0 * 1000.0 * 0.1 / (6.37e6 * muoa),
        "Ad": 1.25 * 8400.0 * 1000.0 * 3.4e6 / (muoa * 6.37e6 * 6.37e6),
        "As": 1360.0 * (1 - 0.43) / (4 * muoa),
        "eta": eta,
        "nuq": 0.7 * 1.0 * (eta / 1800.0) * (1024.0 / 1.25) * (6.37e6 / 0.1),
        "Phv": 3.1e6 / (0.1 * 6.37e6),
        "Eo0": eta * (qso - 8e-3),
        "Cs": (eta * (qsi - 8e-3) - eta * (qso - 8e-3)) / eta / 1e-3,
        "dqso": 5e-4,
        "dqsi": 3.8e-3 * 21.87 * 265.5 / (-5.0 + 265.5) ** 2 * math.exp(21.87 * -5.0 / (-5.0 + 265.5)),
        "lvscale": 1024.0 * 2.5e6 / muoa,
        "tauf": 10.0 * 3600.0 * 24.0 * 0.1 / 6.37e6,
    }
    for k, v in hand.items():
        assert abs(getattr(P, k) - v) <= 1e-14 * abs(v), (k, getattr(P, k), v)

    n, m = 8, 6
    surf = np.zeros((m, n), int)
    surf[2, 5] = 1                                       # one land cell
    at = ao.AtmosOracle(n, m, 0, 359.99, -85.5, 85.5, True, surf, Ooa=5.4, Os=120.0, params=p)
    x = np.zeros(at.dim)
    x[2:3 * n * m:3] = 0.3
    J = at.jacobian(x).toarray()
    deg = math.pi / 180.0
    dx, dy = 359.99 * deg / n, 171.0 * deg / m
    j = 3                                                # 1-based interior latitude, row index 2
    yc = -85.5 * deg + (j - 0.5) * dy
    yvm, yvp = -85.5 * deg + (j - 1) * dy, -85.5 * deg + j * dy
    dat = lambda y: 0.9 + 1.5 * math.exp(-12 * y * y / math.pi)   # noqa: E731 (datc / datv)
    cx = 1.0 / (math.cos(yc) * dx) ** 2
    q4 = math.cos(yvm) / math.cos(yc) / dy ** 2
    q6 = math.cos(yvp) / math.cos(yc) / dy ** 2
    t4, t6 = dat(yvm) * q4, dat(yvp) * q6
    for i, land in ((2, False), (5, True)):              # 0-based longitude of the cell
        rT, rq = at.row(i, j - 1, ao.TT), at.row(i, j - 1, ao.QQ)
        tc = 0.0 if land else 1.0                        # discretize(1): no land points
        # Al(TT,TT) = tdif Ad (txx + tyy) - tc - bmua tc2, centre and east neighbour
        Tc = hand["Ad"] * (-2 * dat(yc) * cx - (t4 + t6)) - tc - hand["bmua"] * 1.0
        assert abs(J[rT, rT] - Tc) <= 1e-13 * abs(Tc), (i, J[rT, rT], Tc)
        rTe = at.row((i + 1) % n, j - 1, ao.TT)
        assert abs(J[rT, rTe] - hand["Ad"] * dat(yc) * cx) <= 1e-13 * hand["Ad"] * dat(yc) * cx
        # Al(QQ,QQ) = Phv (qxx + qyy) - nuq qc
        Qc = hand["Phv"] * (-2 * cx - (q4 + q6)) - hand["nuq"] * tc
        assert abs(J[rq, rq] - Qc) <= 1e-13 * abs(Qc), (i, J[rq, rq], Qc)
        rqn = at.row(i, j, ao.QQ)
        assert abs(J[rq, rqn] - hand["Phv"] * q6) <= 1e-13 * hand["Phv"] * q6
