"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the I-EMIC atmosphere model and of the
ocean <-> atmosphere coupling blocks (the checker of the coupled model).

Restated from (read as text; the reference C++ needs Trilinos and cannot be built here):

* ``AtmosLocal`` (src/atmosphere/AtmosLocal.C): parameters 106-171, coefficients 174-377,
  integral coefficients 560-582, Jacobian 585-746 (atoms ``discretize`` 1141-1234,
  ``boundaries`` 1429-1479, ``assemble`` 1238-1310), right-hand side 782-849, ``forcing``
  871-984, albedo switch ``aF`` 1118-1138, ``fillPdist`` 495-516.
* ``Atmosphere`` (src/atmosphere/Atmosphere.C), the one-process case of the parallel
  wrapper the coupled model uses (aux = 1, integral condition on q): ``setPdist``
  1234-1265, ``computeRHS`` 266-393 (q integral row, precipitation row), ``computeJacobian``
  911-1126 (dense integral rows), mass matrix 1277-1331, ``getBlock(ocean)`` 502-613.
* ``Ocean::getBlock(atmos)`` (src/ocean/Ocean.C:1538-1667) for coupled_T = 1,
  coupled_S = 0 (run/coupled/ocean_params.xml), no sea ice (Msi = 0).

Row order is the reference's: atmosphere row = 3*(j*n + i) + xx (xx = T, q, A), the
global precipitation P last (FIND_ROW_ATMOS0, AtmosphereDefinitions.H:45-54); ocean row
= 6*((k*m + j)*n + i) + var (FIND_ROW2).  Per-latitude tables use Python's ``math``
(the C library's sin/cos/exp, as the reference); per-cell arithmetic keeps the
reference's evaluation order, so the device restatement can be compared bitwise.

Parity status: the reference atmosphere cannot run here (Trilinos absent),
so this restatement is pinned by (1) its own analytic Jacobian against central finite
differences of its residual (the reference's test_atmos.C strategy) and (2) the ocean
side of every coupling entry against the reference Fortran (tests/test_coupled.py).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp

PI = 3.14159265358979323846
TT, QQ, AA = 0, 1, 2
NUN = 3

# run/coupled/atmosphere_params.xml over the AtmosLocal::setParameters defaults
COUPLED_RUN_PARAMS = {
    "restoring timescale tauf (in days)": 10.0,
    "restoring timescale tauc (in days)": 1.0,
    "radiative flux param A": 216.0,
    "radiative flux param B": 1.5,
    "background temperature seaice": -5.0,
    "atmos reference humidity": 8e-3,
    "atmos humidity scale": 1e-3,
    "temperature eddy diffusivity": 3.4e6,
    "humidity eddy diffusivity": 3.1e6,
    "reference albedo": 0.3,
    "albedo excursion": 0.4,
    "melt temperature threshold (deg C)": 0.0,
    "melt threshold width (deg C)": 5.0,
    "accumulation precipitation threshold (m/y)": -100.0,
    "accumulation threshold width (m/y)": 5.0,
    "rain/snow temperature threshold (deg C)": 150.0,
    "rain/snow threshold width (deg C)": 5.0,
    "Combined Forcing": 1.0, "Solar Forcing": 1.0, "Humidity Forcing": 1.0,
    "Latent Heat Forcing": 1.0, "Albedo Forcing": 0.0,
}


def _sq(v):
    """pow(v, 2) of the reference C++: GCC and clang emit v*v for it"""
    return v * v


def _get(p, k, d):
    return float(p.get(k, d))


class AtmosParams:
    """AtmosLocal::setParameters (AtmosLocal.C:106-171) + setup() coefficients (174-245)."""

    def __init__(self, p: dict, Ooa: float, Os: float):
        self.rhoa = _get(p, "atmospheric density", 1.25)
        self.rhoo = _get(p, "oceanic density", 1024)
        self.hdima = _get(p, "atmospheric scale height", 8400.)
        self.hdimq = _get(p, "humidity scale height", 1800.)
        self.hdim = _get(p, "vertical length scale", 4000.)
        self.cpa = _get(p, "heat capacity", 1000.)
        self.D0 = _get(p, "temperature eddy diffusivity", 3.1e+06)
        self.kappa = _get(p, "humidity eddy diffusivity", 1e+06)
        self.arad = _get(p, "radiative flux param A", 212.0)
        self.brad = _get(p, "radiative flux param B", 1.5)
        self.sun0 = _get(p, "solar constant", 1360.)
        self.c0 = _get(p, "atmospheric absorption coefficient", 0.43)
        self.ce = _get(p, "Dalton number", 1.3e-03)
        self.ch = _get(p, "exchange coefficient ch", 0.94 * self.ce)
        self.uw = _get(p, "mean atmospheric surface wind speed", 8.5)
        self.t0a = _get(p, "background temperature atmosphere", 15.0)
        self.t0o = _get(p, "background temperature ocean", 15.0)
        self.t0i = _get(p, "background temperature seaice", -5.0)
        self.tdim = _get(p, "temperature scale", 1.0)
        self.q0 = _get(p, "atmos reference humidity", 2e-3)
        self.qdim = _get(p, "atmos humidity scale", 1e-3)
        self.lv = _get(p, "latent heat of vaporization", 2.5e06)
        self.udim = _get(p, "horizontal velocity of the ocean", 0.1e+00)
        self.r0dim = _get(p, "radius of the earth", 6.37e+06)
        self.a0 = _get(p, "reference albedo", 0.3)
        self.da = _get(p, "albedo excursion", 0.5)
        tauf = _get(p, "restoring timescale tauf (in days)", 1.0)
        tauc = _get(p, "restoring timescale tauc (in days)", 1.0)
        self.tauf = (tauf * 3600. * 24. * self.udim) / self.r0dim
        self.tauc = (tauc * 3600. * 24. * self.udim) / self.r0dim
        self.Tm = _get(p, "melt temperature threshold (deg C)", 0.0)
        self.Tr = _get(p, "rain/snow temperature threshold (deg C)", 1.0)
        self.Pa = _get(p, "accumulation precipitation threshold (m/y)", 0.2)
        self.epm = _get(p, "melt threshold width (deg C)", 5.0)
        self.epr = _get(p, "rain/snow threshold width (deg C)", 1.0)
        self.epa = _get(p, "accumulation threshold width (m/y)", 0.1)
        self.comb = _get(p, "Combined Forcing", 0.0)
        self.sunp = _get(p, "Solar Forcing", 1.0)
        self.lonf = _get(p, "Longwave Forcing", 1.0)
        self.humf = _get(p, "Humidity Forcing", 1.0)
        self.latf = _get(p, "Latent Heat Forcing", 1.0)
        self.albf = _get(p, "Albedo Forcing", 1.0)
        self.tdif = _get(p, "T Eddy Diffusivity", 1.0)
        # setup()
        self.muoa = self.rhoa * self.ch * self.cpa * self.uw
        self.amua = (self.arad + self.brad * self.t0a) / self.muoa
        self.bmua = self.brad / self.muoa
        self.Ai = self.rhoa * self.hdima * self.cpa * self.udim / (self.r0dim * self.muoa)
        self.Ad = self.rhoa * self.hdima * self.cpa * self.D0 / (self.muoa * self.r0dim * self.r0dim)
        self.As = self.sun0 * (1 - self.c0) / (4 * self.muoa)
        self.eta = (self.rhoa / self.rhoo) * self.ce * self.uw
        self.Phv = self.kappa / (self.udim * self.r0dim)
        c1, c2, c3, c4, c5 = 3.8e-3, 21.87, 265.5, 17.67, 243.5
        self.qso = c1 * math.exp(c4 * self.t0o / (self.t0o + c5))
        self.qsi = c1 * math.exp(c2 * self.t0i / (self.t0i + c3))
        self.Eo0 = self.eta * (self.qso - self.q0)
        self.Ei0 = self.eta * (self.qsi - self.q0)
        self.Cs = (self.Ei0 - self.Eo0) / self.eta / self.qdim
        self.Po0 = self.Eo0
        self.Tr = self.Tr - self.t0o
        self.Tm = self.Tm - self.t0o
        self.dqso = 5e-4   # AtmosLocal.C:233 ("hack")
        self.dqsi = (c1 * c2 * c3) / ((self.t0i + c3) * (self.t0i + c3))
        self.dqsi *= math.exp((c2 * self.t0i) / (self.t0i + c3))
        self.lvscale = self.rhoo * self.lv / self.muoa
        self.Ooa, self.Os = Ooa, Os
        self.set_nuq()

    def set_nuq(self):
        """AtmosLocal.C:189 / setPar 1674."""
        self.nuq = self.comb * self.humf * (self.eta / self.hdimq) * (self.rhoo / self.rhoa) * \
            (self.r0dim / self.udim)

    def commpars(self) -> np.ndarray:
        """AtmosLocal::getCommPars (AtmosLocal.C:537-557), CommPars order."""
        return np.array([self.tdim, self.qdim, self.nuq, self.eta, self.dqso, self.dqsi,
                         self.nuq * self.tdim / self.qdim * self.dqso, self.Eo0, self.Ei0,
                         self.Cs, self.t0o, self.t0i, self.a0, self.da, self.tauf, self.tauc,
                         self.comb, self.albf])


class AtmosOracle:
    """One-process restatement of Atmosphere + AtmosLocal (aux = 1, intcond on q)."""

    def __init__(self, n, m, xmin_deg, xmax_deg, ymin_deg, ymax_deg, periodic,
                 surfmask, Ooa, Os, params=None):
        self.n, self.m = n, m
        self.periodic = bool(periodic)
        self.P = AtmosParams(params or {}, Ooa, Os)
        self.surf = np.asarray(surfmask, dtype=np.int64).reshape(m, n)   # 1 = land
        self.dim = n * m * NUN + 1
        self.rowP = self.dim - 1
        self.rowint = NUN * ((m - 1) * n + (n - 1)) + QQ        # Atmosphere.C:49-51
        xmin, xmax = xmin_deg * PI / 180.0, xmax_deg * PI / 180.0
        ymin, ymax = ymin_deg * PI / 180.0, ymax_deg * PI / 180.0
        self.dx = (xmax - xmin) / n
        self.dy = (ymax - ymin) / m
        dx, dy = self.dx, self.dy
        P = self.P
        self.yc = [ymin + (j - 0.5) * dy for j in range(m + 1)]
        self.yv = [ymin + j * dy for j in range(m + 1)]
        self.datc = [0.9 + 1.5 * math.exp(-12 * y * y / PI) for y in self.yc]
        self.datv = [0.9 + 1.5 * math.exp(-12 * y * y / PI) for y in self.yv]
        self.suna = [P.As * (1 - .482 * (3 * _sq(math.sin(y)) - 1.) / 2.) for y in self.yc]
        self.suno = [P.Os * (1 - .482 * (3 * _sq(math.sin(y)) - 1.) / 2.) for y in self.yc]
        # per-latitude stencil weights (discretize, AtmosLocal.C:1162-1232), index j = 1..m
        self.cosdx2i = [0.0] + [1.0 / _sq(math.cos(self.yc[j]) * dx) for j in range(1, m + 1)]
        dy2i = 1.0 / _sq(dy)
        cy = [0.0] + [math.cos(self.yc[j]) for j in range(1, m + 1)]
        self.t4 = [0.0] + [dy2i * self.datv[j - 1] * math.cos(self.yv[j - 1]) / cy[j] for j in range(1, m + 1)]
        self.t6 = [0.0] + [dy2i * self.datv[j] * math.cos(self.yv[j]) / cy[j] for j in range(1, m + 1)]
        self.q4 = [0.0] + [dy2i * math.cos(self.yv[j - 1]) / cy[j] for j in range(1, m + 1)]
        self.q6 = [0.0] + [dy2i * math.cos(self.yv[j]) / cy[j] for j in range(1, m + 1)]
        # integral coefficients (integralCoeff 560-582 + Atmosphere::setupIntCoeff 168-242)
        area = np.array([math.cos(self.yc[j]) * dx * dy for j in range(1, m + 1)])
        self.pint = np.where(self.surf == 0, area[:, None], 0.0).reshape(-1)   # (j, i)
        self.intc = np.zeros(self.dim)
        self.intc[NUN * np.arange(n * m) + QQ] = self.pint
        total = 0.0
        for v in self.pint:          # sequential sums (the device's order)
            total += abs(float(v))
        self.total_area = total
        # Pdist (fillPdist 495-516, corrected by Atmosphere::setPdist 1234-1265)
        pd = np.zeros(n * m)
        for j in range(1, m + 1):
            y = self.yc[j]
            v = 2 * math.exp(-_sq(6 * y)) + _sq(math.sin(2.0 * y))
            for i in range(n):
                if self.surf[j - 1, i] == 0:
                    pd[(j - 1) * n + i] = v
        ipd = 0.0
        for a_, b_ in zip(self.pint, pd):
            ipd += float(a_) * float(b_)
        corr = 1 - ipd / self.total_area
        ones = (np.abs(self.pint) > 1e-7).astype(np.float64)
        self.pdist = corr * ones + pd
        self.msi = np.zeros(n * m)
        self.sit = np.zeros(n * m)

    # --- helpers ----------------------------------------------------------------
    def row(self, i, j, xx):
        return NUN * (j * self.n + i) + xx

    def _nb(self, i, j, di, dj):
        i2, j2 = i + di, j + dj
        if self.periodic:
            i2 %= self.n
        return i2, j2

    def _Tl(self, A, Ta, j):
        P = self.P
        return Ta + P.comb * P.sunp * self.suno[j] * ((1 - P.a0) - P.da * A) / P.Ooa

    def _aF(self, A, Ta, Pv, i, j):
        P = self.P
        H = lambda x, eps: (1. / 2.) * (1.0 + math.tanh(x / eps))  # noqa: E731
        dimP = 3600. * 24. * 365. * self.pdist[(j - 1) * self.n + i] * (P.Po0 + P.eta * P.qdim * Pv)
        tl = self._Tl(A, Ta, j)
        return H(P.Tm - tl, P.epm) * H(P.Tr - tl, P.epr) * H(dimP - P.Pa, P.epa)

    # --- local stencil (computeJacobian 585-746 + boundaries + assemble) ---------
    def local_entries(self, x):
        """{row: [(col, value), ...]} in the reference's CRS order (loc, then column var)."""
        n, m, P = self.n, self.m, self.P
        sT = P.tdif * P.Ad
        out = {}
        for j1 in range(1, m + 1):
            j = j1 - 1
            for i in range(n):
                land = self.surf[j, i] != 0
                sr = j * n + i
                # T-T atom per loc {2: W, 4: S, 5: C, 6: N, 8: E}
                cx, t4, t6 = self.datc[j1] * self.cosdx2i[j1], self.t4[j1], self.t6[j1]
                txx = {2: cx, 8: cx, 5: -2 * cx}
                tyy = {4: t4, 6: t6, 5: -(t4 + t6)}
                tc = 0.0 if land else 1.0
                att = {}
                for loc in (2, 4, 5, 6, 8):
                    v = sT * txx.get(loc, 0.0) + sT * tyy.get(loc, 0.0)
                    v = v + (-1.0) * (tc if loc == 5 else 0.0)
                    v = v + (-P.bmua) * (1.0 if loc == 5 else 0.0)
                    att[loc] = v
                qxv = self.cosdx2i[j1]
                qxx = {2: qxv, 8: qxv, 5: -2 * qxv}
                qyy = {4: self.q4[j1], 6: self.q6[j1], 5: -(self.q4[j1] + self.q6[j1])}
                qc = 0.0 if land else 1.0
                aqq = {}
                for loc in (2, 4, 5, 6, 8):
                    v = P.Phv * qxx.get(loc, 0.0) + P.Phv * qyy.get(loc, 0.0)
                    v = v + (-P.nuq) * (qc if loc == 5 else 0.0)
                    aqq[loc] = v
                # boundaries (1429-1479): W, E only when not periodic; then N, S
                for a in (att, aqq):
                    if i == 0 and not self.periodic:
                        a[5] = a[5] + a[2]; a[2] = 0.0
                    if i == n - 1 and not self.periodic:
                        a[5] = a[5] + a[8]; a[8] = 0.0
                    if j1 == m:
                        a[5] = a[5] + a[6]; a[6] = 0.0
                    if j1 == 1:
                        a[5] = a[5] + a[4]; a[4] = 0.0
                tt_pp = P.comb * P.latf * P.lvscale * P.eta * P.qdim * self.pdist[sr]
                dTadA = -P.comb * P.sunp * self.suna[j1] * P.da
                dTldA = -P.comb * P.sunp * self.suno[j1] * P.da / P.Ooa
                tt_aa = (dTldA + dTadA) if land else dTadA
                qq_pp = -P.nuq * self.pdist[sr]
                A = x[self.row(i, j, AA)]
                Ta = x[self.row(i, j, TT)]
                Pv = x[self.rowP]
                if land:
                    df = 1e-6
                    f0 = self._aF(A, Ta, Pv, i, j1)
                    daA = (self._aF(A + df, Ta, Pv, i, j1) - f0) / df
                    daP = (self._aF(A, Ta, Pv + df, i, j1) - f0) / df
                    daT = (self._aF(A, Ta + df, Pv, i, j1) - f0) / df
                    dAdA = (P.comb * P.albf * daA - 1) / P.tauf
                    dAdP = (P.comb * P.albf * daP) / P.tauf
                    dAdT = (P.comb * P.albf * daT) / P.tauf
                else:
                    dAdA, dAdP, dAdT = -1 / P.tauc, 0.0, 0.0
                locs = {2: (-1, 0), 4: (0, -1), 6: (0, 1), 8: (1, 0)}
                rt, rq, ra = [], [], []
                for loc in (2, 4, 5, 6, 8):
                    if loc == 5:
                        rt += [(self.row(i, j, TT), att[5]), (self.row(i, j, AA), tt_aa),
                               (self.rowP, tt_pp)]
                        rq += [(self.row(i, j, QQ), aqq[5]), (self.rowP, qq_pp)]
                        ra += [(self.row(i, j, TT), dAdT), (self.row(i, j, AA), dAdA),
                               (self.rowP, dAdP)]
                        continue
                    i2, j2 = self._nb(i, j, *locs[loc])
                    if att[loc] != 0.0:
                        rt.append((self.row(i2, j2, TT), att[loc]))
                    if aqq[loc] != 0.0:
                        rq.append((self.row(i2, j2, QQ), aqq[loc]))
                out[self.row(i, j, TT)] = [(c, v) for c, v in rt if v != 0.0]
                out[self.row(i, j, QQ)] = [(c, v) for c, v in rq if v != 0.0]
                out[self.row(i, j, AA)] = [(c, v) for c, v in ra if v != 0.0]
        return out

    def forcing(self, x, sst):
        """AtmosLocal::forcing (871-984), parallel mode (no integral-row zeroing)."""
        n, m, P = self.n, self.m, self.P
        frc = np.zeros(self.dim)
        for j1 in range(1, m + 1):
            j = j1 - 1
            for i in range(n):
                sr = j * n + i
                tr, hr, ar = self.row(i, j, TT), self.row(i, j, QQ), self.row(i, j, AA)
                A, Ta = x[ar], x[tr]
                QSW = self.suna[j1] * (1 - P.a0)
                land = self.surf[j, i] != 0
                if land:
                    v = P.comb * P.sunp * self.suno[j1] * (1 - P.a0) / P.Ooa
                    v += P.comb * (P.sunp * QSW - P.lonf * P.amua)
                else:
                    Ts = sst[sr] + self.msi[sr] * (self.sit[sr] - sst[sr] + P.t0i - P.t0o)
                    v = Ts + P.comb * (P.sunp * QSW - P.lonf * P.amua)
                    v += P.comb * P.latf * P.lvscale * self.pdist[sr] * P.Po0
                frc[tr] = v
                if land:
                    v = 0.0
                else:
                    Eo = (P.tdim / P.qdim) * P.dqso * sst[sr]
                    Ei = (P.tdim / P.qdim) * P.dqsi * self.sit[sr]
                    v = P.nuq * (Eo + self.msi[sr] * (Ei - Eo + P.Cs))
                frc[hr] = v
                if land:
                    v = (P.comb * P.albf * self._aF(A, Ta, x[self.rowP], i, j1) - A) / P.tauf
                else:
                    v = (P.comb * P.albf * self.msi[sr] - A) / P.tauc
                frc[ar] = v
        return frc

    def rhs(self, x, sst):
        """Atmosphere::computeRHS (266-393) with AtmosLocal::computeRHS (782-849)."""
        x = np.asarray(x, dtype=np.float64)
        sst = np.asarray(sst, dtype=np.float64)
        ent = self.local_entries(x)
        frc = self.forcing(x, sst)
        F = np.zeros(self.dim)
        for r in range(self.dim - 1):
            v = 0.0
            if r % NUN != AA:
                mv = 0.0
                for c, a in ent[r]:
                    mv += a * x[c]
                v += mv
            v += frc[r]
            F[r] = v
        P = self.P
        intcond = float(np.dot(self.intc, x))
        F[self.rowint] = intcond
        tmp = P.dqsi * self.sit + (-P.dqso) * sst
        sigma = P.dqso * sst + 1.0 * self.msi * tmp
        sst_int = float(np.dot(self.pint, sigma)) * (1.0 / self.total_area) * (P.tdim / P.qdim)
        q_int = intcond * 1.0 / self.total_area
        mcs_int = float(np.dot(self.pint, self.msi)) * P.Cs / self.total_area
        F[self.rowP] = -x[self.rowP] - q_int + sst_int + mcs_int
        return F

    def jacobian(self, x) -> sp.csr_matrix:
        """Atmosphere::computeJacobian (911-1126): local stencil rows, then the dense q
        integral row (rowIntCon) and the precipitation row."""
        ent = self.local_entries(np.asarray(x, dtype=np.float64))
        rows, cols, vals = [], [], []
        for r, lst in ent.items():
            if r == self.rowint:
                continue
            for c, v in lst:
                rows.append(r); cols.append(c); vals.append(v)
        qrows = NUN * np.arange(self.n * self.m) + QQ
        rows += [self.rowint] * len(qrows); cols += list(qrows); vals += list(self.intc[qrows])
        rows += [self.rowP] * len(qrows); cols += list(qrows)
        vals += list((-1.0 / self.total_area) * self.intc[qrows])
        rows.append(self.rowP); cols.append(self.rowP); vals.append(-1.0)
        J = sp.csr_matrix((vals, (rows, cols)), shape=(self.dim, self.dim))
        J.sum_duplicates()
        return J

    def mass(self):
        """Atmosphere::computeMassMat (1277-1331)."""
        B = np.zeros(self.dim)
        B[0:-1:NUN] = self.P.Ai
        B[1:-1:NUN] = 1.0
        B[2:-1:NUN] = 1.0
        B[self.rowint] = 0.0
        B[self.rowP] = 0.0
        return B

    # --- coupling blocks ---------------------------------------------------------
    def block_from_ocean(self, l) -> sp.csr_matrix:
        """Atmosphere::getBlock(ocean) (502-613): d F_atmos / d T_ocean(surface)."""
        n, m, P = self.n, self.m, self.P
        N_o = 6 * n * m * l
        rows, cols, vals = [], [], []
        for j in range(m):
            for i in range(n):
                sr = j * n + i
                M = self.msi[sr]
                if self.surf[j, i] != 0:
                    continue
                oc = 6 * (((l - 1) * m + j) * n + i) + 4
                dTFT = 1.0 - M
                dTFQ = P.nuq * P.tdim / P.qdim * P.dqso * (1.0 - M)
                for xx, v in ((TT, dTFT), (QQ, dTFQ)):
                    r = self.row(i, j, xx)
                    if r == self.rowint:
                        continue
                    rows.append(r); cols.append(oc); vals.append(v)
                qid = self.row(i, j, QQ)
                dTFP = self.intc[qid] * (1.0 / self.total_area) * (P.tdim / P.qdim) * P.dqso * (1.0 - M)
                rows.append(self.rowP); cols.append(oc); vals.append(dTFP)
        return sp.csr_matrix((vals, (rows, cols)), shape=(self.dim, N_o))

    def block_to_ocean(self, l, ocean_surf, deps, comb, sunp, coupled_s=False,
                       rowintcon=-1) -> sp.csr_matrix:
        """Ocean::getBlock(atmos) (Ocean.C:1538-1667), coupled_T = 1 (and coupled_S).
        deps = getdeps (Ooa, Os, nus, eta, lvsc, qdim, pQSnd); comb/sunp: the ocean's."""
        n, m, P = self.n, self.m, self.P
        Ooa, _, nus, eta, lvsc, qdim, _ = [float(v) for v in deps]
        N_o = 6 * n * m * l
        rows, cols, vals = [], [], []
        osurf = np.asarray(ocean_surf).reshape(m, n)
        for j in range(m):
            for i in range(n):
                if osurf[j, i] != 0:
                    continue
                sr = j * n + i
                M = self.msi[sr]
                S = self.suno_ocean[j] if hasattr(self, "suno_ocean") else self.suno[j + 1]
                r = 6 * (((l - 1) * m + j) * n + i) + 4
                dTFT = Ooa * (1.0 - M)
                dAFT = -comb * sunp * S * P.da * (1.0 - M)
                dQFT = lvsc * eta * qdim * (1.0 - M)
                for c, v in ((self.row(i, j, TT), -dTFT), (self.row(i, j, AA), -dAFT),
                             (self.row(i, j, QQ), -dQFT)):
                    rows.append(r); cols.append(c); vals.append(v)
                rs = r + 1                          # the surface S row
                if coupled_s and rs != rowintcon:
                    dQFS = -nus * (1.0 - M)
                    dPFS = -nus * self.pdist[sr] * (1.0 - M)
                    for c, v in ((self.row(i, j, QQ), -dQFS), (self.rowP, -dPFS)):
                        rows.append(rs); cols.append(c); vals.append(v)
        return sp.csr_matrix((vals, (rows, cols)), shape=(N_o, self.dim))


def fd_jacobian(fun, x, h=1e-6):
    """Central-difference Jacobian of fun at x (columns one by one)."""
    x = np.asarray(x, dtype=np.float64)
    J = np.zeros((len(fun(x)), len(x)))
    for c in range(len(x)):
        e = np.zeros_like(x)
        e[c] = h
        J[:, c] = (fun(x + e) - fun(x - e)) / (2 * h)
    return J
