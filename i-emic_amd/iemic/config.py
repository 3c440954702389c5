"""THCM configurations and input preparation (land mask, synthetic states).

Host-side input data only; nothing here computes the hot path.

* ``THCMConfig`` mirrors the THCM ParameterList consumed by the reference
  (defaults: ``THCM::getDefaultInitParameters``, src/ocean/THCM.C:2748-2813; names:
  THCM.C:189-265).
* ``landmask()`` restates the serial land-mask pipeline of the reference:
  ``m_global::get_landm`` -> ``topofit`` (src/ocean/topo.F90:6-134 readmask,
  136-336 depth3land, itopo = 1 case) that the THCM constructor hands to ``init_``
  (THCM.C:378-397, 583-589).  The border handling done inside ``init``
  (usrc.F90:83-107) is applied by the device library itself, like the reference.
* Presets reproduce the reference's run/test XML files (test/ocean, test/2dmoc,
  run/ocean/global) and the synthetic benchmark grids of SURVEY.md §8d (C2 4°,
  C3 "2°", C5 "1°").
"""
from __future__ import annotations

import dataclasses
import os
from typing import Dict, Optional

import numpy as np

OCEAN, LAND, WATER, PERIO = 0, 1, 2, 3
NUN = 6
DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")

# THCM::par2int (src/ocean/THCM.C:1754-1807)
PAR_INDEX = {
    "AL_T": 1, "Rayleigh-Number": 2, "Vertical Ekman-Number": 3,
    "Horizontal Ekman-Number": 4, "Rossby-Number": 5, "MIXP": 6, "RESC": 7, "SPL1": 8,
    "Salinity Homotopy": 9, "Solar Forcing": 10, "Horizontal Peclet-Number": 11,
    "Vertical Peclet-Number": 12, "P_VC": 13, "LAMB": 14, "Salinity Forcing": 15,
    "Wind Forcing": 16, "Temperature Forcing": 17, "Nonlinear Factor": 18,
    "Combined Forcing": 19, "ARCL": 20, "NLES": 21, "IFRICB": 22, "CONT": 23,
    "Energy": 24, "ALPC": 25, "CMPR": 26, "Flux Perturbation": 27,
    "Salinity Perturbation": 28, "MKAP": 29, "SPL2": 30,
}


@dataclasses.dataclass
class THCMConfig:
    """Subset of the THCM ParameterList used on the hot path (THCM.C:189-265)."""
    name: str = "Unnamed"
    n: int = 16
    m: int = 16
    l: int = 16
    xmin: float = 286.0           # degrees, "Global Bound xmin"
    xmax: float = 350.0
    ymin: float = 10.0
    ymax: float = 74.0
    periodic: bool = False
    hdim: float = 4000.0
    qz: float = 1.0
    topography: int = 1           # itopo
    flat: bool = False
    read_land_mask: bool = False
    land_mask: str = "no_mask_specified"
    inhomogeneous_mixing: int = 0  # ih
    mixing: int = 1               # vmix
    rho_mixing: bool = True
    taper: int = 1
    alpha_t: float = 1.0e-4
    alpha_s: float = 7.6e-4
    tres: int = 1
    sres: int = 1
    int_sign: int = -1
    levitus_t: int = 1            # ite
    levitus_s: int = 1            # its
    wind_forcing_type: int = 2    # iza
    coriolis: int = 1
    forcing_type: int = 0
    integral_i: int = -1
    integral_j: int = -1
    coupled_t: int = 0            # "Coupled Temperature" (coupled_T, THCM.C:232)
    coupled_s: int = 0            # "Coupled Salinity" (coupled_S)
    fix_pressure_points: bool = False  # "Fix Pressure Points" (THCM.C:2201-2238): not restated
    refine: int = 1               # synthetic horizontal refinement of the mask
    refine_l: int = 0             # target layer count for vertical remap (0: none)
    start_params: Dict[str, float] = dataclasses.field(default_factory=dict)

    @property
    def ncell(self) -> int:
        return self.n * self.m * self.l

    @property
    def nrows(self) -> int:
        return NUN * self.ncell

    def validate(self) -> None:
        """Refuse, by name, the THCM options the device library does not restate (the model
        would otherwise silently run another problem)."""
        if self.fix_pressure_points:
            raise NotImplementedError(
                "THCM 'Fix Pressure Points' (THCM::fixPressurePoints, THCM.C:2201-2238) is not "
                "restated: the device model pins the pressure null space in the Schur solve "
                "instead; every reference run XML leaves it false (THCM.C:2792)")

    def par_list(self):
        """(index, value) pairs of the starting parameters, THCM::setParameter order."""
        out = []
        for k, v in self.start_params.items():
            if k not in PAR_INDEX:
                raise ValueError(f"invalid THCM parameter {k!r}")
            out.append((PAR_INDEX[k], float(v)))
        return out

    def with_(self, **kw) -> "THCMConfig":
        c = dataclasses.replace(self, **kw)
        c.start_params = dict(self.start_params)
        if "start_params" in kw:
            c.start_params = dict(kw["start_params"])
        return c

    def ref_dict(self) -> dict:
        """Flat dict used by the oracle/reference drivers (test infrastructure)."""
        return dict(
            n=self.n, m=self.m, l=self.l, xmin_deg=self.xmin, xmax_deg=self.xmax,
            ymin_deg=self.ymin, ymax_deg=self.ymax, periodic=int(self.periodic),
            hdim=self.hdim, qz=self.qz, itopo=self.topography, flat=int(self.flat),
            rd_mask=int(self.read_land_mask), maskfile=self.land_mask, tres=self.tres,
            sres=self.sres, iza=self.wind_forcing_type, ite=self.levitus_t,
            its=self.levitus_s, rd_spertm=0, coupled_T=self.coupled_t, coupled_S=self.coupled_s,
            forcing_type=self.forcing_type, ih=self.inhomogeneous_mixing, vmix=self.mixing,
            tap=self.taper, rho_mixing=int(self.rho_mixing), coriolis_on=self.coriolis,
            alphaT=self.alpha_t, alphaS=self.alpha_s, int_sign=self.int_sign,
            nic=self.integral_i, mic=self.integral_j)


# --------------------------------------------------------------------------------
# land mask (topo.F90)

def _read_mask_file(path: str, n: int, m: int, l: int) -> np.ndarray:
    """topo.F90:41-62 readmask: per level one header line, then rows j = m+1..0."""
    with open(path) as f:
        lines = f.read().split("\n")
    L = np.full((l + 2, m + 2, n + 2), LAND, dtype=np.int32)
    p = 0
    for k in range(l + 2):
        p += 1  # header
        for j in range(m + 1, -1, -1):
            s = lines[p]
            p += 1
            L[k, j, :] = [int(c) for c in s[: n + 2]]
    return L


def _fix_inversions(L: np.ndarray) -> None:
    """topo.F90:94-103 (also usrc.F90:372-381): land above ocean becomes land below."""
    l = L.shape[0] - 2
    for k in range(l, 1, -1):
        bad = (L[k, 1:-1, 1:-1] == LAND) & (L[k - 1, 1:-1, 1:-1] == OCEAN)
        L[k - 1, 1:-1, 1:-1][bad] = LAND


def _perio_borders(L: np.ndarray) -> None:
    """depth3land periodic marking (topo.F90:314-319), also matches the mask files."""
    n = L.shape[2] - 2
    both = (L[:, :, 1] == OCEAN) & (L[:, :, n] == OCEAN)
    L[:, :, 0] = np.where(both, PERIO, LAND)
    L[:, :, n + 1] = np.where(both, PERIO, LAND)


def _refine(L: np.ndarray, r: int, l_new: int) -> np.ndarray:
    """SURVEY.md §8d synthetic grids: r-fold nearest-neighbour horizontal refinement,
    vertical remap k' ocean iff source layer floor((k'+1/2) l / l') is ocean."""
    l, m2, n2 = L.shape[0] - 2, L.shape[1], L.shape[2]
    m, n = m2 - 2, n2 - 2
    ln = l_new if l_new > 0 else l
    out = np.full((ln + 2, r * m + 2, r * n + 2), LAND, dtype=np.int32)
    ksrc = [0] + [int(np.floor(((kp - 1) + 0.5) * l / ln)) + 1 for kp in range(1, ln + 1)] + [l + 1]
    jsrc = [0] + [(jp - 1) // r + 1 for jp in range(1, r * m + 1)] + [m + 1]
    isrc = [0] + [(ip - 1) // r + 1 for ip in range(1, r * n + 1)] + [n + 1]
    out[:] = L[np.ix_(ksrc, jsrc, isrc)]
    _fix_inversions(out)
    return out


def landmask(cfg: THCMConfig) -> np.ndarray:
    """Global land mask landm(0:n+1,0:m+1,0:l+1) as m_global::get_landm returns it,
    as an int32 array of shape (l+2, m+2, n+2) (i fastest in memory)."""
    if cfg.read_land_mask:
        n0, m0, l0 = cfg.n // cfg.refine, cfg.m // cfg.refine, cfg.l
        if cfg.refine_l:
            l0 = _mask_levels(cfg.land_mask)
        L = _read_mask_file(os.path.join(DATA_DIR, "mkmask", cfg.land_mask), n0, m0, l0)
        _fix_inversions(L)
        if cfg.flat:
            for k in range(1, L.shape[0] - 2):
                L[k] = L[L.shape[0] - 2]
        if cfg.refine > 1 or cfg.refine_l:
            L = _refine(L, cfg.refine, cfg.l)
            if cfg.periodic:
                _perio_borders(L)
        assert L.shape == (cfg.l + 2, cfg.m + 2, cfg.n + 2), L.shape
        return L
    if cfg.topography != 1:
        raise NotImplementedError("only itopo=1 (no continents) or a mask file")
    n, m, l = cfg.n, cfg.m, cfg.l
    L = np.full((l + 2, m + 2, n + 2), LAND, dtype=np.int32)
    L[1:l + 1, 1:m + 1, 1:n + 1] = OCEAN     # topo.F90:177-187
    if cfg.flat:
        for k in range(1, l):
            L[k] = L[l]
    if cfg.periodic:
        _perio_borders(L)
    return L


def _mask_levels(name: str) -> int:
    with open(os.path.join(DATA_DIR, "mkmask", name)) as f:
        lines = f.read().split("\n")
    hdr = sum(1 for s in lines if s.strip().startswith("_") or s.strip().startswith("level"))
    return hdr - 2


def init_landmask(cfg: THCMConfig, L: np.ndarray) -> np.ndarray:
    """The border handling init_ applies to its local copy (usrc.F90:83-107)."""
    L = L.copy()
    if not cfg.periodic:
        L[L == PERIO] = OCEAN
        L[:, :, 0] = LAND
        L[:, :, -1] = LAND
    L[:, 0, :] = LAND
    L[:, -1, :] = LAND
    L[0] = LAND
    L[-1] = LAND
    return L


# --------------------------------------------------------------------------------
# synthetic states: splitmix64 over the global row index

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64_uniform(seed: int, idx: np.ndarray) -> np.ndarray:
    """U[0,1) from splitmix64(seed + (idx+1) * golden), one draw per index."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def synthetic_state(cfg: THCMConfig, landm: np.ndarray, seed: int = 20261015,
                    amp_uvwp: float = 1e-3, amp_ts: float = 0.1) -> np.ndarray:
    """u,v,w,p ~ U(±1e-3), T,S ~ U(±0.1) on ocean cells, 0 on land."""
    N = cfg.nrows
    rows = np.arange(N, dtype=np.int64)
    r = splitmix64_uniform(seed, rows) * 2.0 - 1.0
    var = rows % NUN
    amp = np.where(var >= 4, amp_ts, amp_uvwp)
    x = r * amp
    ocean = (landm[1:-1, 1:-1, 1:-1] == OCEAN).reshape(-1)
    x = x.reshape(-1, NUN) * ocean[:, None]
    return np.ascontiguousarray(x.reshape(-1))


def prolong_state(cfg_c: THCMConfig, x_c: np.ndarray, cfg_f: THCMConfig, landm_f: np.ndarray) -> np.ndarray:
    """A state of a coarser global grid on a finer one (an initial guess, e.g. the 1-degree
    continuation state from the 2-degree branch state): each fine cell takes the values
    of the coarse cell containing it -- horizontal refinement r = n_f / n_c, layer k' from
    the coarse layer floor((k' + 1/2) l_c / l_f) (the mask refinement's rule) -- and land
    cells of the fine mask are 0."""
    r = cfg_f.n // cfg_c.n
    assert cfg_f.n == r * cfg_c.n and cfg_f.m == r * cfg_c.m
    xc = np.asarray(x_c, dtype=np.float64).reshape(cfg_c.l, cfg_c.m, cfg_c.n, NUN)
    ks = np.floor((np.arange(cfg_f.l) + 0.5) * cfg_c.l / cfg_f.l).astype(np.int64)
    js = np.arange(cfg_f.m) // r
    is_ = np.arange(cfg_f.n) // r
    xf = xc[np.ix_(ks, js, is_)]
    ocean = landm_f[1:-1, 1:-1, 1:-1] == OCEAN
    xf = xf * ocean[..., None]
    return np.ascontiguousarray(xf.reshape(-1))


def synthetic_vector(cfg: THCMConfig, seed: int = 7) -> np.ndarray:
    rows = np.arange(cfg.nrows, dtype=np.int64)
    return splitmix64_uniform(seed, rows) * 2.0 - 1.0


# --------------------------------------------------------------------------------
# presets

def preset(name: str, mixing: Optional[int] = None) -> THCMConfig:
    """Named configurations.  ``mixing`` overrides "Mixing" (vmix)."""
    if name == "test6x6x4":
        c = THCMConfig(name=name, n=6, m=6, l=4, read_land_mask=True, land_mask="test6x6x4",
                       topography=0, mixing=1, rho_mixing=False, sres=1,
                       start_params={"Combined Forcing": 0.5, "Salinity Forcing": 1.0,
                                     "Wind Forcing": 1.0, "Temperature Forcing": 10.0,
                                     "SPL1": 2.0e3, "SPL2": 0.01})
    elif name == "natl8":      # test/ocean/ocean_params.xml (test_ocean.C)
        c = THCMConfig(name=name, n=8, m=8, l=4, read_land_mask=True, land_mask="mask_natl8",
                       topography=0, mixing=1, rho_mixing=False, tres=1, sres=0,
                       start_params={"Combined Forcing": 0.5, "Solar Forcing": 0.0,
                                     "Salinity Forcing": 1.0, "Wind Forcing": 1.0,
                                     "Temperature Forcing": 10.0, "SPL1": 2.0e3,
                                     "SPL2": 0.01})
    elif name == "gateway16":  # test/ocean/reft_ocean_params.xml
        c = THCMConfig(name=name, n=16, m=16, l=16, xmin=300, xmax=340, ymin=20, ymax=60,
                       periodic=True, read_land_mask=True, land_mask="mask_gateway",
                       topography=0, mixing=2, rho_mixing=False, forcing_type=2, sres=1,
                       start_params={"Combined Forcing": 0.5, "Solar Forcing": 0.0,
                                     "Salinity Forcing": 0.1, "Wind Forcing": 1.0,
                                     "Temperature Forcing": 10.0, "SPL1": 2.0e3,
                                     "SPL2": 0.01})
    elif name in ("2dmoc", "2dmoc_run"):  # test/2dmoc (3x6x6) / run/2dmoc (4x32x16)
        nn, mm, ll = (3, 6, 6) if name == "2dmoc" else (4, 32, 16)
        c = THCMConfig(name=name, n=nn, m=mm, l=ll, xmin=286, xmax=350, ymin=-60, ymax=60,
                       periodic=True, topography=1, flat=True, mixing=1, rho_mixing=False,
                       coriolis=0, forcing_type=1, tres=1, sres=0,
                       start_params={"Combined Forcing": 0.5, "Solar Forcing": 0.0,
                                     "Salinity Forcing": 0.0, "Wind Forcing": 0.0,
                                     "Temperature Forcing": 10.0, "SPL1": 2e3,
                                     "SPL2": 0.01, "P_VC": 0.0, "Rossby-Number": 0.0,
                                     "CMPR": 0.0, "Horizontal Ekman-Number": 371.764,
                                     "Rayleigh-Number": 15.6869})
    elif name in ("global4", "global2", "global1"):
        # run/ocean/global/ocean_params.xml on mask_global_96x38x12; Levitus data files are
        # absent -> idealized T/S (ite = its = 1), wind type 2.
        r, ll = {"global4": (1, 12), "global2": (2, 16), "global1": (4, 32)}[name]
        c = THCMConfig(name=name, n=96 * r, m=38 * r, l=ll, xmin=0.0, xmax=359.99,
                       ymin=-85.5, ymax=85.5, periodic=True, hdim=5000.0, qz=2.25,
                       topography=0, read_land_mask=True, land_mask="mask_global_96x38x12",
                       mixing=1, rho_mixing=False, tres=1, sres=1, refine=r,
                       refine_l=(ll if ll != 12 else 0),
                       start_params={"Combined Forcing": 0.5, "Solar Forcing": 0.0,
                                     "Salinity Forcing": 1.0, "Wind Forcing": 1.0,
                                     "Temperature Forcing": 1.0, "SPL1": 2.0e3,
                                     "SPL2": 0.01, "Horizontal Ekman-Number": 0.0027037})
    elif name == "coupled_natl8s":
        # coupled_natl8 with "Coupled Salinity" = 1 as well (E - P salinity flux)
        c = preset("coupled_natl8").with_(name=name, coupled_s=1)
    elif name in ("coupled4", "coupled_natl8"):
        # run/coupled/ocean_params.xml: the global 4-degree ocean with Coupled Temperature 1,
        # Coupled Salinity 0, qz 1.5 (config C4); coupled_natl8: the same physics on the
        # 8x8x4 test basin (full-array fixtures)
        if name == "coupled4":
            c = preset("global4").with_(name=name, qz=1.5, coupled_t=1)
        else:
            c = preset("natl8").with_(name=name, coupled_t=1, sres=1)
        c.start_params = {"Combined Forcing": 0.5, "Solar Forcing": 1.0, "Salinity Forcing": 1.0,
                          "Wind Forcing": 1.0, "Temperature Forcing": 1.0, "SPL1": 2.0e3,
                          "SPL2": 0.01}
    else:
        raise KeyError(name)
    if mixing is not None:
        c.mixing = mixing
    return c


PRESETS = ("test6x6x4", "natl8", "gateway16", "2dmoc", "2dmoc_run", "global4", "global2",
           "global1", "coupled4", "coupled_natl8", "coupled_natl8s")
