"""The CPU twin of the block Gauss-Seidel preconditioner (oracle/prec_oracle.c) on its own:
the default variant, the early T/S right-hand side (ts_at) and the correction passes without
the Schur solve (schur_passes) are fixed linear operators that precondition FGMRES to the
tolerance; ts_at = dyn_iters and schur_passes = dyn_iters are the defaults."""
import numpy as np
import pytest

from iemic import config as cf
from helpers import mask_fix


@pytest.fixture(scope="module")
def system(oracle_lib):
    cfg = cf.preset("global4", mixing=1)
    L = mask_fix(oracle_lib, cfg, cf.landmask(cfg))
    o = oracle_lib.Oracle(cfg.ref_dict(), L, cfg.par_list())
    x = cf.synthetic_state(cfg, L, amp_ts=1e-3)
    val, _ = o.jacobian(x)
    return cfg, o, val, o.rhs(x)


@pytest.mark.parametrize("ts_at,schur_passes", [(0, 0), (1, 0), (2, 0), (0, 2), (2, 2)])
def test_block_gs_cpu_linear_and_converges(oracle_lib, system, ts_at, schur_passes):
    cfg, o, val, F = system
    P = oracle_lib.BlockGS(o, val, 3, dyn_iters=4, dyn_omega=0.95, ts_mg=1, ts_at=ts_at,
                           schur_passes=schur_passes)
    r1, r2 = cf.synthetic_vector(cfg, seed=3), cf.synthetic_vector(cfg, seed=4)
    z = P.apply(0.5 * r1 + r2)
    zl = 0.5 * P.apply(r1) + P.apply(r2)
    assert np.max(np.abs(z - zl)) <= 1e-10 * np.max(np.abs(z))
    _, its, rel, _ = P.fgmres(np.ascontiguousarray(-F), tol=1e-8, m=100, maxit=600)
    assert rel <= 1e-8 and its < 200


def test_ts_at_last_pass_is_default(oracle_lib, system):
    cfg, o, val, _ = system
    r = cf.synthetic_vector(cfg, seed=3)
    kw = dict(dyn_iters=4, dyn_omega=0.95, ts_mg=1)
    z0 = oracle_lib.BlockGS(o, val, 3, **kw).apply(r)
    z4 = oracle_lib.BlockGS(o, val, 3, ts_at=4, **kw).apply(r)
    z2 = oracle_lib.BlockGS(o, val, 3, ts_at=2, **kw).apply(r)
    assert np.array_equal(z0, z4)
    assert not np.array_equal(z0, z2)


def test_schur_passes_all_is_default(oracle_lib, system):
    cfg, o, val, _ = system
    r = cf.synthetic_vector(cfg, seed=3)
    kw = dict(dyn_iters=4, dyn_omega=0.95, ts_mg=1)
    z0 = oracle_lib.BlockGS(o, val, 3, **kw).apply(r)
    z4 = oracle_lib.BlockGS(o, val, 3, schur_passes=4, **kw).apply(r)
    z2 = oracle_lib.BlockGS(o, val, 3, schur_passes=2, **kw).apply(r)
    assert np.array_equal(z0, z4)
    assert not np.array_equal(z0, z2)
