"""Decomp2D subdomains on the GPU (TRIOS_Domain.C:81-195): latitude bands
(npx = 1), x splits and 2-D process grids.

* In-process group (one GPU, one host thread per subdomain, host-staged collectives):
  every subdomain's Jacobian rows equal the oracle's bit for bit, the residual norm equals
  the oracle's, and the distributed Newton step solves the linearised system of the whole
  problem: ||F + J dx|| <= 1e-8 ||F|| with dx gathered from the subdomains.
* Across processes: several processes on one GPU through the library's host transport
  (iemic.transport.GlooTransport over gloo) run the library's own exchange batches
  (comm.hip run_msgs); RCCL with one GPU per process is skipped on a one-GPU box (RCCL
  refuses two ranks on one device); the driver's multi-GPU bench exercises it.
"""
import os
import threading

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import free_port, golden_landm, mask_fix
from iemic import config as cf

pytestmark = pytest.mark.gpu


def owned_rows(c, lay):
    return [6 * ((k * c.m + j) * c.n + i) + v for k in range(c.l) for j in range(lay["jb0"], lay["jb1"])
            for i in range(lay["ib0"], lay["ib1"]) for v in range(6)]


@pytest.mark.parametrize("name,nranks,npx", [("natl8", 2, 1), ("gateway16", 2, 1), ("gateway16", 3, 1),
                                             ("global4", 4, 1), ("natl8", 2, 2), ("gateway16", 2, 2),
                                             ("gateway16", 4, 2), ("global4", 4, 0), ("global4", 6, 3)])
def test_subdomains_in_one_process(oracle_lib, name, nranks, npx):
    from iemic import _lib
    from iemic.ocean import Ocean
    c = cf.preset(name, mixing=0)
    L0 = golden_landm(name)
    L = mask_fix(oracle_lib, c, L0)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    ov, _ = o.jacobian(x)
    oF = o.rhs(x)
    group = _lib.lib().iemic_local_group_new(nranks)
    res = [None] * nranks
    x1 = np.zeros(c.nrows)

    def work(r):
        try:
            oc = Ocean(c, landm=L0, local_group=group, rank=r, nranks=nranks, npx=npx,
                       solver_params={"Preconditioner": 2, "FGMRES tolerance": 1e-10,
                                      "FGMRES iterations": 1000})
            oc.setState(x)
            oc.computeJacobian()
            rowptr, col, val = oc.exportCSR()
            lay = oc.layout()
            F = np.zeros(c.nrows)
            _lib.check(_lib.lib().iemic_rhs(oc._h, _lib.ptr(F)), "rhs")
            info = oc.newtonStep()
            _lib.check(_lib.lib().iemic_get_state(oc._h, _lib.ptr(x1)), "get_state")
            res[r] = dict(lay=lay, csr=(rowptr, col, val), F=F, info=info)
            oc.close()
        except Exception as e:  # noqa: BLE001
            res[r] = dict(err=repr(e))

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    _lib.lib().iemic_local_group_free(group)
    errs = [r["err"] for r in res if r and "err" in r]
    assert not errs, errs
    covered = []
    for r in res:
        rowptr, col, val = r["csr"]
        rows = owned_rows(c, r["lay"])
        covered += rows
        for a, q in enumerate(rows):
            b0, b1 = o.rowptr[q], o.rowptr[q + 1]
            np.testing.assert_array_equal(col[rowptr[a]:rowptr[a + 1]], o.col[b0:b1])
            np.testing.assert_array_equal(val[rowptr[a]:rowptr[a + 1]], ov[b0:b1])
        Fr = r["F"][rows].copy()
        ri = o.rowintcon
        if ri in rows:
            k = rows.index(ri)
            assert abs(Fr[k] - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
            Fr[k] = oF[ri]
        np.testing.assert_array_equal(Fr.view(np.int64), oF[rows].view(np.int64))
    assert sorted(covered) == list(range(c.nrows))
    f0 = np.linalg.norm(oF)
    for r in res:
        assert abs(r["info"].norm_f0 - f0) <= 1e-12 * f0
        assert r["info"].solve.converged == 1
    lin = np.linalg.norm(oF + o.spmv(ov, x1 - x)) / f0
    assert lin <= 1e-8
    f1 = np.linalg.norm(o.rhs(x1))
    assert abs(res[0]["info"].norm_f1 - f1) <= 1e-9 * f1 + 1e-14 * f0


@pytest.mark.parametrize("nranks,npx,schur_passes", [(2, 1, 0), (8, 1, 0), (4, 0, 0), (8, 0, 0),
                                                     (4, 1, 2), (8, 0, 2)])
def test_subdomains_global2_newton_mixing(oracle_lib, nranks, npx, schur_passes):
    """The bench workload split as the multi-GPU bench splits it (global 2 deg, Mixing = 1,
    default solver: block GS with 4 damped defect passes, T/S multigrid per subdomain;
    npx = 0: the reference's Decomp2D, 2 x 2 and 4 x 2; schur_passes 2: the middle two
    passes without the Schur reduction): the distributed Newton step converges and solves the
    linearised system of the whole problem."""
    from iemic.ocean import Ocean
    c = cf.preset("global2", mixing=1)
    L0 = cf.init_landmask(c, cf.landmask(c))
    L = mask_fix(oracle_lib, c, L0)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    x1 = np.zeros(c.nrows)

    def fn(r, group):
        from iemic import _lib
        oc = Ocean(c, landm=L0, local_group=group, rank=r, nranks=nranks, npx=npx,
                   solver_params={"FGMRES iterations": 100, "FGMRES restarts": 20,
                                  "Schur passes": schur_passes})
        oc.setState(x)
        info = oc.newtonStep()
        lay = oc.layout()
        xx = np.zeros(c.nrows)
        _lib.check(_lib.lib().iemic_get_state(oc._h, _lib.ptr(xx)), "get_state")
        oc.close()
        return dict(lay=lay, info=info, x=xx)

    res = _run_bands(nranks, fn)
    for r in res:
        rows = np.array(owned_rows(c, r["lay"]))
        x1[rows] = r["x"][rows]
        assert r["info"].solve.converged == 1
    ov, _ = o.jacobian(x)
    F0 = o.rhs(x)
    lin = np.linalg.norm(F0 + o.spmv(ov, x1 - x)) / np.linalg.norm(F0)
    assert lin <= 2e-8, lin


def _run_bands(nranks, fn):
    """Run fn(rank, group) on nranks host threads sharing one in-process group."""
    from iemic import _lib
    group = _lib.lib().iemic_local_group_new(nranks)
    res = [None] * nranks

    def work(r):
        try:
            res[r] = fn(r, group)
        except Exception as e:  # noqa: BLE001
            res[r] = dict(err=repr(e))

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    _lib.lib().iemic_local_group_free(group)
    errs = [r["err"] for r in res if isinstance(r, dict) and "err" in r]
    assert not errs, errs
    return res


@pytest.mark.parametrize("name,nranks,npx,prec", [("natl8", 2, 1, 1), ("natl8", 2, 1, 2),
                                                  ("gateway16", 3, 1, 2), ("global4", 4, 1, 2),
                                                  ("natl8", 2, 2, 2), ("gateway16", 4, 2, 2),
                                                  ("global4", 4, 2, 2), ("natl8", 2, 2, 1),
                                                  ("global4", 8, 0, 2)])
def test_subdomains_spmv_and_solve(oracle_lib, name, nranks, npx, prec):
    """Subdomain SpMV equals the oracle's J v on the owned rows; a distributed FGMRES solve
    (block Jacobi, block GS) gives ||b - J x|| <= 1e-8 ||b|| globally."""
    from iemic import _lib
    from iemic.ocean import Ocean
    c = cf.preset(name, mixing=0)
    L0 = golden_landm(name)
    L = mask_fix(oracle_lib, c, L0)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    ov, _ = o.jacobian(x)
    v = cf.synthetic_vector(c)
    yref = o.spmv(ov, v)
    b = -o.rhs(x)
    y = np.zeros(c.nrows)
    xs = np.zeros(c.nrows)

    def fn(r, group):
        oc = Ocean(c, landm=L0, local_group=group, rank=r, nranks=nranks, npx=npx,
                   solver_params={"Preconditioner": prec, "FGMRES tolerance": 1e-10,
                                  "FGMRES iterations": 1000})
        oc.setState(x)
        oc.computeJacobian()
        lay = oc.layout()
        yy = oc.applyMatrix(v)
        sol = oc.solve(b)
        oc.close()
        return dict(lay=lay, y=yy, sol=sol)

    res = _run_bands(nranks, fn)
    for r in res:
        rows = np.array(owned_rows(c, r["lay"]))
        y[rows] = r["y"][rows]
        xs[rows] = r["sol"][rows]
    scale = np.abs(ov).max() * np.abs(v).max()
    assert np.max(np.abs(y - yref)) <= 1e-13 * scale
    lin = np.linalg.norm(b - o.spmv(ov, xs)) / np.linalg.norm(b)
    assert lin <= 1e-8, lin


def _rccl_worker(rank, nranks, npx, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "i-emic_amd"), os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        from iemic.ocean import Ocean
        ids = [Ocean.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, 0)
        c = cf.preset("gateway16", mixing=0)
        L0 = golden_landm("gateway16")
        oc = Ocean(c, landm=L0, device=rank, rank=rank, nranks=nranks, comm_id=ids[0], npx=npx,
                   solver_params={"FGMRES tolerance": 1e-10})
        assert oc.comm_size() == (nranks, "rccl"), oc.comm_size()
        L = oc.landmask().reshape(c.l + 2, c.m + 2, c.n + 2)
        x = cf.synthetic_state(c, L, amp_ts=1e-3)
        v = cf.synthetic_vector(c, seed=5)
        oc.setState(x)
        oc.computeJacobian()
        y = oc.applyMatrix(v)
        sol = oc.solve(y)
        lay = oc.layout()
        q.put((rank, {"lay": lay, "y": y, "sol": sol, "x": x, "v": v,
                      "converged": oc.last_solve.converged}))
        oc.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("npx", [1, 2])
def test_rccl_ranks(oracle_lib, npx):
    """Two ranks, one GPU each, over RCCL (latitude bands, and an x split whose strided
    messages go through the device staging buffer): J (through J v), the halo exchanges and
    the Krylov all-reduces of a solve; the gathered owned rows match the oracle."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL refuses two ranks on one device)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rccl_worker, args=(r, 2, npx, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert all(isinstance(v, dict) for v in out.values()), out
    c = cf.preset("gateway16", mixing=0)
    L = mask_fix(oracle_lib, c, golden_landm("gateway16"))
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x, v = out[0]["x"], out[0]["v"]
    ov, _ = o.jacobian(x)
    yref = o.spmv(ov, v)
    y = np.zeros(c.nrows)
    xs = np.zeros(c.nrows)
    for r in out.values():
        rows = np.array(owned_rows(c, r["lay"]))
        y[rows] = r["y"][rows]
        xs[rows] = r["sol"][rows]
        assert r["converged"] == 1
    assert np.max(np.abs(y - yref)) <= 1e-13 * np.abs(ov).max() * np.abs(v).max()
    lin = np.linalg.norm(yref - o.spmv(ov, xs)) / np.linalg.norm(yref)
    assert lin <= 1e-8, lin


def _transport_worker(rank, nranks, npx, name, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "i-emic_amd"), os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        from iemic.ocean import Ocean
        from iemic.transport import GlooTransport
        c = cf.preset(name, mixing=0)
        L0 = golden_landm(name)
        tp = GlooTransport()
        oc = Ocean(c, landm=L0, device=0, rank=rank, nranks=nranks, npx=npx, transport=tp,
                   solver_params={"FGMRES tolerance": 1e-10, "FGMRES iterations": 1000})
        L = oc.landmask().reshape(c.l + 2, c.m + 2, c.n + 2)
        x = cf.synthetic_state(c, L, amp_ts=1e-3)
        v = cf.synthetic_vector(c, seed=5)
        oc.setState(x)
        oc.computeJacobian()
        rowptr, col, val = oc.exportCSR()
        y = oc.applyMatrix(v)
        colint = oc.getColumnIntegral()
        info = oc.newtonStep()
        x1 = oc.getState().copy()
        lay = oc.layout()
        q.put((rank, {"lay": lay, "y": y, "x": x, "v": v, "x1": x1, "csr": (rowptr, col, val),
                      "converged": info.solve.converged, "f0": info.norm_f0, "f1": info.norm_f1,
                      "colint": colint, "coeff": oc.getIntCondCoeff(), "ri": oc.rowintcon,
                      "comm": oc.comm_size()}))
        oc.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,nranks,npx", [("gateway16", 2, 2), ("global4", 4, 2)])
def test_transport_processes(oracle_lib, name, nranks, npx):
    """One process per subdomain on one GPU, the library's exchange batches and sums over
    its host transport (gloo): J rows bit-exact, J v to 1e-13, and a Newton step whose
    gathered update solves the whole linearised system to 1e-8."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, nranks, npx, name, port, q))
             for r in range(nranks)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
    assert all(isinstance(v, dict) for v in out.values()), out
    c = cf.preset(name, mixing=0)
    L = mask_fix(oracle_lib, c, golden_landm(name))
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x, v = out[0]["x"], out[0]["v"]
    ov, _ = o.jacobian(x)
    yref = o.spmv(ov, v)
    y = np.zeros(c.nrows)
    x1 = np.zeros(c.nrows)
    for r in out.values():
        rows = owned_rows(c, r["lay"])
        rowptr, col, val = r["csr"]
        for a, qr in enumerate(rows):
            b0, b1 = o.rowptr[qr], o.rowptr[qr + 1]
            np.testing.assert_array_equal(col[rowptr[a]:rowptr[a + 1]], o.col[b0:b1])
            np.testing.assert_array_equal(val[rowptr[a]:rowptr[a + 1]], ov[b0:b1])
        rows = np.array(rows)
        y[rows] = r["y"][rows]
        x1[rows] = r["x1"][rows]
        assert r["converged"] == 1
    assert np.max(np.abs(y - yref)) <= 1e-13 * np.abs(ov).max() * np.abs(v).max()
    # Ocean::getColumnIntegral over the ranks (Epetra SumAll): the whole matrix's S-column sums
    coef = np.zeros(c.nrows)
    for r in out.values():
        rows = np.array(owned_rows(c, r["lay"]))
        coef[rows] = r["coeff"][rows]
        assert r["comm"] == (nranks, "host")
    ri = out[0]["ri"]
    if ri >= 0:
        coef[ri] = 0.0
    ref = np.zeros(c.nrows)
    np.add.at(ref, o.col, coef[np.repeat(np.arange(c.nrows), np.diff(o.rowptr))] * ov)
    ref[np.arange(c.nrows) % 6 != 5] = 0.0
    for r in out.values():
        np.testing.assert_allclose(r["colint"], ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    F0 = o.rhs(x)
    f0 = np.linalg.norm(F0)
    assert abs(out[0]["f0"] - f0) <= 1e-12 * f0
    lin = np.linalg.norm(F0 + o.spmv(ov, x1 - x)) / f0
    assert lin <= 1e-8, lin


def test_unmatched_exchange_fails_fast(oracle_lib):
    """Fail-fast path (comm.hip group_barrier / rccl_wait): a halo exchange whose peer never
    posts the matching call returns IEMIC_EDEVICE within the context's bound instead of
    hanging.  Both ranks are created (creation is collective and checks that the exchange
    plans pair up); then only rank 0 runs an SpMV, whose halo batch waits for rank 1."""
    import time
    from iemic import _lib
    from iemic.ocean import Ocean
    c = cf.preset("natl8", mixing=0)
    L0 = golden_landm("natl8")
    group = _lib.lib().iemic_local_group_new(2)
    ocs = [None, None]

    def mk(r):
        ocs[r] = Ocean(c, landm=L0, local_group=group, rank=r, nranks=2, npx=1)

    th = [threading.Thread(target=mk, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert all(o is not None for o in ocs)
    oc = ocs[0]
    _lib.check(_lib.lib().iemic_set_comm_timeout(oc._h, 2.0), "set_comm_timeout")
    x = np.zeros(c.nrows)
    oc.setState(x)
    t0 = time.perf_counter()
    with pytest.raises(_lib.IemicError, match="did not arrive"):
        oc.applyMatrix(x)
    dt = time.perf_counter() - t0
    assert dt < 10.0, dt
    for o in ocs:
        o.close()
    _lib.lib().iemic_local_group_free(group)


@pytest.mark.parametrize("nranks", [1, 2, 4])
def test_reused_preconditioner_after_new_jacobian(oracle_lib, nranks):
    """Ocean::solve reuses the preconditioner until preProcess flags a rebuild (Ocean.C:790-801,
    1360-1374), and TRIOS::BlockPreconditioner keeps applying the blocks it extracted from the
    set-up Jacobian.  The block GS is set up at state x, then J is assembled at x2 (into the
    second Jacobian buffer):
    * the apply is bitwise the apply before the new Jacobian, on every band: the bands'
      halo-row recomputation and the owners' kernels read the same set-up Jacobian;
    * the solve with the reused preconditioner (compressed basis, SpMV of J(x2) from the
      repacked stream) solves the new system: ||b - J(x2) s|| <= 1e-8 ||b|| with the oracle's
      J(x2); and a rebuilt preconditioner (preProcess) still gives the same solution."""
    from iemic import _lib
    from iemic.ocean import Ocean
    name = "global4"
    c = cf.preset(name, mixing=0)
    L0 = golden_landm(name)
    L = mask_fix(oracle_lib, c, L0)
    o = oracle_lib.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    x2 = cf.synthetic_state(c, L, seed=11, amp_ts=2e-3)
    r = cf.synthetic_vector(c, seed=3)
    b1, b2 = -o.rhs(x), -o.rhs(x2)
    sp = {"Preconditioner": 2, "FGMRES tolerance": 1e-10, "FGMRES iterations": 1000}

    def fn(rk, group):
        kw = dict(local_group=group, rank=rk, nranks=nranks, npx=1) if group is not None else {}
        oc = Ocean(c, landm=L0, solver_params=sp, **kw)
        oc.setState(x)
        oc.computeJacobian()
        oc.solve(b1)                           # builds the block GS at x
        z0 = oc.applyPrecon(r).copy()
        oc.setState(x2)
        oc.computeJacobian()                   # J(x2), the preconditioner stays that of x
        z1 = oc.applyPrecon(r).copy()
        s2 = oc.solve(b2).copy()
        info = oc.last_solve
        oc.preProcess()
        s3 = oc.solve(b2).copy()
        lay = oc.layout()
        oc.close()
        return dict(lay=lay, z0=z0, z1=z1, s2=s2, s3=s3, conv=info.converged)

    res = [fn(0, None)] if nranks == 1 else _run_bands(nranks, fn)
    s2, s3 = np.zeros(c.nrows), np.zeros(c.nrows)
    for q in res:
        rows = np.array(owned_rows(c, q["lay"]))
        np.testing.assert_array_equal(q["z1"][rows].view(np.int64), q["z0"][rows].view(np.int64))
        assert q["conv"] == 1
        s2[rows] = q["s2"][rows]
        s3[rows] = q["s3"][rows]
    ov2, _ = o.jacobian(x2)
    nb = np.linalg.norm(b2)
    assert np.linalg.norm(b2 - o.spmv(ov2, s2)) <= 1e-8 * nb
    assert np.linalg.norm(b2 - o.spmv(ov2, s3)) <= 1e-8 * nb


def test_mid_solve_mismatch_fails_fast():
    """Fail-fast in the middle of a solve (comm.hip: every barrier of the in-process group,
    every host wait of an RCCL context is bounded): both ranks run FGMRES without reaching its
    tolerance, rank 1 with 10 steps, rank 0 with 40, so rank 0's collectives from step 11 on
    have no partner.  Rank 0's solve returns an error within the 2 s bound instead of hanging,
    and every rank returns."""
    import time
    from iemic import _lib
    from iemic.ocean import Ocean
    c = cf.preset("natl8", mixing=0)
    L0 = golden_landm("natl8")
    x = cf.synthetic_state(c, L0, amp_ts=1e-3)
    b = cf.synthetic_vector(c, seed=9)

    def fn(r, group):
        sp = {"Preconditioner": 2, "FGMRES tolerance": 1e-30, "FGMRES restarts": 0,
              "FGMRES iterations": 40 if r == 0 else 10}
        oc = Ocean(c, landm=L0, local_group=group, rank=r, nranks=2, npx=1, solver_params=sp)
        _lib.check(_lib.lib().iemic_set_comm_timeout(oc._h, 2.0), "set_comm_timeout")
        oc.setState(x)
        oc.computeJacobian()
        t0 = time.perf_counter()
        err = None
        try:
            oc.solve(b)
        except _lib.IemicError as e:
            err = str(e)
        dt = time.perf_counter() - t0
        oc.close()
        return dict(msg=err, dt=dt)

    t0 = time.perf_counter()
    res = _run_bands(2, fn)
    assert time.perf_counter() - t0 < 60.0
    assert res[0]["msg"] is not None, res
    assert res[0]["dt"] < 20.0, res
