"""Latitude-band decomposition on the CPU: world_size 2 and 3 over gloo.

Each rank assembles its band with the device code run on the CPU (tests/emul), after a
halo exchange of the state done exactly like comm.hip (whole latitude rows, contiguous in
the ext layout, sent to the neighbouring bands), and sums the integral-condition dot over
the ranks.  Every rank's Jacobian rows (Epetra CSR, reference numbering) and residual rows
must be bit-identical to the oracle's rows of the undivided problem.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HALO = 2


def band(rank, nranks, m):
    return rank * m // nranks, (rank + 1) * m // nranks


def _worker(rank, nranks, name, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "i-emic_amd"), os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        from helpers import Emul, golden_landm
        from iemic import config as cf
        from oracle import oracle as orc
        c = cf.preset(name, mixing=0)
        L = golden_landm(name)
        x = cf.synthetic_state(c, L)
        jb0, jb1 = band(rank, nranks, c.m)
        e = Emul(c, L, jb0, jb1)
        xe = e.to_ext(x)
        slab = 6 * c.l * c.n
        o0, o1 = HALO * slab, HALO * slab + (jb1 - jb0) * slab
        # halo exchange of HALO latitude rows (comm.hip halo_exchange)
        t = torch.from_numpy(xe)
        reqs = []
        if rank > 0:
            reqs.append(dist.isend(t[o0:o0 + HALO * slab].clone(), rank - 1))
            lo = torch.empty(HALO * slab, dtype=torch.float64)
            reqs.append(dist.irecv(lo, rank - 1))
        if rank < nranks - 1:
            reqs.append(dist.isend(t[o1 - HALO * slab:o1].clone(), rank + 1))
            hi = torch.empty(HALO * slab, dtype=torch.float64)
            reqs.append(dist.irecv(hi, rank + 1))
        for r in reqs:
            r.wait()
        if rank > 0:
            xe[o0 - HALO * slab:o0] = lo.numpy()
        if rank < nranks - 1:
            xe[o1:o1 + HALO * slab] = hi.numpy()
        # assembly of the band
        Be = e.jacobian_ext(xe)
        rowptr, col, val = e.csr()
        Fe, part = e.rhs_ext(xe)
        s = torch.tensor([part], dtype=torch.float64)
        dist.all_reduce(s)
        F = e.to_ref(Fe)
        B = e.to_ref(Be)
        # oracle of the whole problem, restricted to this band's rows
        o = orc.Oracle(c.ref_dict(), L, c.par_list())
        ov, oB = o.jacobian(x)
        oF = o.rhs(x)
        rows = [6 * ((k * c.m + j) * c.n + i) + v for k in range(c.l) for j in range(jb0, jb1)
                for i in range(c.n) for v in range(6)]
        ok = True
        for a, r in enumerate(rows):
            b0, b1 = o.rowptr[r], o.rowptr[r + 1]
            if not (np.array_equal(col[rowptr[a]:rowptr[a + 1]], o.col[b0:b1]) and
                    np.array_equal(val[rowptr[a]:rowptr[a + 1]], ov[b0:b1])):
                ok = False
        rows = np.array(rows)
        ri = o.rowintcon
        Fr = F[rows].copy()
        if ri >= 0:
            s_val = c.int_sign * s.item()
            assert abs(s_val - oF[ri]) <= 1e-13 * max(1.0, abs(oF[ri]))
            Fr[rows == ri] = oF[ri]
        ok &= np.array_equal(Fr.view(np.int64), oF[rows].view(np.int64))
        ok &= np.array_equal(B[rows].view(np.int64), oB[rows].view(np.int64))
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(flag)
        if rank == 0:
            q.put(int(flag.item()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,nranks", [("gateway16", 2), ("natl8", 3), ("gateway16", 4)])
def test_band_assembly_matches_oracle(oracle_lib, emul, name, nranks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + nranks + (hash(name) % 100)
    procs = [ctx.Process(target=_worker, args=(r, nranks, name, port, q)) for r in range(nranks)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == 0


def test_band_partition_matches_library_rule():
    """iemic_create_dist splits rows as r*m//P (C integer division); every band >= HALO rows."""
    for m, P in [(76, 8), (38, 8), (152, 8), (16, 4)]:
        bands = [band(r, P, m) for r in range(P)]
        assert bands[0][0] == 0 and bands[-1][1] == m
        assert all(b1 - b0 >= HALO for b0, b1 in bands)
        assert all(bands[r][1] == bands[r + 1][0] for r in range(P - 1))
