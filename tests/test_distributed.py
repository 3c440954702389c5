"""Decomp2D domain decomposition (TRIOS_Domain.C:81-195) on the CPU over gloo.

Each rank builds the library's subdomain of its rank (tests/emul: decomp.h's partition and
neighbours, the device assembly code run on the CPU), refreshes the halo of its state by
executing the library's own exchange plan (decomp.h plan_ext: phase x, then phase y, the
k-th message from a to b paired with the k-th b receives from a) over gloo, assembles its
rows and sums the integral-condition dot over the ranks.  Every rank's Jacobian rows
(Epetra CSR, reference numbering) and residual rows must be bit-identical to the oracle's
rows of the undivided problem -- for latitude bands, x splits (periodic, with W = E at
npx = 2) and 2 x 2 / 3 x 1 process grids.
"""
import collections
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HALO = 2


def run_plan(msgs, v):
    """execute one phase of a plan on the flat vector v (gloo, tag = message index per peer)"""
    ks, kr = collections.Counter(), collections.Counter()
    reqs, recvs = [], []
    for send, peer, off, nblk, ln, stride in msgs:
        idx = off + (np.arange(nblk)[:, None] * stride + np.arange(ln)[None, :]).reshape(-1)
        if send:
            reqs.append(dist.isend(torch.from_numpy(v[idx].copy()), peer, tag=ks[peer]))
            ks[peer] += 1
        else:
            buf = torch.empty(idx.size, dtype=torch.float64)
            reqs.append(dist.irecv(buf, peer, tag=kr[peer]))
            kr[peer] += 1
            recvs.append((idx, buf))
    for r in reqs:
        r.wait()
    for idx, buf in recvs:
        v[idx] = buf.numpy()


def _worker(rank, nranks, npx, name, port, q):
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
        e = Emul(c, L, sub=(rank, nranks, npx))
        xe = e.to_ext(x)
        # the assembly halo: HALO rows and columns, the library's plan
        run_plan(e.plan(6, HALO, 0), xe)
        run_plan(e.plan(6, HALO, 1), xe)
        # every halo cell now holds the neighbour's value (corners included): compare with
        # the whole state laid out the same way
        full = Emul(c, L, sub=(rank, nranks, npx))
        ok = True
        Be = e.jacobian_ext(xe)
        rowptr, col, val = e.csr()
        Fe, part = e.rhs_ext(xe)
        s = torch.tensor([part], dtype=torch.float64)
        dist.all_reduce(s)
        F = e.to_ref(Fe)
        B = e.to_ref(Be)
        o = orc.Oracle(c.ref_dict(), L, c.par_list())
        ov, oB = o.jacobian(x)
        oF = o.rhs(x)
        rows = [6 * ((k * c.m + j) * c.n + i) + v for k in range(c.l) for j in range(e.jb0, e.jb1)
                for i in range(e.ib0, e.ib1) for v in range(6)]
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
        del full
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(flag)
        if rank == 0:
            q.put(int(flag.item()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,nranks,npx", [
    ("gateway16", 2, 1),     # latitude bands
    ("natl8", 3, 1),         # bands, uneven rows
    ("natl8", 2, 2),         # x split, closed basin
    ("gateway16", 2, 2),     # x split, periodic: W and E are the same rank
    ("gateway16", 4, 2),     # 2 x 2, periodic
    ("global4", 3, 3),       # 3 x 1, periodic, uneven columns
])
def test_subdomain_assembly_matches_oracle(oracle_lib, emul, name, nranks, npx):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    from helpers import free_port
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, nranks, npx, name, port, q)) for r in range(nranks)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == 0


def part_of(N, np_, p):
    return p * (N // np_) + min(p, N % np_), N // np_ + (1 if p < N % np_ else 0)


def test_decomp2d_matches_reference_rule(emul):
    """TRIOS_Domain.C:88-109 (factorisation) and 151-162 (remainders to the first ranks):
    2 degrees on 8 ranks is 4 x 2 with 48 x 38 subdomains."""
    from helpers import Emul, golden_landm
    from iemic import config as cf
    import ctypes as C
    lib = C.CDLL(os.path.join(os.path.dirname(__file__), "_build", "libstencil_emul.so"))
    a, b = C.c_int(), C.c_int()
    for (n, m, P), want in {(192, 76, 8): (4, 2), (96, 38, 4): (4, 1), (384, 152, 8): (4, 2),
                            (96, 38, 8): (4, 2), (16, 16, 4): (2, 2), (8, 8, 3): (3, 1)}.items():
        lib.emul_decomp2d(n, m, P, C.byref(a), C.byref(b))
        assert (a.value, b.value) == want, (n, m, P)
    c = cf.preset("global4", mixing=0)
    L = golden_landm("global4")
    for nranks, npx in [(8, 0), (3, 3), (6, 2)]:
        seen = np.zeros((c.m, c.n), dtype=int)
        for r in range(nranks):
            e = Emul(c, L, sub=(r, nranks, npx))
            px, py = r % e.npx, r // e.npx
            i0, nx = part_of(c.n, e.npx, px)
            j0, my = part_of(c.m, e.npy, py)
            assert (e.ib0, e.ib1, e.jb0, e.jb1) == (i0, i0 + nx, j0, j0 + my)
            seen[e.jb0:e.jb1, e.ib0:e.ib1] += 1
            # neighbours: W/E wrap on the periodic grid, S/N none at the poles
            assert e.nb[0] == (r - 1 if px > 0 else (r + e.npx - 1 if e.npx > 1 else -1))
            assert e.nb[3] == (r + e.npx if py < e.npy - 1 else -1)
        assert (seen == 1).all()
