"""Block ILU(0) factor handles (the MRILU seam, Ifpack_MRILU.cpp:22-39 / mrilucpp.F90):
CPU twin (oracle/ilu_oracle.c) and GPU handle (i-emic_amd/csrc/ilu.hip).

* On a block-tridiagonal matrix ILU(0) has no dropped fill, so the factorisation is the
  exact block LU and the apply solves the system: checked against numpy on the CPU and GPU.
* On the THCM Jacobian (6x6 cell blocks; point ILU(0) would meet the zero W-W / P-P
  diagonals) the GPU factor and apply equal the CPU twin's, and the factor preconditions a
  Krylov solve to 1e-8.  The reference's MRILU (multilevel ILU) is not restated: parity for
  the factor itself is against the twin ("parity unpinned" w.r.t. MRILU).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from helpers import golden_landm, mask_fix
from iemic import config as cf


def block_tridiag(nb=24, bs=6, seed=4):
    rng = np.random.default_rng(seed)
    n = nb * bs
    A = np.zeros((n, n))
    for I in range(nb):
        A[I * bs:(I + 1) * bs, I * bs:(I + 1) * bs] = rng.standard_normal((bs, bs)) + 8 * np.eye(bs)
        for J in (I - 1, I + 1):
            if 0 <= J < nb:
                A[I * bs:(I + 1) * bs, J * bs:(J + 1) * bs] = rng.standard_normal((bs, bs))
    # structurally zero diagonal entries inside the blocks (like W-W, P-P)
    for I in range(nb):
        A[I * bs + 2, I * bs + 2] = 0.0
    S = sp.csr_matrix(A)
    return S, A


def test_cpu_twin_exact_on_block_tridiagonal(oracle_lib):
    S, A = block_tridiag()
    f = oracle_lib.BlockILU(S.indptr.astype(np.int64), S.indices, S.data, 6)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    np.testing.assert_allclose(f.apply(b), np.linalg.solve(A, b), rtol=1e-10, atol=1e-12)


def make(orc, name):
    c = cf.preset(name, mixing=0)
    L = mask_fix(orc, c, golden_landm(name))
    o = orc.Oracle(c.ref_dict(), L, c.par_list())
    x = cf.synthetic_state(c, L, amp_ts=1e-3)
    val, _ = o.jacobian(x)
    return c, o, val


@pytest.mark.gpu
def test_gpu_exact_on_block_tridiagonal():
    from iemic.ilu import BlockILU
    S, A = block_tridiag()
    f = BlockILU(S.indptr.astype(np.int64), S.indices, S.data, 6)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    np.testing.assert_allclose(f.apply(b), np.linalg.solve(A, b), rtol=1e-10, atol=1e-12)
    assert f.stats() == (24, 24, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["natl8", "gateway16", "global4"])
def test_gpu_matches_cpu_twin(oracle_lib, name):
    from iemic.ilu import BlockILU
    c, o, val = make(oracle_lib, name)
    g = BlockILU(o.rowptr, o.col, val, 6)
    h = oracle_lib.BlockILU(o.rowptr, o.col, val, 6)
    r = cf.synthetic_vector(c, seed=3)
    z, zc = g.apply(r), h.apply(r)
    assert g.stats()[2] == h.perturbed      # unit-completed pivot columns (surface P rows)
    assert np.all(np.isfinite(z))
    assert np.max(np.abs(z - zc)) <= 1e-10 * np.max(np.abs(zc))


@pytest.mark.gpu
def test_gpu_ilu_preconditions_gmres(oracle_lib):
    """right-preconditioned GMRES with the GPU block ILU(0) on natl8's J reaches 1e-8"""
    from iemic.ilu import BlockILU
    c, o, val = make(oracle_lib, "natl8")
    A = sp.csr_matrix((val, o.col, o.rowptr), shape=(c.nrows, c.nrows))
    M = BlockILU(o.rowptr, o.col, val, 6)
    b = A @ cf.synthetic_vector(c, seed=5)
    m = 300
    V = np.zeros((m + 1, len(b)))
    H = np.zeros((m + 1, m))
    beta = np.linalg.norm(b)
    V[0] = b / beta
    for j in range(m):
        w = A @ M.apply(V[j])
        for _ in range(2):
            h = V[:j + 1] @ w
            w -= h @ V[:j + 1]
            H[:j + 1, j] += h
        H[j + 1, j] = np.linalg.norm(w)
        V[j + 1] = w / H[j + 1, j]
        e = np.zeros(j + 2)
        e[0] = beta
        y = np.linalg.lstsq(H[:j + 2, :j + 1], e, rcond=None)[0]
        res = np.linalg.norm(e - H[:j + 2, :j + 1] @ y) / beta
        if res <= 1e-8:
            break
    x = M.apply(y @ V[:j + 1])           # M^-1 is linear: x = M^-1 V y
    assert res <= 1e-8, (j, res)
    assert np.linalg.norm(b - A @ x) / beta <= 1e-7
