/*
 * prec.hip -- preconditioners for the FGMRES solve.
 *
 * Replaces TRIOS::BlockPreconditioner + ML/MRILU (src/trios/TRIOS_BlockPreconditioner.C,
 * src/mrilucpp) behind the Ifpack-style compute/apply seam (Ifpack_MRILU.cpp:183-377):
 *
 *   prec = 1  cell block-Jacobi: exact 6x6 inverse of every cell's diagonal block.
 *
 * (The block Gauss-Seidel variant after de Niet & Wubs is in prec_gs.hip.)
 */
#include "common.h"

namespace iemic {

int gs_compute(iemic_ctx* c, const iemic_krylov* opt);
int gs_apply(iemic_ctx* c, const double* r, double* z);

/* in-register Gauss-Jordan with partial pivoting of a 6x6 block */
__device__ __forceinline__ bool inv6(double a[6][6], double inv[6][6])
{
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) inv[i][j] = (i == j) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        int p = k;
        double best = fabs(a[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabs(a[i][k]) > best) { best = fabs(a[i][k]); p = i; }
        if (best == 0.0) return false;
        if (p != k) {
#pragma unroll
            for (int j = 0; j < 6; j++) {
                double t = a[k][j]; a[k][j] = a[p][j]; a[p][j] = t;
                t = inv[k][j]; inv[k][j] = inv[p][j]; inv[p][j] = t;
            }
        }
        const double d = 1.0 / a[k][k];
#pragma unroll
        for (int j = 0; j < 6; j++) { a[k][j] *= d; inv[k][j] *= d; }
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if (i == k) continue;
            const double f = a[i][k];
#pragma unroll
            for (int j = 0; j < 6; j++) { a[i][j] -= f * a[k][j]; inv[i][j] -= f * inv[k][j]; }
        }
    }
    return true;
}

__global__ void __launch_bounds__(128) k_bj_compute(const double* __restrict__ val, int64_t ncell,
                                                    double* __restrict__ dinv, int* __restrict__ bad)
{
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= ncell) return;
    double a[6][6], inv[6][6];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) a[i][j] = 0.0;
#pragma unroll
    for (int s = 0; s < NSLOT; s++) {
        const Slot sl = SLOTS[s];
        if (sl.di == 0 && sl.dj == 0 && sl.dk == 0) {
            int row = 0;
#pragma unroll
            for (int q = 0; q < NUN; q++)
                if (s >= ROW_BEGIN[q] && s < ROW_BEGIN[q + 1]) row = q;
            a[row][sl.var] = val[(int64_t)s * ncell + cell];
        }
    }
    if (!inv6(a, inv)) {
        /* singular pivot block (e.g. rowintcon's cell): identity */
        atomicAdd(bad, 1);
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = 0; j < 6; j++) inv[i][j] = (i == j) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) dinv[(int64_t)(i * 6 + j) * ncell + cell] = inv[i][j];
}

/* r, z: ext vectors already offset to the first owned row; dinv per owned cell */
__global__ void __launch_bounds__(256) k_bj_apply(const double* __restrict__ dinv, int64_t ncell,
                                                  const double* __restrict__ r, double* __restrict__ z)
{
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= ncell) return;
    double rv[6];
#pragma unroll
    for (int j = 0; j < 6; j++) rv[j] = r[6 * cell + j];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 6; j++) acc += dinv[(int64_t)(i * 6 + j) * ncell + cell] * rv[j];
        z[6 * cell + i] = acc;
    }
}

int prec_compute(iemic_ctx* c, const iemic_krylov* opt)
{
    if (!c->jac_valid) {
        set_error("prec_compute: no Jacobian assembled");
        return IEMIC_ESTATE;
    }
    c->gs.kind = opt ? opt->prec : 1;
    if (c->gs.kind == 2) return gs_compute(c, opt);
    if (c->gs.dinv.n < (size_t)36 * c->nloc) {
        if (c->gs.dinv.alloc((size_t)36 * c->nloc)) {
            set_error("prec_compute: out of memory");
            return IEMIC_ENOMEM;
        }
    }
    HIP_OK(hipMemsetAsync(c->d_red.p, 0, sizeof(int), c->stream));
    hipLaunchKernelGGL(k_bj_compute, dim3((unsigned)((c->nloc + 127) / 128)), dim3(128), 0, c->stream,
                       c->d_val.p, c->nloc, c->gs.dinv.p, (int*)c->d_red.p);
    HIP_OK(hipGetLastError());
    c->gs.ready = 1;
    return 0;
}

/* stagnation safeguard of the solvers: the block GS's damped correction passes diverge on
 * states where the fixed step is too long (eigenvalues of the pass near 1 - 2 omega); the
 * minimal-residual step length cannot.  Returns 1 when it switched, 0 when there is nothing
 * to switch (another preconditioner, one pass, or already minimal-residual). */
int prec_safeguard(iemic_ctx* c)
{
    BlockGS& gs = c->gs;
    if (!gs.ready || gs.kind != 2 || gs.dyn_iters < 2 || gs.dyn_mr) return 0;
    gs.dyn_mr = 1;
    return 1;
}

int prec_apply(iemic_ctx* c, const double* r, double* z)
{
    if (!c->gs.ready) {
        set_error("prec_apply: preconditioner not computed");
        return IEMIC_ESTATE;
    }
    if (c->gs.kind == 2) return gs_apply(c, r, z);
    const int64_t o = NUN * c->own0;
    hipLaunchKernelGGL(k_bj_apply, dim3((unsigned)((c->nloc + 255) / 256)), dim3(256), 0, c->stream,
                       c->gs.dinv.p, c->nloc, r + o, z + o);
    HIP_OK(hipGetLastError());
    return 0;
}

}  // namespace iemic
