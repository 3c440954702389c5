/*
 * assembly.hip -- Jacobian, residual and forcing assembly on the device.
 *
 * Replaces the THCM Fortran assembly behind THCM::evaluate (src/ocean/THCM.C:949-1192):
 *   matrix_ (usrc.F90:432-504) + the C++ copy into the maximal graph (THCM.C:1074-1155)
 *   -> k_jacobian: one thread per (cell, equation) writes its slots of the stencil-ELL
 *   rhs_ (usrc.F90:506-586) + sign flip (THCM.C:1003) -> k_rhs: Picard coefficients are
 *   formed in registers and contracted with the state in fillcolA order (matAvec,
 *   matetc.F90:147-166); no matrix is stored.
 *   forcing (forcing.F90:4-218) -> k_forcing (+ k_qint for the flux corrections).
 * Compiled with -ffp-contract=off: values are bit-identical to the reference.
 */
#include <cmath>
#include <vector>
#include <utility>

#include "common.h"

namespace iemic {

/* Kernels run over the owned cells lc = 0 .. nloc-1 (ext cell own0 + lc); the Jacobian is
 * stored slot-major over owned cells, val[s * nloc + lc]; vectors are in the ext layout. */
template <int R>
__device__ __forceinline__ void jac_row(const Geo& g, const double* __restrict__ x, int i, int j,
                                        int k, int64_t lc, int64_t nloc, int64_t rowintcon,
                                        double* __restrict__ val)
{
    constexpr int B = RowInfo<R>::B, NS = RowInfo<R>::NS;
    double A[NS];
    bool fz;
    assemble_row<R, true>(g, x, i, j, k, A, fz);
    const bool dense_row = (NUN * (own0(g) + lc) + R) == rowintcon; /* replaced by intcond_S */
#pragma unroll
    for (int s = 0; s < NS; s++) val[(int64_t)(B + s) * nloc + lc] = dense_row ? 0.0 : A[s];
}

__global__ void __launch_bounds__(128) k_jacobian(Geo g, const double* __restrict__ x,
                                                  double* __restrict__ val, int64_t nloc,
                                                  int64_t rowintcon)
{
    const int64_t lc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lc >= nloc) return;
    int i, j, k;
    owned_cell(g, lc, i, j, k);
    switch (blockIdx.y) {
    case UU: jac_row<UU>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    case VV: jac_row<VV>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    case WW: jac_row<WW>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    case PP: jac_row<PP>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    case TT: jac_row<TT>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    default: jac_row<SS>(g, x, i, j, k, lc, nloc, rowintcon, val); break;
    }
}

/* fillcolB times Mass (THCM.C:1150-1153), B = 0 at rowintcon */
__global__ void k_diagB(Geo g, double* __restrict__ B, int64_t nloc, int64_t rowintcon)
{
    const int64_t lc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lc >= nloc) return;
    int i, j, k;
    owned_cell(g, lc, i, j, k);
    double b[NUN];
    diagB_cell(g, i, j, k, b);
    const int64_t cell = own0(g) + lc;
    for (int v = 0; v < NUN; v++) {
        const int64_t row = NUN * cell + v;
        B[row] = (row == rowintcon) ? 0.0 : b[v];
    }
}

__global__ void __launch_bounds__(128) k_rhs(Geo g, const double* __restrict__ x,
                                             const double* __restrict__ frc,
                                             double* __restrict__ F, int64_t nloc)
{
    const int64_t lc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lc >= nloc) return;
    int i, j, k;
    owned_cell(g, lc, i, j, k);
    const int64_t cell = own0(g) + lc;
    double f;
    switch (blockIdx.y) {
    case UU: f = rhs_row_value<UU>(g, x, frc, i, j, k, cell); break;
    case VV: f = rhs_row_value<VV>(g, x, frc, i, j, k, cell); break;
    case WW: f = rhs_row_value<WW>(g, x, frc, i, j, k, cell); break;
    case PP: f = rhs_row_value<PP>(g, x, frc, i, j, k, cell); break;
    case TT: f = rhs_row_value<TT>(g, x, frc, i, j, k, cell); break;
    default: f = rhs_row_value<SS>(g, x, frc, i, j, k, cell); break;
    }
    F[NUN * cell + blockIdx.y] = f;
}

/* deterministic block partial sums of a*b (for the intcond dot) */
__global__ void k_dot_partial(const double* __restrict__ a, const double* __restrict__ b,
                              int64_t n, double* __restrict__ part)
{
    __shared__ double sm[256];
    double s = 0.0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
         q += (int64_t)gridDim.x * blockDim.x)
        s += a[q] * b[q];
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) sm[threadIdx.x] += sm[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}
/* out = sum of the block partials (fixed order) */
__global__ void k_sum_partials(const double* __restrict__ part, int nb, double* __restrict__ out)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double s = 0.0;
        for (int q = 0; q < nb; q++) s += part[q];
        *out = s;
    }
}
/* F[rowintcon] = intSign*(coeff . x - intCorrection)  (THCM.C:1005-1018) */
__global__ void k_intcond_set(const double* __restrict__ dotv, double* __restrict__ F, int64_t row,
                              int sign, double corr)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) F[row] = sign * (*dotv - corr);
}

__global__ void k_qint(Geo g, const double* __restrict__ ftab, double* __restrict__ qcor,
                       int need_t, int need_s)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    forcing_qint(g, ftab, qcor, need_t, need_s);
}

__global__ void k_forcing(Geo g, const double* __restrict__ ftab, const double* __restrict__ qcor,
                          double* __restrict__ frc, int64_t nloc)
{
    const int64_t lc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lc >= nloc) return;
    int i, j, k;
    owned_cell(g, lc, i, j, k);
    const int64_t cell = own0(g) + lc;
    double f[NUN];
    forcing_cell(g, ftab, qcor, i, j, k, f);
    for (int v = 0; v < NUN; v++) frc[NUN * cell + v] = f[v];
}

/* block partials of sum T^2 and sum S^2 over the owned cells (fixed order) */
__global__ void __launch_bounds__(256) k_ts_sq_partial(const double* __restrict__ x, int64_t own0,
                                                       int64_t nloc, double* __restrict__ part)
{
    __shared__ double sm[2][256];
    double st = 0.0, ss = 0.0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nloc;
         q += (int64_t)gridDim.x * blockDim.x) {
        const double t = x[NUN * (own0 + q) + TT], sv = x[NUN * (own0 + q) + SS];
        st += t * t;
        ss += sv * sv;
    }
    sm[0][threadIdx.x] = st;
    sm[1][threadIdx.x] = ss;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            sm[0][threadIdx.x] += sm[0][threadIdx.x + w];
            sm[1][threadIdx.x] += sm[1][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[blockIdx.x] = sm[0][0];
        part[gridDim.x + blockIdx.x] = sm[1][0];
    }
}

/* ------------------------------------------------------------------------------------ */
/* vmix_control (mix_imp.f:131-166) for Mixing = 2: the Ocean layer calls fixMixing(0)
 * before every evaluation (Ocean.C:1271/1292), so whether T and S mix (L2 norm of the
 * field > 1e-12, summed over the bands) is re-decided at each call; and the restated
 * subset of vmix_fun must cover the current parameters */
static int mix_control(iemic_ctx* c, const double* x_dev)
{
    host::Setup& su = c->su;
    if (su.cfg.vmix == 0) return 0;
    if (su.cfg.vmix == 2) {   /* Ocean.C:1271/1292: fixMixing(0) before every evaluation */
        /* squared field norms on the device (block partials + fixed-order sums), summed
         * over the bands; only the two totals come to the host */
        const int nb = 256;
        double* part = c->d_red.p;
        hipLaunchKernelGGL(k_ts_sq_partial, dim3(nb), dim3(256), 0, c->stream, x_dev, (int64_t)c->own0,
                           (int64_t)c->nloc, part);
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, c->stream, part, nb, part + 2 * nb);
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, c->stream, part + nb, nb, part + 2 * nb + 1);
        int rc = allreduce_sum(c, part + 2 * nb, 2);
        if (rc) return rc;
        double sq[2] = {0.0, 0.0};
        if ((rc = d2h(c, sq, part + 2 * nb, sizeof(sq)))) return rc;
        su.vmix_t = std::sqrt(sq[0]) > 1.0e-12;
        su.vmix_s = std::sqrt(sq[1]) > 1.0e-12;
        /* vmix_control partitions only when T mixes (mix_imp.f:158): salinity-only mixing
         * stays off; temperature-only mixing (zero salinity field) is not restated */
        if (!su.vmix_t) su.vmix_s = 0;
        su.vmix_fix = 1;
        if (su.vmix_t && !su.vmix_s) {
            set_error("Mixing = 2 with a zero salinity field is not supported");
            return IEMIC_EINVAL;
        }
    }
    if ((su.vmix_t || su.vmix_s) && !su.vmix_supported()) {
        set_error("vertical mixing: neutral physics / Gent-McWilliams / energetically consistent "
                  "mixing (MIXP, MKAP != 0 or ALPC != 1) are not restated");
        return IEMIC_EINVAL;
    }
    return 0;
}

int assemble_jacobian(iemic_ctx* c, const double* x_dev)
{
    int rc = mix_control(c, x_dev);
    if (rc) return rc;
    BlockGS& gs = c->gs;
    if (gs.ready && gs.kind == 2) {
        /* the block GS reads its set-up Jacobian (BlockGS::vp): assemble into the other buffer */
        if (gs.vp == c->d_val.p) {
            if (gs.vold.n != c->d_val.n && gs.vold.alloc(c->d_val.n)) {
                set_error("assemble_jacobian: out of device memory for the second Jacobian buffer");
                return IEMIC_ENOMEM;
            }
            std::swap(c->d_val, gs.vold);
        }
        gs.coef_stale = 1;
    }
    Geo g = c->geo();
    dim3 blk(128), grd((unsigned)((c->nloc + 127) / 128), NUN);
    hipLaunchKernelGGL(k_jacobian, grd, blk, 0, c->stream, g, x_dev, c->d_val.p, c->nloc,
                       (int64_t)c->rowintcon);
    hipLaunchKernelGGL(k_diagB, dim3((unsigned)((c->nloc + 255) / 256)), dim3(256), 0, c->stream,
                       g, c->d_B.p, c->nloc, (int64_t)c->rowintcon);
    HIP_OK(hipGetLastError());
    c->jac_valid = 1;
    return 0;
}

int assemble_rhs(iemic_ctx* c, const double* x_dev, double* F_dev)
{
    int rc0 = mix_control(c, x_dev);
    if (rc0) return rc0;
    Geo g = c->geo();
    dim3 blk(128), grd((unsigned)((c->nloc + 127) / 128), NUN);
    hipLaunchKernelGGL(k_rhs, grd, blk, 0, c->stream, g, x_dev, c->d_frc.p, F_dev, c->nloc);
    if (c->su.rowintcon_ref >= 0) {
        /* the integral condition couples every S unknown: owned partial dot, a sum over the
         * ranks, and the owning rank writes the entry */
        const int nb = 256;
        const int64_t o = NUN * c->own0;
        hipLaunchKernelGGL(k_dot_partial, dim3(nb), dim3(256), 0, c->stream, c->d_intc.p + o,
                           x_dev + o, c->nlrows, c->d_red.p);
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, c->stream, c->d_red.p, nb,
                           c->d_red.p + nb);
        int rc = allreduce_sum(c, c->d_red.p + nb, 1);
        if (rc) return rc;
        if (c->rowintcon >= 0)
            hipLaunchKernelGGL(k_intcond_set, dim3(1), dim3(64), 0, c->stream, c->d_red.p + nb, F_dev,
                               (int64_t)c->rowintcon, c->cfg.int_sign, c->int_correction);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

/* THCM::setIntCondCorrection (THCM.C:2020-2038): intCorrection = coeff . x (SRES = 0) */
int intcond_correction(iemic_ctx* c, const double* x_dev)
{
    if (c->su.rowintcon_ref < 0) {
        c->int_correction = 0.0;
        return 0;
    }
    const int nb = 256;
    const int64_t o = NUN * c->own0;
    hipLaunchKernelGGL(k_dot_partial, dim3(nb), dim3(256), 0, c->stream, c->d_intc.p + o, x_dev + o, c->nlrows,
                       c->d_red.p);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(64), 0, c->stream, c->d_red.p, nb, c->d_red.p + nb);
    int rc = allreduce_sum(c, c->d_red.p + nb, 1);
    if (rc) return rc;
    return d2h(c, &c->int_correction, c->d_red.p + nb, sizeof(double));
}

int compute_forcing(iemic_ctx* c)
{
    Geo g = c->geo();
    hipLaunchKernelGGL(k_qint, dim3(1), dim3(64), 0, c->stream, g, c->d_ftab.p, c->d_qcor.p,
                       c->cfg.tres == 0 ? 1 : 0, c->cfg.sres == 0 ? 1 : 0);
    hipLaunchKernelGGL(k_forcing, dim3((unsigned)((c->nloc + 255) / 256)), dim3(256), 0,
                       c->stream, g, c->d_ftab.p, c->d_qcor.p, c->d_frc.p, c->nloc);
    HIP_OK(hipGetLastError());
    return 0;
}

}  // namespace iemic
