/*
 * ilu.hip -- block ILU(0) factor handles on a rank-local CSR matrix: the build's
 * replacement for the reference's MRILU seam (src/mrilucpp/Ifpack_MRILU.cpp:22-39,
 * mrilucpp.F90:120-553: mrilucpp_create(id, n, nnz, beg, jco, co) / compute / apply /
 * destroy on an integer handle).  MRILU's multilevel incomplete factorisation is replaced,
 * as the north star states, by a block ILU(0) on the pattern of bs x bs blocks (bs = 6:
 * the THCM cell block (u, v, w, p, T, S), whose W-W and P-P diagonals are structurally
 * zero, so point ILU(0) breaks down while the 6x6 pivot blocks are invertible).
 *
 * Factorisation (IKJ order, no fill outside the block pattern):
 *     for I: for K < I in row I (ascending): A_IK <- A_IK D_K^-1;
 *                                           A_IJ -= A_IK A_KJ  for J > K with (I,J),(K,J) in the pattern
 *            D_I^-1 <- (A_II)^-1 (Gauss-Jordan, partial pivoting; a pivot column with no
 *            entry at all gets a unit pivot -- counted, iemic_ilu_stats)
 * Apply: (L + D)(I + D^-1 U)-form triangular solves, L unit lower: y_I = b_I - sum A_IK y_K,
 * x_I = D_I^-1 (y_I - sum_{J > I} A_IJ x_J).  Rows are processed by dependency levels
 * (level scheduling, computed on the host at create), one launch per level and one
 * wavefront per block row; within a level every row is independent.
 */
#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"

struct iemic_ilu {
    int device = 0;
    hipStream_t stream = nullptr;
    int n = 0, bs = 0, nb = 0;           /* scalar rows, block size, block rows          */
    int64_t nnzb = 0;                    /* stored blocks                                 */
    /* block CSR (columns ascending per row), blocks row-major bs x bs */
    iemic::DevBuf<int> rowptr, col, diag; /* diag: position of the diagonal block         */
    iemic::DevBuf<double> val, dinv;     /* factors in place; inverses of the pivots      */
    /* factor schedule: per block row its (IK) positions; per (IK) the (IJ, KJ) pairs    */
    iemic::DevBuf<int> ik_ptr, ik_pos, ik_k, upd_ptr, upd_ij, upd_kj;
    /* levels: rows of each level (lower-triangular dependencies; upper for the U solve) */
    std::vector<int> lev_ptr_l, lev_ptr_u;
    iemic::DevBuf<int> lev_rows_l, lev_rows_u;
    iemic::DevBuf<double> y, rb, xb;     /* apply work (scalar order)                     */
    iemic::DevBuf<int> info;
    int computed = 0;
    int perturbed = 0;                   /* pivot columns completed by a unit pivot       */
    ~iemic_ilu()
    {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace iemic {
namespace {

constexpr int BS_MAX = 8;

/* factor one level: one wavefront per block row (lanes = block entries, bs*bs <= 64) */
__global__ void __launch_bounds__(256) k_ilu_factor(const int* __restrict__ rows, int nrows, int bs,
                                                    const int* __restrict__ ik_ptr, const int* __restrict__ ik_pos,
                                                    const int* __restrict__ ik_k, const int* __restrict__ upd_ptr,
                                                    const int* __restrict__ upd_ij, const int* __restrict__ upd_kj,
                                                    const int* __restrict__ diag, double* __restrict__ val,
                                                    double* __restrict__ dinv, int* __restrict__ info)
{
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    __shared__ double sa[4][BS_MAX * BS_MAX], sb[4][BS_MAX * BS_MAX];
    const int wl = threadIdx.x >> 6;
    if (w >= nrows) return;
    const int I = rows[w];
    const int bb = bs * bs;
    const int r = lane / bs, cc = lane % bs;
    for (int q = ik_ptr[I]; q < ik_ptr[I + 1]; q++) {
        const int pos = ik_pos[q], K = ik_k[q];
        /* A_IK <- A_IK D_K^-1 */
        double* aik = val + (int64_t)pos * bb;
        const double* dk = dinv + (int64_t)K * bb;
        if (lane < bb) sa[wl][lane] = aik[lane];
        __builtin_amdgcn_wave_barrier();
        double v = 0.0;
        if (lane < bb)
            for (int t = 0; t < bs; t++) v += sa[wl][r * bs + t] * dk[t * bs + cc];
        __builtin_amdgcn_wave_barrier();
        if (lane < bb) {
            aik[lane] = v;
            sa[wl][lane] = v;
        }
        __builtin_amdgcn_wave_barrier();
        /* A_IJ -= A_IK A_KJ */
        for (int u = upd_ptr[q]; u < upd_ptr[q + 1]; u++) {
            const double* akj = val + (int64_t)upd_kj[u] * bb;
            double* aij = val + (int64_t)upd_ij[u] * bb;
            if (lane < bb) sb[wl][lane] = akj[lane];
            __builtin_amdgcn_wave_barrier();
            double s = 0.0;
            if (lane < bb)
                for (int t = 0; t < bs; t++) s += sa[wl][r * bs + t] * sb[wl][t * bs + cc];
            if (lane < bb) aij[lane] -= s;
            __builtin_amdgcn_wave_barrier();
        }
    }
    __threadfence_block();           /* the wave's stores to A_II before lane 0 reads it */
    __builtin_amdgcn_wave_barrier();
    /* D_I^-1: Gauss-Jordan with partial pivoting, lane 0 (bs <= 8) */
    if (lane == 0) {
        double a[BS_MAX * BS_MAX], x[BS_MAX * BS_MAX];
        const double* d = val + (int64_t)diag[I] * bb;
        for (int e = 0; e < bb; e++) { a[e] = d[e]; x[e] = 0.0; }
        for (int e = 0; e < bs; e++) x[e * bs + e] = 1.0;
        int zero = 0;
        for (int k = 0; k < bs; k++) {
            int p = k;
            for (int i = k + 1; i < bs; i++)
                if (fabs(a[i * bs + k]) > fabs(a[p * bs + k])) p = i;
            /* a pivot column without any entry (e.g. the continuity unknown of a surface
             * cell whose own W is an identity row): completed by a unit pivot, counted */
            if (a[p * bs + k] == 0.0) { p = k; a[k * bs + k] = 1.0; zero++; }
            if (p != k)
                for (int j = 0; j < bs; j++) {
                    double t = a[p * bs + j]; a[p * bs + j] = a[k * bs + j]; a[k * bs + j] = t;
                    t = x[p * bs + j]; x[p * bs + j] = x[k * bs + j]; x[k * bs + j] = t;
                }
            const double iv = 1.0 / a[k * bs + k];
            for (int j = 0; j < bs; j++) { a[k * bs + j] *= iv; x[k * bs + j] *= iv; }
            for (int i = 0; i < bs; i++) {
                if (i == k) continue;
                const double f = a[i * bs + k];
                if (f == 0.0) continue;
                for (int j = 0; j < bs; j++) {
                    a[i * bs + j] -= f * a[k * bs + j];
                    x[i * bs + j] -= f * x[k * bs + j];
                }
            }
        }
        if (zero) atomicAdd(info, zero);
        double* di = dinv + (int64_t)I * bb;
        for (int e = 0; e < bb; e++) di[e] = x[e];
    }
}

/* one level of the unit-lower solve y_I = b_I - sum_{K<I} A_IK y_K, or of the upper solve
 * x_I = D_I^-1 (y_I - sum_{J>I} A_IJ x_J); one wavefront per block row, lanes over
 * (block entry) with a shuffle-free LDS reduction per row of the block */
__global__ void __launch_bounds__(256) k_ilu_solve(const int* __restrict__ rows, int nrows, int bs, int upper,
                                                   const int* __restrict__ rowptr, const int* __restrict__ col,
                                                   const int* __restrict__ diag, const double* __restrict__ val,
                                                   const double* __restrict__ dinv, const double* __restrict__ rhs,
                                                   double* __restrict__ out)
{
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int wl = threadIdx.x >> 6;
    __shared__ double acc[4][64];
    __shared__ double tv[4][BS_MAX];
    if (w >= nrows) return;
    const int I = rows[w];
    const int bb = bs * bs;
    const int r = lane / bs, cc = lane % bs;
    double a = 0.0;
    const int p0 = upper ? diag[I] + 1 : rowptr[I];
    const int p1 = upper ? rowptr[I + 1] : diag[I];
    for (int p = p0; p < p1; p++) {
        const int J = col[p];
        if (lane < bb) a += val[(int64_t)p * bb + lane] * out[(int64_t)J * bs + cc];
    }
    acc[wl][lane] = lane < bb ? a : 0.0;
    __builtin_amdgcn_wave_barrier();
    if (lane < bs) {
        double s = 0.0;
        for (int t = 0; t < bs; t++) s += acc[wl][lane * bs + t];
        tv[wl][lane] = rhs[(int64_t)I * bs + lane] - s;
    }
    __builtin_amdgcn_wave_barrier();
    if (!upper) {
        if (lane < bs) out[(int64_t)I * bs + lane] = tv[wl][lane];
        return;
    }
    if (lane < bs) {
        const double* di = dinv + (int64_t)I * bb;
        double s = 0.0;
        for (int t = 0; t < bs; t++) s += di[lane * bs + t] * tv[wl][t];
        out[(int64_t)I * bs + lane] = s;
    }
    (void)r;
}

}  // namespace
}  // namespace iemic

using namespace iemic;

#define ILU_OK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));              \
            return IEMIC_EDEVICE;                                                      \
        }                                                                              \
    } while (0)

static int ilu_h2d(iemic_ilu* h, void* dst, const void* src, size_t bytes)
{
    if (!bytes) return 0;
    ILU_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream));
    ILU_OK(hipStreamSynchronize(h->stream));
    return 0;
}

/* level of every block row: 1 + the deepest row it depends on (lower: K < I, upper: J > I) */
static void levels(int nb, const std::vector<int>& rp, const std::vector<int>& cl, bool upper,
                   std::vector<int>& ptr, std::vector<int>& rows)
{
    std::vector<int> lev(nb, 0);
    int maxl = 0;
    if (!upper) {
        for (int I = 0; I < nb; I++) {
            int L = 0;
            for (int p = rp[I]; p < rp[I + 1]; p++)
                if (cl[p] < I) L = std::max(L, lev[cl[p]] + 1);
            lev[I] = L;
            maxl = std::max(maxl, L);
        }
    } else {
        for (int I = nb - 1; I >= 0; I--) {
            int L = 0;
            for (int p = rp[I]; p < rp[I + 1]; p++)
                if (cl[p] > I) L = std::max(L, lev[cl[p]] + 1);
            lev[I] = L;
            maxl = std::max(maxl, L);
        }
    }
    ptr.assign(maxl + 2, 0);
    for (int I = 0; I < nb; I++) ptr[lev[I] + 1]++;
    for (int q = 0; q <= maxl; q++) ptr[q + 1] += ptr[q];
    rows.assign(nb, 0);
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (int I = 0; I < nb; I++) rows[fill[lev[I]]++] = I;
}

extern "C" int iemic_ilu_create(iemic_ilu** out, int device, int n, int64_t nnz, const int64_t* rowptr,
                                const int* col, const double* val, int bs)
{
    if (!out || n <= 0 || !rowptr || !col || !val || bs < 1 || bs > BS_MAX || n % bs) {
        set_error("iemic_ilu_create: bad arguments (block size 1..8 dividing n)");
        return IEMIC_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("iemic_ilu_create: no HIP device");
        return IEMIC_ENODEV;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_error("iemic_ilu_create: hipSetDevice failed");
        return IEMIC_EDEVICE;
    }
    auto* h = new iemic_ilu();
    h->device = device;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        set_error("iemic_ilu_create: stream");
        return IEMIC_EDEVICE;
    }
    h->n = n;
    h->bs = bs;
    h->nb = n / bs;
    const int nb = h->nb, bb = bs * bs;
    /* block pattern (sorted), always with the diagonal block */
    std::vector<int> brp(nb + 1, 0), bcl;
    {
        std::vector<int> mark(nb, -1), tmp;
        for (int I = 0; I < nb; I++) {
            tmp.clear();
            for (int r = I * bs; r < (I + 1) * bs; r++)
                for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) {
                    const int J = col[p] / bs;
                    if (col[p] < 0 || col[p] >= n) continue;
                    if (mark[J] != I) { mark[J] = I; tmp.push_back(J); }
                }
            if (mark[I] != I) tmp.push_back(I);
            std::sort(tmp.begin(), tmp.end());
            bcl.insert(bcl.end(), tmp.begin(), tmp.end());
            brp[I + 1] = (int)bcl.size();
        }
    }
    h->nnzb = (int64_t)bcl.size();
    std::vector<int> dg(nb);
    std::vector<double> bval((size_t)h->nnzb * bb, 0.0);
    for (int I = 0; I < nb; I++) {
        for (int p = brp[I]; p < brp[I + 1]; p++)
            if (bcl[p] == I) dg[I] = p;
        for (int r = I * bs; r < (I + 1) * bs; r++)
            for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) {
                if (col[p] < 0 || col[p] >= n) continue;
                const int J = col[p] / bs;
                const int pos = (int)(std::lower_bound(bcl.begin() + brp[I], bcl.begin() + brp[I + 1], J) - bcl.begin());
                bval[(size_t)pos * bb + (r - I * bs) * bs + (col[p] - J * bs)] += val[p];
            }
    }
    /* factor schedule */
    std::vector<int> ikp(nb + 1, 0), ikpos, ikk, updp(1, 0), uij, ukj;
    for (int I = 0; I < nb; I++) {
        for (int p = brp[I]; p < dg[I]; p++) {
            const int K = bcl[p];
            ikpos.push_back(p);
            ikk.push_back(K);
            /* J > K in row I and in row K */
            int a = p + 1, b = dg[K] + 1;
            while (a < brp[I + 1] && b < brp[K + 1]) {
                if (bcl[a] < bcl[b]) a++;
                else if (bcl[a] > bcl[b]) b++;
                else { uij.push_back(a); ukj.push_back(b); a++; b++; }
            }
            updp.push_back((int)uij.size());
        }
        ikp[I + 1] = (int)ikpos.size();
    }
    std::vector<int> rows_l, rows_u;
    levels(nb, brp, bcl, false, h->lev_ptr_l, rows_l);
    levels(nb, brp, bcl, true, h->lev_ptr_u, rows_u);
    int rc = 0;
    rc |= h->rowptr.alloc(nb + 1);
    rc |= h->col.alloc(bcl.size());
    rc |= h->diag.alloc(nb);
    rc |= h->val.alloc(bval.size());
    rc |= h->dinv.alloc((size_t)nb * bb);
    rc |= h->ik_ptr.alloc(nb + 1);
    rc |= h->ik_pos.alloc(std::max<size_t>(1, ikpos.size()));
    rc |= h->ik_k.alloc(std::max<size_t>(1, ikk.size()));
    rc |= h->upd_ptr.alloc(updp.size());
    rc |= h->upd_ij.alloc(std::max<size_t>(1, uij.size()));
    rc |= h->upd_kj.alloc(std::max<size_t>(1, ukj.size()));
    rc |= h->lev_rows_l.alloc(nb);
    rc |= h->lev_rows_u.alloc(nb);
    rc |= h->y.alloc(n);
    rc |= h->rb.alloc(n);
    rc |= h->xb.alloc(n);
    rc |= h->info.alloc(1);
    if (rc) {
        delete h;
        set_error("iemic_ilu_create: out of device memory");
        return IEMIC_ENOMEM;
    }
    if ((rc = ilu_h2d(h, h->rowptr.p, brp.data(), sizeof(int) * brp.size())) ||
        (rc = ilu_h2d(h, h->col.p, bcl.data(), sizeof(int) * bcl.size())) ||
        (rc = ilu_h2d(h, h->diag.p, dg.data(), sizeof(int) * dg.size())) ||
        (rc = ilu_h2d(h, h->val.p, bval.data(), sizeof(double) * bval.size())) ||
        (rc = ilu_h2d(h, h->ik_ptr.p, ikp.data(), sizeof(int) * ikp.size())) ||
        (rc = ilu_h2d(h, h->ik_pos.p, ikpos.data(), sizeof(int) * ikpos.size())) ||
        (rc = ilu_h2d(h, h->ik_k.p, ikk.data(), sizeof(int) * ikk.size())) ||
        (rc = ilu_h2d(h, h->upd_ptr.p, updp.data(), sizeof(int) * updp.size())) ||
        (rc = ilu_h2d(h, h->upd_ij.p, uij.data(), sizeof(int) * uij.size())) ||
        (rc = ilu_h2d(h, h->upd_kj.p, ukj.data(), sizeof(int) * ukj.size())) ||
        (rc = ilu_h2d(h, h->lev_rows_l.p, rows_l.data(), sizeof(int) * nb)) ||
        (rc = ilu_h2d(h, h->lev_rows_u.p, rows_u.data(), sizeof(int) * nb))) {
        delete h;
        return rc;
    }
    *out = h;
    return 0;
}

extern "C" int iemic_ilu_compute(iemic_ilu* h)
{
    if (!h) return IEMIC_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return IEMIC_EDEVICE;
    if (h->computed) {
        set_error("iemic_ilu_compute: already factorised (mrilucpp_compute consumes the matrix)");
        return IEMIC_ESTATE;
    }
    ILU_OK(hipMemsetAsync(h->info.p, 0, sizeof(int), h->stream));
    const int nl = (int)h->lev_ptr_l.size() - 1;
    for (int q = 0; q < nl; q++) {
        const int r0 = h->lev_ptr_l[q], cnt = h->lev_ptr_l[q + 1] - r0;
        if (!cnt) continue;
        hipLaunchKernelGGL(k_ilu_factor, dim3((unsigned)((cnt + 3) / 4)), dim3(256), 0, h->stream,
                           h->lev_rows_l.p + r0, cnt, h->bs, h->ik_ptr.p, h->ik_pos.p, h->ik_k.p, h->upd_ptr.p,
                           h->upd_ij.p, h->upd_kj.p, h->diag.p, h->val.p, h->dinv.p, h->info.p);
    }
    ILU_OK(hipGetLastError());
    int info = 0;
    ILU_OK(hipMemcpyAsync(&info, h->info.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    ILU_OK(hipStreamSynchronize(h->stream));
    h->perturbed = info;
    h->computed = 1;
    return 0;
}

/* sol = (L U)^-1 rhs on device vectors (scalar order, length n) */
extern "C" int iemic_ilu_apply_dev(iemic_ilu* h, const double* rhs, double* sol)
{
    if (!h || !rhs || !sol) return IEMIC_EINVAL;
    if (!h->computed) {
        set_error("iemic_ilu_apply: not factorised");
        return IEMIC_ESTATE;
    }
    if (hipSetDevice(h->device) != hipSuccess) return IEMIC_EDEVICE;
    const int nl = (int)h->lev_ptr_l.size() - 1, nu = (int)h->lev_ptr_u.size() - 1;
    for (int q = 0; q < nl; q++) {
        const int r0 = h->lev_ptr_l[q], cnt = h->lev_ptr_l[q + 1] - r0;
        if (!cnt) continue;
        hipLaunchKernelGGL(k_ilu_solve, dim3((unsigned)((cnt + 3) / 4)), dim3(256), 0, h->stream,
                           h->lev_rows_l.p + r0, cnt, h->bs, 0, h->rowptr.p, h->col.p, h->diag.p, h->val.p,
                           h->dinv.p, rhs, h->y.p);
    }
    for (int q = 0; q < nu; q++) {
        const int r0 = h->lev_ptr_u[q], cnt = h->lev_ptr_u[q + 1] - r0;
        if (!cnt) continue;
        hipLaunchKernelGGL(k_ilu_solve, dim3((unsigned)((cnt + 3) / 4)), dim3(256), 0, h->stream,
                           h->lev_rows_u.p + r0, cnt, h->bs, 1, h->rowptr.p, h->col.p, h->diag.p, h->val.p,
                           h->dinv.p, (const double*)h->y.p, sol);
    }
    ILU_OK(hipGetLastError());
    return 0;
}

extern "C" int iemic_ilu_apply(iemic_ilu* h, const double* rhs, double* sol)
{
    if (!h || !rhs || !sol) return IEMIC_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return IEMIC_EDEVICE;
    const size_t bytes = sizeof(double) * (size_t)h->n;
    ILU_OK(hipMemcpyAsync(h->rb.p, rhs, bytes, hipMemcpyHostToDevice, h->stream));
    int rc = iemic_ilu_apply_dev(h, h->rb.p, h->xb.p);
    if (rc) return rc;
    ILU_OK(hipMemcpyAsync(sol, h->xb.p, bytes, hipMemcpyDeviceToHost, h->stream));
    ILU_OK(hipStreamSynchronize(h->stream));
    return 0;
}

extern "C" int iemic_ilu_stats(const iemic_ilu* h, int* lower, int* upper, int* perturbed)
{
    if (!h) return IEMIC_EINVAL;
    if (lower) *lower = (int)h->lev_ptr_l.size() - 1;
    if (upper) *upper = (int)h->lev_ptr_u.size() - 1;
    if (perturbed) *perturbed = h->perturbed;
    return 0;
}

extern "C" void iemic_ilu_destroy(iemic_ilu* h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    delete h;
}
