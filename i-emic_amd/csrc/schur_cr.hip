/*
 * schur_cr.hip -- exact solve of the 2-D (barotropic) Schur complement of the block
 * Gauss-Seidel preconditioner by block cyclic reduction over longitudes.
 *
 * The pinned Schur matrix S (prec_gs.hip, step 3; the depth-averaged pressure problem that
 * TRIOS::BlockPreconditioner solves iteratively with AztecOO/ML, TRIOS_BlockPreconditioner.C:
 * 1479-1611 SolveLower1 and 2113-2173 Compute) couples water column (i, j) only to
 * (i+di, j+dj), |di|, |dj| <= 1.  Numbered c = i*m + j it is block tridiagonal in i with
 * m x m blocks (periodic in i for a periodic grid):
 *     L_i x_{i-1} + D_i x_i + R_i x_{i+1} = b_i .
 * Cyclic reduction eliminates the odd blocks of every level,
 *     D'_e = D_e - L_e D_{e-1}^-1 R_{e-1} - R_e D_{e+1}^-1 L_{e+1},
 *     L'_e = -L_e D_{e-1}^-1 L_{e-1},  R'_e = -R_e D_{e+1}^-1 R_{e+1},
 * halving the block count per level (ceil(log2 n) levels, a direct coupling kept where an
 * odd count leaves two even blocks adjacent across the periodic wrap, the two couplings of
 * a periodic pair merged), down to one m x m block.  Set-up per level: one Gauss-Jordan
 * inverse per odd block (one workgroup each) and two batched GEMM launches; the apply is one
 * GEMV launch per level down and one per level up.  The deepest levels (the first level of
 * at most 1024 unknowns and below) form a dense tail: its explicit inverse is built at set-up
 * by running those levels on the identity, and the apply replaces their 2 (nlev - lt) + 1
 * launches with one GEMV (9 -> 1 at 2 degrees).  Cost: O(n m^3) set-up flops spread over
 * n/2 workgroups per level and O(n m^2) apply bytes -- against the O(ncol^2) dense inverse
 * and the single-workgroup band LU it replaces.  Land columns are identity rows; pivoting
 * happens inside the diagonal blocks only (tested against the band LU with partial
 * pivoting of the CPU twin, oracle/prec_oracle.c).
 *
 * Every m x m block is stored column-major: a(r, c) at [r + c*m].
 */
#include <algorithm>
#include <map>
#include <tuple>
#include <vector>

#include "common.h"

namespace iemic {

namespace {

constexpr int CR_MAXM = 512;

/* level-0 blocks from the 9-point rows S9[c*9 + (dj+1)*3 + (di+1)], c = i*m + j; inactive
 * columns (no water) become identity rows.  One thread per row (i, j): no write races. */
__global__ void k_cr_expand(const double* __restrict__ S9, const int* __restrict__ col_of_ij, int n,
                            int m, int periodic, double* __restrict__ D, double* __restrict__ Lb,
                            double* __restrict__ Rb)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n * m) return;
    const int i = c / m, j = c % m;
    const size_t mm = (size_t)m * m;
    double* Di = D + (size_t)i * mm;
    if (col_of_ij[j * n + i] < 0) {
        Di[j + (size_t)j * m] = 1.0;
        return;
    }
    for (int o = 0; o < 9; o++) {
        const double v = S9[(size_t)c * 9 + o];
        if (v == 0.0) continue;
        const int di = o % 3 - 1, dj = o / 3 - 1;
        int ti = i + di;
        const int tj = j + dj;
        if (tj < 0 || tj >= m) continue;
        if (ti < 0 || ti >= n) {
            if (!periodic) continue;
            ti = (ti + n) % n;
        }
        double* B = ti == i ? Di : (di < 0 ? Lb + (size_t)i * mm : Rb + (size_t)i * mm);
        B[j + (size_t)tj * m] += v;
    }
}

/* Gauss-Jordan inverse with partial pivoting of src block (s0 + blockIdx.x * sstep) into
 * dst block blockIdx.x (m x m column-major, m <= TR RA, m <= 32 RB), in place in registers:
 * 32 TR threads as a TR x 32 grid, thread (tr, tc) holds rows tr + TR x and columns
 * tc + 32 y.  Rows are never swapped: step k takes the unused row p with the largest
 * |a(p, k)|, scales it, eliminates column k from every other row, and column k -- dead in
 * the eliminated matrix -- keeps column p of the inverse's row-permuted form (the in-place
 * trick), so the result is written out through the two permutations (row p_k of the
 * storage is row k of the inverse, storage column k is its column p_k).  The step loop is
 * unrolled over blocks of TR steps, so the register column of k is a compile-time index;
 * the pivot row's register row is selected under a branch on its row lane.
 * One barrier per step (round 6; two before): the owners of column k + 1 write it to LDS and
 * search its pivot right after their step-k update, and every thread takes the pivot row's
 * entries of its own columns from the lane of thread (p's row lane, its column lane) -- the
 * threads of one column lane are TR consecutive lanes of one wave -- by a cross-lane read
 * instead of a second LDS round.  Same operations in the same order: the inverse is bitwise
 * the two-barrier kernel's.  A zero pivot sets *info. */
template <int TR, int RA, int RB>
__device__ __forceinline__ void cr_inv_pivot(const double* cv, unsigned used, int m, int k, int tr,
                                             double* __restrict__ pcol, int* __restrict__ s_p,
                                             int* __restrict__ piv_row, int* __restrict__ step_of,
                                             int* __restrict__ info)
{
    double best = -1.0;
    int bi = m;
#pragma unroll
    for (int x = 0; x < RA; x++) {
        const int i = tr + TR * x;
        const double v = cv[x];
        if (i < m) pcol[i] = v;
        /* a NaN candidate counts as 0, so some unused row is always taken and step_of /
         * piv_row stay a permutation (the zero pivot sets *info) */
        const double av = (i < m && !((used >> x) & 1u)) ? (v == v ? fabs(v) : 0.0) : -1.0;
        if (av > best) { best = av; bi = i; }
    }
#pragma unroll
    for (int o = 1; o < TR; o <<= 1) {
        const double ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (tr == 0) {
        if (!(best > 0.0)) *info = 1;
        *s_p = bi;
        piv_row[k] = bi;
        step_of[bi < m ? bi : 0] = k;
    }
}

template <int TR, int RA, int RB>
__global__ void __launch_bounds__(32 * TR) k_cr_inv(const double* __restrict__ src, int s0, int sstep,
                                                     double* __restrict__ dst, int m, int* __restrict__ info)
{
    const size_t mm = (size_t)m * m;
    const double* A = src + (size_t)(s0 + blockIdx.x * sstep) * mm;
    double* X = dst + (size_t)blockIdx.x * mm;
    const int t = threadIdx.x, tr = t % TR, tc = t / TR;
    const int lbase = (t & 63) - tr;                    /* lane of thread (0, tc) in this wave */
    __shared__ double pcol[2][TR * RA];
    __shared__ int s_p[2];
    __shared__ int piv_row[TR * RA], step_of[TR * RA];
    double a[RA][RB];
#pragma unroll
    for (int x = 0; x < RA; x++)
#pragma unroll
        for (int y = 0; y < RB; y++) {
            const int i = tr + TR * x, j = tc + 32 * y;
            a[x][y] = (i < m && j < m) ? A[i + (size_t)j * m] : 0.0;
        }
    unsigned used = 0;                                 /* bit x: row tr + TR x was a pivot */
    if (tc == 0) {                                     /* column 0: LDS and its pivot */
        double cv[RA];
#pragma unroll
        for (int x = 0; x < RA; x++) cv[x] = a[x][0];
        cr_inv_pivot<TR, RA, RB>(cv, used, m, 0, tr, pcol[0], &s_p[0], piv_row, step_of, info);
    }
#pragma unroll
    for (int kbr = 0; kbr < RA; kbr++) {
        const int yk = kbr * TR / 32;                   /* register column of k (compile time) */
        const int ykn = ((kbr + 1) * TR / 32) < RB ? (kbr + 1) * TR / 32 : RB - 1;   /* of the next block's first */
        for (int kk = 0; kk < TR; kk++) {
            const int k = kbr * TR + kk;
            if (k >= m) break;
            const int sel = k & 1, kc = k & 31;
            __syncthreads();                            /* column k and its pivot in LDS */
            const int p = __builtin_amdgcn_readfirstlane(s_p[sel]);
            const int pr = p % TR, pa = p / TR;
            if (tr == pr) used |= 1u << pa;
            /* the pivot row's entries of this thread's columns: thread (pr, tc)'s registers */
            double prw[RB];
#pragma unroll
            for (int y = 0; y < RB; y++) {
                double mine = a[0][y];
#pragma unroll
                for (int x = 1; x < RA; x++)
                    if (x == pa) mine = a[x][y];
                prw[y] = __shfl(mine, lbase + pr, 64);
            }
            /* scale row p, eliminate column k from the other rows; column k keeps the
             * inverse's column (1 / piv in row p, -a(i, k) / piv elsewhere) */
            const double piv = pcol[sel][p];
            const double inv = piv != 0.0 ? 1.0 / piv : 0.0;
            double pr_s[RB];
#pragma unroll
            for (int y = 0; y < RB; y++) {
                const int j = tc + 32 * y;
                pr_s[y] = j < m ? prw[y] * inv : 0.0;
            }
            const bool colk = tc == kc;
#pragma unroll
            for (int x = 0; x < RA; x++) {
                const int i = tr + TR * x;
                const double f = i < m ? pcol[sel][i] : 0.0;
#pragma unroll
                for (int y = 0; y < RB; y++) {
                    if (y == yk && colk) a[x][y] = -f * inv;
                    else a[x][y] -= f * pr_s[y];
                }
            }
            if (tr == pr) {
#pragma unroll
                for (int x = 0; x < RA; x++)
                    if (x == pa)
#pragma unroll
                        for (int y = 0; y < RB; y++) a[x][y] = (y == yk && colk) ? inv : pr_s[y];
            }
            /* column k + 1 (updated above) to LDS and its pivot, by its owners */
            if (k + 1 < m && tc == ((k + 1) & 31)) {
                double cv[RA];
#pragma unroll
                for (int x = 0; x < RA; x++) cv[x] = kk + 1 < TR ? a[x][yk] : a[x][ykn];
                cr_inv_pivot<TR, RA, RB>(cv, used, m, k + 1, tr, pcol[sel ^ 1], &s_p[sel ^ 1], piv_row,
                                         step_of, info);
            }
        }
    }
    __syncthreads();
    /* storage (i, k) = inverse (step_of[i], piv_row[k]) */
#pragma unroll
    for (int x = 0; x < RA; x++)
#pragma unroll
        for (int y = 0; y < RB; y++) {
            const int i = tr + TR * x, j = tc + 32 * y;
            if (i < m && j < m) X[step_of[i] + (size_t)piv_row[j] * m] = a[x][y];
        }
}

/* C = C0 + C0b + s1 A1 B1 + s2 A2 B2 for a batch of m x m column-major blocks: one 32x32
 * tile of one descriptor per workgroup (blockIdx.y = descriptor) */
__global__ void __launch_bounds__(256) k_cr_gemm(const CrGemm* __restrict__ dd, int m)
{
    const CrGemm d = dd[blockIdx.y];
    const int T = (m + 31) / 32;
    const int r0 = (blockIdx.x % T) * 32, c0 = (blockIdx.x / T) * 32;
    const int t = threadIdx.x, tr = t & 31, tc = t >> 5;
    __shared__ double As[32][33], Bs[32][33];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int prod = 0; prod < 2; prod++) {
        const double* A = prod ? d.A2 : d.A1;
        const double* B = prod ? d.B2 : d.B1;
        if (!A) continue;
        const double s = prod ? d.s2 : d.s1;
        double pa[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < m; k0 += 32) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int e = t + 256 * q;
                const int rr = e & 31, kk = e >> 5;
                As[kk][rr] = (r0 + rr < m && k0 + kk < m) ? A[(r0 + rr) + (size_t)(k0 + kk) * m] : 0.0;
                const int kb = e & 31, cc = e >> 5;
                Bs[cc][kb] = (k0 + kb < m && c0 + cc < m) ? B[(k0 + kb) + (size_t)(c0 + cc) * m] : 0.0;
            }
            __syncthreads();
#pragma unroll 8
            for (int kk = 0; kk < 32; kk++) {
                const double a = As[kk][tr];
#pragma unroll
                for (int q = 0; q < 4; q++) pa[q] += a * Bs[tc + 8 * q][kk];
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < 4; q++) acc[q] += s * pa[q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = r0 + tr, c = c0 + tc + 8 * q;
        if (r >= m || c >= m) continue;
        const size_t idx = r + (size_t)c * m;
        double v = acc[q];
        if (d.C0) v += d.C0[idx];
        if (d.C0b) v += d.C0b[idx];
        d.C[idx] = v;
    }
}

/* Rows [r0, r0 + CR_RC) of y = y0 + s0 (A0 v0 + A1 v1 + A2 v2) for m x m column-major
 * blocks (m <= CR_RC * CR_CPT): thread = (row, column group), CR_RC rows x CR_G groups,
 * each thread CR_CPT columns per block.  The block entries are loaded into registers BEFORE
 * the vectors arrive in LDS (crf_load, then the caller's vector loads and barrier, then
 * crf_finish), so both memory latencies overlap; the groups' partial sums are added in LDS
 * in a fixed order (deterministic). */
constexpr int CR_RC = 16, CR_G = 256 / CR_RC, CR_CPT = 12;
struct CrFrag {
    double a[3][CR_CPT];
};
__device__ __forceinline__ void crf_load(CrFrag& f, const double* __restrict__ A0, const double* __restrict__ A1,
                                         const double* __restrict__ A2, int m, int r0)
{
    const int t = threadIdx.x, g = t / CR_RC, r = r0 + t % CR_RC;
    const double* A[3] = {A0, A1, A2};
#pragma unroll
    for (int q = 0; q < 3; q++)
#pragma unroll
        for (int u = 0; u < CR_CPT; u++) {
            const int c = g + CR_G * u;
            f.a[q][u] = (A[q] && r < m && c < m) ? A[q][r + (size_t)c * m] : 0.0;
        }
}
__device__ __forceinline__ void crf_finish(const CrFrag& f, const double* v0, const double* v1, const double* v2,
                                           double s0, const double* __restrict__ y0, double* __restrict__ y,
                                           int m, int r0, double* red)
{
    const int t = threadIdx.x, g = t / CR_RC, r = r0 + t % CR_RC;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int u = 0; u < CR_CPT; u++) {
        const int c = g + CR_G * u;
        if (c < m) {
            a0 += f.a[0][u] * v0[c];
            a1 += f.a[1][u] * v1[c];
            a2 += f.a[2][u] * v2[c];
        }
    }
    red[t] = (a0 + a1) + a2;
    __syncthreads();
    if (t < CR_RC && r < m) {
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < CR_G; q++) sum += red[q * CR_RC + t];
        y[r] = (y0 ? y0[r] : 0.0) + s0 * sum;
    }
}

/* Set-up (batched right-hand sides: the tail's inverse is built by solving for the
 * identity): each workgroup keeps its row chunk of the level operators in registers and runs
 * CR_RB right-hand sides (blockIdx.y groups), so the blocks are read once per CR_RB columns
 * instead of once per column. */
constexpr int CR_RB = 8;

/* level down, one row chunk of one even block per workgroup (blockIdx.x = q * nch + chunk):
 * b'_q = b_e - XL_q b_{e-1} - XR_q b_{e+1} (odd neighbours only), e = 2q */
__global__ void __launch_bounds__(256) k_cr_fwd(const double* __restrict__ bl, double* __restrict__ bn,
                                                const double* __restrict__ XL, const double* __restrict__ XR,
                                                int N, int per, int m, int nch, int64_t sl, int64_t sn, int nrhs)
{
    __shared__ double vl[CR_MAXM], vr[CR_MAXM], red[256];
    const int q = blockIdx.x / nch, r0 = (blockIdx.x % nch) * CR_RC, e = 2 * q;
    const bool lex = e > 0 || per, rex = e + 1 < N || per;
    const int lnb = e > 0 ? e - 1 : N - 1, rnb = (e + 1) % N;
    const bool lo = lex && (lnb & 1), ro = rex && (rnb & 1);
    const size_t mm = (size_t)m * m;
    CrFrag f;
    crf_load(f, lo ? XL + q * mm : nullptr, ro ? XR + q * mm : nullptr, nullptr, m, r0);
    const int r1 = min(nrhs, (int)(blockIdx.y + 1) * CR_RB);
    for (int rh = blockIdx.y * CR_RB; rh < r1; rh++) {
        const double* b = bl + rh * sl;
        for (int c = threadIdx.x; c < m; c += 256) {
            vl[c] = lo ? b[(size_t)lnb * m + c] : 0.0;
            vr[c] = ro ? b[(size_t)rnb * m + c] : 0.0;
        }
        __syncthreads();
        crf_finish(f, vl, vr, vl, -1.0, b + (size_t)e * m, bn + rh * sn + (size_t)q * m, m, r0, red);
    }
}

/* level up, one row chunk of one odd block per workgroup (blockIdx.x = p * nch + chunk):
 * x_o = Dinv b_o - YL x_{o-1} - YR x_{o+1}, o = 2p + 1; the even blocks are copied from
 * the level below (x_{o-1} by block o, the last even block of an odd count by block N-2) */
__global__ void __launch_bounds__(256) k_cr_bwd(const double* __restrict__ bl, const double* __restrict__ xn,
                                                double* __restrict__ xl, const double* __restrict__ Dinv,
                                                const double* __restrict__ YL, const double* __restrict__ YR,
                                                int N, int per, int m, int nch, int64_t sl, int64_t sn, int nrhs)
{
    __shared__ double vb[CR_MAXM], vl[CR_MAXM], vr[CR_MAXM], red[256];
    const int p = blockIdx.x / nch, r0 = (blockIdx.x % nch) * CR_RC, b = 2 * p + 1;
    const bool rex = b + 1 < N || per;
    const int rn = (b + 1) % N;
    const size_t mm = (size_t)m * m;
    CrFrag f;
    crf_load(f, Dinv + p * mm, YL + p * mm, rex ? YR + p * mm : nullptr, m, r0);
    const int r1 = min(nrhs, (int)(blockIdx.y + 1) * CR_RB);
    for (int rh = blockIdx.y * CR_RB; rh < r1; rh++) {
        const double* bq = bl + rh * sl;
        const double* xq = xn + rh * sn;
        double* xo = xl + rh * sl;
        for (int c = threadIdx.x; c < m; c += 256) {
            vb[c] = bq[(size_t)b * m + c];
            vl[c] = -xq[(size_t)p * m + c];
            vr[c] = rex ? -xq[(size_t)(rn / 2) * m + c] : 0.0;
        }
        if (threadIdx.x < CR_RC && r0 + threadIdx.x < m) {
            const int r = r0 + threadIdx.x;
            xo[(size_t)(b - 1) * m + r] = xq[(size_t)p * m + r];
            if (b == N - 2) xo[(size_t)(N - 1) * m + r] = xq[(size_t)((N - 1) / 2) * m + r];
        }
        __syncthreads();
        crf_finish(f, vb, vl, vr, 1.0, nullptr, xo + (size_t)b * m, m, r0, red);
    }
}

/* the last level: x = Dfin b, one row chunk per workgroup */
__global__ void __launch_bounds__(256) k_cr_final(const double* __restrict__ Dfin, const double* __restrict__ b,
                                                  double* __restrict__ x, int m, int nrhs)
{
    __shared__ double vb[CR_MAXM], red[256];
    CrFrag f;
    crf_load(f, Dfin, nullptr, nullptr, m, blockIdx.x * CR_RC);
    const int r1 = min(nrhs, (int)(blockIdx.y + 1) * CR_RB);
    for (int rh = blockIdx.y * CR_RB; rh < r1; rh++) {
        for (int c = threadIdx.x; c < m; c += 256) vb[c] = b[(size_t)rh * m + c];
        __syncthreads();
        crf_finish(f, vb, vb, vb, 1.0, nullptr, x + (size_t)rh * m, m, blockIdx.x * CR_RC, red);
    }
}


/* dense tail, set-up: the identity as tM right-hand sides of the tail's first level */
__global__ void k_cr_eye(double* __restrict__ B, int M)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < (int64_t)M * M) B[e] = (e / M == e % M) ? 1.0 : 0.0;
}

/* T = X^T for the M x M column-major X (32 x 32 tiles through LDS) */
__global__ void k_cr_transpose(const double* __restrict__ X, double* __restrict__ T, int M)
{
    __shared__ double t[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int y = ty; y < 32; y += 8)
        if (r0 + tx < M && c0 + y < M) t[y][tx] = X[(r0 + tx) + (size_t)(c0 + y) * M];
    __syncthreads();
    for (int y = ty; y < 32; y += 8)
        if (c0 + tx < M && r0 + y < M) T[(r0 + y) * (size_t)M + c0 + tx] = t[tx][y];
}

/* dense tail, apply: x = Tinv b (row-major, M <= CR_TAIL_MAX), one wave per row, b staged
 * in LDS; every load of the row is issued before the first multiply (up to 32 per lane,
 * eight independent accumulators), then a fixed shuffle tree (deterministic) */
constexpr int CR_TAIL_MAX = 1024;          /* cr_init: tail_max */
__global__ void __launch_bounds__(256) k_cr_tail(const double* __restrict__ Tinv, const double* __restrict__ b,
                                                 double* __restrict__ x, int M, double* __restrict__ xT, int nT, int m)
{
    __shared__ double vb[CR_TAIL_MAX];
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const double* A = Tinv + (size_t)(r < M ? r : 0) * M;
    constexpr int NL = CR_TAIL_MAX / 64;
    double a[NL];
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int c = lane + 64 * u;
        a[u] = c < M ? A[c] : 0.0;
    }
    for (int c = threadIdx.x; c < M; c += 256) vb[c] = b[c];
    __syncthreads();
    if (r >= M) return;
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int c = lane + 64 * u;
        if (c < M) acc[u & 7] += a[u] * vb[c];
    }
    double v = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) {
        x[r] = v;
        if (xT) xT[(int64_t)(r % m) * nT + r / m] = v;   /* a tail holding the whole problem */
    }
}

/* Apply step (packed, CrStep): workgroup w computes rows [r0, r0 + RC) of one output block,
 * y = sum_t A_t v_t (+ v_id), its nA scaled matrix terms read from its own run of P
 * (term, column, row; thread = (row, column group) with the row fastest; default load
 * policy: non-temporal loads measured 44 against 39 us per solve).  The class
 * bounds are kernel arguments, so the matrix loads are issued before the vector references
 * arrive; the vectors are staged in LDS meanwhile.  Per row the column groups' partial sums
 * meet by a fixed shuffle tree inside each wave and in LDS across the four waves
 * (deterministic). */
template <int RC, int CPT>
__global__ void __launch_bounds__(256) k_cr_pk(const double* __restrict__ P, const CrCls cls,
                                               const CrWg* __restrict__ wgs, int m, const double* __restrict__ b,
                                               double* __restrict__ x, double* __restrict__ bv,
                                               double* __restrict__ xv, double* __restrict__ xT, int nT)
{
    constexpr int G = 256 / RC;
    __shared__ double vs[CR_MT + 1][192];          /* m <= 192 (cr_init) */
    __shared__ double red[4][RC];
    const int w = blockIdx.x;
    int k = 0;
#pragma unroll
    for (int q = 1; q < CR_NCLS; q++)
        if (q < cls.ncls && w >= cls.w0[q]) k = q;
    const int nA = cls.nA[k];
    const double* __restrict__ Pw = P + cls.p0[k] + (int64_t)(w - cls.w0[k]) * nA * m * RC;
    const int t = threadIdx.x, g = t / RC, rr = t % RC;
    double a[CR_MT][CPT];
#pragma unroll
    for (int q = 0; q < CR_MT; q++)
#pragma unroll
        for (int u = 0; u < CPT; u++) {
            const int c = g + G * u;
            a[q][u] = (q < nA && c < m) ? Pw[((int64_t)q * m + c) * RC + rr] : 0.0;
        }
    const CrWg& d = wgs[w];
    const int nv = d.nv;
    const double* base[4] = {b, x, bv, xv};
    {
        /* (vector, element) pairs dealt over the lanes, all loads before the first store */
        constexpr int SPT = ((CR_MT + 1) * 192 + 255) / 256;
        const int tot = nv * m;
        double v[SPT];
        int qv[SPT], cv[SPT], refs[CR_MT];
#pragma unroll
        for (int q = 0; q < CR_MT; q++) refs[q] = d.vref[q];
#pragma unroll
        for (int i = 0; i < SPT; i++) {
            const int e = t + 256 * i;
            qv[i] = e < tot ? e / m : 0;
            cv[i] = e < tot ? e - qv[i] * m : -1;
            int ref = refs[0];
#pragma unroll
            for (int q = 1; q < CR_MT; q++)
                if (qv[i] == q) ref = refs[q];
            v[i] = cv[i] >= 0 ? base[ref >> 28][(ref & 0x0fffffff) + cv[i]] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < SPT; i++)
            if (cv[i] >= 0) vs[qv[i]][cv[i]] = v[i];
    }
    __syncthreads();
    const int r = d.r0 + rr;
    double acc = (d.hasid && g == 0 && r < m) ? vs[nv - 1][r] : 0.0;
#pragma unroll
    for (int q = 0; q < CR_MT; q++) {
        if (q >= nA) break;
        double p = 0.0;
#pragma unroll
        for (int u = 0; u < CPT; u++) {
            const int c = g + G * u;
            if (c < m) p += a[q][u] * vs[q][c];
        }
        acc += p;
    }
    /* lanes of one row within a wave are RC apart */
#pragma unroll
    for (int o = 32; o >= RC; o >>= 1) acc += __shfl_xor(acc, o, 64);
    const int lane = t & 63, wave = t >> 6;
    if (lane < RC) red[wave][lane] = acc;
    __syncthreads();
    if (t < RC && r < m) {
        const double sum = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
        double* const ys[4] = {nullptr, x, bv, xv};
        const int yb = d.yref >> 28, yo = d.yref & 0x0fffffff;
        ys[yb][yo + r] = sum;
        /* the solution also transposed (row j of block i at j * n + i) for its consumers,
         * whose lanes run along i */
        if (xT && yb == 1) xT[(int64_t)r * nT + yo / m] = sum;
    }
}

/* set-up copy of the matrix terms into the packed layout, one job per workgroup */
__global__ void __launch_bounds__(256) k_cr_pack(const CrPack* __restrict__ jobs, double* __restrict__ P, int m, int rc)
{
    const CrPack j = jobs[blockIdx.x];
    for (int e = threadIdx.x; e < m * rc; e += 256) {
        const int c = e / rc, rr = e - c * rc, r = j.r0 + rr;
        P[j.dst + e] = r < m ? j.s * j.A[r + (size_t)c * m] : 0.0;
    }
}

/* composite operators C = sum_k s_k A_k B_k: one 32x32 tile of one descriptor per workgroup */
__global__ void __launch_bounds__(256) k_cr_comp(const CrComp* __restrict__ dd, int m)
{
    const CrComp d = dd[blockIdx.y];
    const int T = (m + 31) / 32;
    const int r0 = (blockIdx.x % T) * 32, c0 = (blockIdx.x / T) * 32;
    const int t = threadIdx.x, tr = t & 31, tc = t >> 5;
    __shared__ double As[32][33], Bs[32][33];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int term = 0; term < d.nt; term++) {
        const double* A = d.A[term];
        const double* B = d.B[term];
        const double sc = d.s[term];
        if (!A) {                                           /* identity */
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (r0 + tr == c0 + tc + 8 * q && r0 + tr < m) acc[q] += sc;
            continue;
        }
        if (!B) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int rr = r0 + tr, cc = c0 + tc + 8 * q;
                if (rr < m && cc < m) acc[q] += sc * A[rr + (size_t)cc * m];
            }
            continue;
        }
        double pa[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < m; k0 += 32) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int e = t + 256 * q;
                const int rr = e & 31, kk = e >> 5;
                As[kk][rr] = (r0 + rr < m && k0 + kk < m) ? A[(r0 + rr) + (size_t)(k0 + kk) * m] : 0.0;
                const int kb = e & 31, cc = e >> 5;
                Bs[cc][kb] = (k0 + kb < m && c0 + cc < m) ? B[(k0 + kb) + (size_t)(c0 + cc) * m] : 0.0;
            }
            __syncthreads();
#pragma unroll 8
            for (int kk = 0; kk < 32; kk++) {
                const double av = As[kk][tr];
#pragma unroll
                for (int q = 0; q < 4; q++) pa[q] += av * Bs[tc + 8 * q][kk];
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < 4; q++) acc[q] += sc * pa[q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int rr = r0 + tr, cc = c0 + tc + 8 * q;
        if (rr < m && cc < m) d.C[rr + (size_t)cc * m] = acc[q];
    }
}

}  // namespace

/* one level down / up for nrhs right-hand sides (level vectors N[l] m apart) */
static void cr_down(const SchurCR& cr, int l, const double* bl, double* bn, int nrhs, hipStream_t s)
{
    const int m = cr.m, nch = (m + CR_RC - 1) / CR_RC, Nl = cr.N[l], ne = (Nl + 1) / 2;
    const size_t mm = (size_t)m * m;
    const double* ap = cr.ap.p + cr.ap_off[l];
    hipLaunchKernelGGL(k_cr_fwd, dim3(ne * nch, (nrhs + CR_RB - 1) / CR_RB), dim3(256), 0, s, bl, bn, ap,
                       ap + (size_t)ne * mm, Nl, cr.per[l], m, nch, (int64_t)Nl * m, (int64_t)cr.N[l + 1] * m, nrhs);
}
static void cr_up(const SchurCR& cr, int l, const double* bl, const double* xn, double* xl, int nrhs, hipStream_t s)
{
    const int m = cr.m, nch = (m + CR_RC - 1) / CR_RC, Nl = cr.N[l], ne = (Nl + 1) / 2, no = Nl / 2;
    const size_t mm = (size_t)m * m;
    const double* ap = cr.ap.p + cr.ap_off[l];
    hipLaunchKernelGGL(k_cr_bwd, dim3(no * nch, (nrhs + CR_RB - 1) / CR_RB), dim3(256), 0, s, bl, xn, xl,
                       ap + (size_t)2 * ne * mm, ap + (size_t)(2 * ne + no) * mm, ap + (size_t)(2 * ne + 2 * no) * mm,
                       Nl, cr.per[l], m, nch, (int64_t)Nl * m, (int64_t)cr.N[l + 1] * m, nrhs);
}

/* ---- apply steps: the level operations as block expressions, composed two levels at a
 * time.  A quantity (a block of a level vector) is a sum over leaves -- blocks of the
 * right-hand sides b_l or solutions x_l of other levels -- of coefficient matrices, each a
 * signed product of at most two level operators.  Composing level l with level l + 1 (the
 * down step b_l -> b_{l+2}, the up step x_{l+2} -> x_l) halves the apply launches; the
 * merged coefficients are materialised once per factorisation (k_cr_comp). */
namespace {
using Leaf = std::tuple<int, int, int>;          /* (0: b / 1: x, level, block) */
struct Prod {
    double s;
    const double* A;                             /* null: identity */
    const double* B;                             /* null: none     */
};
using Expr = std::map<Leaf, std::vector<Prod>>;

struct CrLevel {                                 /* level l operators (cr.ap) */
    const SchurCR& cr;
    int l;
    const double* op(int which, int idx) const
    {
        const size_t mm = (size_t)cr.m * cr.m;
        const int Nl = cr.N[l], ne = (Nl + 1) / 2, no = Nl / 2;
        const double* ap = cr.ap.p + cr.ap_off[l];
        switch (which) {
        case 0: return ap + (size_t)idx * mm;                        /* XL_q */
        case 1: return ap + (size_t)(ne + idx) * mm;                 /* XR_q */
        case 2: return ap + (size_t)(2 * ne + idx) * mm;             /* Dinv_p */
        case 3: return ap + (size_t)(2 * ne + no + idx) * mm;        /* YL_p */
        default: return ap + (size_t)(2 * ne + 2 * no + idx) * mm;   /* YR_p */
        }
    }
};

/* b_{l+1}[q] over b_l (k_cr_fwd) */
Expr fwd_expr(const SchurCR& cr, int l, int q)
{
    const CrLevel L{cr, l};
    const int Nl = cr.N[l], per = cr.per[l], e = 2 * q;
    const bool lex = e > 0 || per, rex = e + 1 < Nl || per;
    const int lnb = e > 0 ? e - 1 : Nl - 1, rnb = (e + 1) % Nl;
    Expr E;
    E[Leaf{0, l, e}].push_back({1.0, nullptr, nullptr});
    if (lex && (lnb & 1)) E[Leaf{0, l, lnb}].push_back({-1.0, L.op(0, q), nullptr});
    if (rex && (rnb & 1)) E[Leaf{0, l, rnb}].push_back({-1.0, L.op(1, q), nullptr});
    return E;
}
/* x_l[t] over x_{l+1} and b_l (k_cr_bwd; even blocks are copies) */
Expr bwd_expr(const SchurCR& cr, int l, int t)
{
    Expr E;
    if ((t & 1) == 0) {
        E[Leaf{1, l + 1, t / 2}].push_back({1.0, nullptr, nullptr});
        return E;
    }
    const CrLevel L{cr, l};
    const int Nl = cr.N[l], per = cr.per[l], p = t / 2;
    const bool rex = t + 1 < Nl || per;
    const int rn = (t + 1) % Nl;
    E[Leaf{0, l, t}].push_back({1.0, L.op(2, p), nullptr});
    E[Leaf{1, l + 1, p}].push_back({-1.0, L.op(3, p), nullptr});
    if (rex) E[Leaf{1, l + 1, rn / 2}].push_back({-1.0, L.op(4, p), nullptr});
    return E;
}
/* dst += s M E  (E's coefficients single operators) */
void add_mul(Expr& dst, double s, const double* M, const Expr& E)
{
    for (const auto& kv : E)
        for (const Prod& p : kv.second) {
            Prod q{s * p.s, p.A, nullptr};
            if (M) {
                if (p.A) { q.A = M; q.B = p.A; }
                else q.A = M;
            }
            dst[kv.first].push_back(q);
        }
}
/* E with every leaf of (kind, level) replaced by sub(block) */
template <class F>
Expr substitute(const Expr& E, int kind, int level, F sub)
{
    Expr R;
    for (const auto& kv : E) {
        if (std::get<0>(kv.first) != kind || std::get<1>(kv.first) != level) {
            for (const Prod& p : kv.second) R[kv.first].push_back(p);
            continue;
        }
        const Expr S = sub(std::get<2>(kv.first));
        for (const Prod& p : kv.second) {
            if (p.B) return Expr{};              /* not composable (never: single operators) */
            add_mul(R, p.s, p.A, S);
        }
    }
    return R;
}
struct OutSpec {
    int kind, level, block;                      /* the output quantity */
    Expr e;
};
}  // namespace

/* the outputs of the apply step(s) for levels [l0, l0 + nl) (nl = 1 or 2), down or up */
static std::vector<OutSpec> step_outputs(const SchurCR& cr, int l0, int nl, bool down)
{
    std::vector<OutSpec> out;
    if (down) {
        if (nl == 1) {
            for (int q = 0; q < cr.N[l0 + 1]; q++) out.push_back({0, l0 + 1, q, fwd_expr(cr, l0, q)});
            return out;
        }
        for (int r = 0; r < cr.N[l0 + 2]; r++)
            out.push_back({0, l0 + 2, r, substitute(fwd_expr(cr, l0 + 1, r), 0, l0 + 1,
                                                    [&](int q) { return fwd_expr(cr, l0, q); })});
        for (int q = 1; q < cr.N[l0 + 1]; q += 2) out.push_back({0, l0 + 1, q, fwd_expr(cr, l0, q)});
        return out;
    }
    if (nl == 1) {
        for (int t = 0; t < cr.N[l0]; t++) out.push_back({1, l0, t, bwd_expr(cr, l0, t)});
        return out;
    }
    for (int t = 0; t < cr.N[l0]; t++)
        out.push_back({1, l0, t, substitute(bwd_expr(cr, l0, t), 1, l0 + 1,
                                            [&](int q) { return bwd_expr(cr, l0 + 1, q); })});
    return out;
}

/* the packed form of one apply step (CrStep): 8 rows per chunk (16 measured 1.3 ms slower per
 * Newton step at 2 degrees, scripts/ab/cr_rc8.sh), fewer where the step would have < 448
 * workgroups (the small steps of the deep levels would leave CUs idle), the workgroups
 * sorted by matrix-term count into classes, the set-up copy jobs */
static int cr_pack_step(iemic_ctx* c, const SchurCR& cr, const std::vector<CrOut>& outs, CrStep& st)
{
    const int m = cr.m;
    int rcw = 8;
    while (rcw > 4 && (int64_t)outs.size() * ((m + rcw - 1) / rcw) < 448) rcw /= 2;
    const int nch = (m + rcw - 1) / rcw;
    struct W { int nA, o, ch; };
    std::vector<W> ws;
    for (int o = 0; o < (int)outs.size(); o++) {
        int nA = 0, nid = 0;
        for (int t = 0; t < outs[o].nt; t++) {
            if (outs[o].A[t]) nA++;
            else if (outs[o].s[t] != 1.0 || ++nid > 1) {
                set_error("Schur cyclic reduction: unexpected identity term in an apply step");
                return IEMIC_EINVAL;
            }
        }
        for (int ch = 0; ch < nch; ch++) ws.push_back({nA, o, ch});
    }
    std::stable_sort(ws.begin(), ws.end(), [](const W& a, const W& b) { return a.nA > b.nA; });
    CrCls cls{};
    std::vector<CrWg> wg(ws.size());
    std::vector<CrPack> jobs;
    int64_t pos = 0;
    auto ref = [](int base, int64_t off) { return (base << 28) | (int)off; };
    for (size_t w = 0; w < ws.size(); w++) {
        const W& q = ws[w];
        if (w == 0 || q.nA != ws[w - 1].nA) {
            if (cls.ncls == CR_NCLS) {
                set_error("Schur cyclic reduction: too many term classes in an apply step");
                return IEMIC_EINVAL;
            }
            cls.w0[cls.ncls] = (int)w;
            cls.nA[cls.ncls] = q.nA;
            cls.p0[cls.ncls] = pos;
            cls.ncls++;
        }
        const CrOut& o = outs[q.o];
        CrWg& d = wg[w];
        d.yref = ref(o.yb, o.yo);
        d.r0 = q.ch * rcw;
        int v = 0, id = -1;
        for (int t = 0; t < o.nt; t++) {
            if (!o.A[t]) {
                id = t;
                continue;
            }
            d.vref[v++] = ref(o.vb[t], o.vo[t]);
            jobs.push_back({o.A[t], o.s[t], pos, d.r0});
            pos += (int64_t)m * rcw;
        }
        d.hasid = id >= 0;
        if (id >= 0) d.vref[v++] = ref(o.vb[id], o.vo[id]);
        d.nv = v;
    }
    cls.w0[cls.ncls] = (int)ws.size();
    st.nwg = (int)ws.size();
    st.rc = rcw;
    st.cls = cls;
    st.njobs = (int)jobs.size();
    if (st.wg.alloc(wg.size()) || st.P.alloc(std::max<int64_t>(pos, 1)) || st.jobs.alloc(std::max<size_t>(jobs.size(), 1))) {
        set_error("Schur cyclic reduction: out of device memory");
        return IEMIC_ENOMEM;
    }
    int rc = h2d(c, st.wg.p, wg.data(), sizeof(CrWg) * wg.size());
    if (!rc && !jobs.empty()) rc = h2d(c, st.jobs.p, jobs.data(), sizeof(CrPack) * jobs.size());
    return rc;
}

/* apply steps (descriptors) and the composite operators they need; two levels per step
 * where the composed step stays within CR_MT terms */
static int cr_build_steps(iemic_ctx* c, SchurCR& cr)
{
    const int m = cr.m;
    const size_t mm = (size_t)m * m;
    const int le = cr.tM ? cr.lt : cr.nlev;
    struct Plan { int l0, nl; std::vector<OutSpec> dn, up; };
    std::vector<Plan> plan;
    for (int l = 0; l < le;) {
        Plan P{l, std::min(2, le - l), {}, {}};
        P.dn = step_outputs(cr, l, P.nl, true);
        P.up = step_outputs(cr, l, P.nl, false);
        bool ok = true;
        for (const auto* v : {&P.dn, &P.up})
            for (const OutSpec& o : *v) {
                ok &= (int)o.e.size() <= CR_MT;
                for (const auto& kv : o.e) ok &= kv.second.size() <= 4;
            }
        if (!ok && P.nl == 2) {                  /* fall back to one level */
            P.nl = 1;
            P.dn = step_outputs(cr, l, 1, true);
            P.up = step_outputs(cr, l, 1, false);
        }
        l += P.nl;
        plan.push_back(std::move(P));
    }
    /* composite operators: coefficients that are not a single signed operator */
    std::vector<CrComp> comps;
    auto is_single = [](const std::vector<Prod>& v) { return v.size() == 1 && !v[0].B; };
    for (const Plan& P : plan)
        for (const auto* v : {&P.dn, &P.up})
            for (const OutSpec& o : *v)
                for (const auto& kv : o.e)
                    if (!is_single(kv.second)) comps.push_back(CrComp{});
    cr.ncomp = (int)comps.size();
    if (cr.ncomp && (cr.cmat.alloc(comps.size() * mm) || cr.cdesc.alloc(comps.size()))) {
        set_error("Schur cyclic reduction: out of device memory");
        return IEMIC_ENOMEM;
    }
    auto vref = [&](int kind, int level, int block, int& base, int64_t& off) {
        if (level == 0) { base = kind; off = (int64_t)block * m; }
        else { base = 2 + kind; off = (int64_t)cr.v_off[level] + (int64_t)block * m; }
    };
    size_t ic = 0;
    cr.down.clear();
    cr.up.clear();
    cr.down.resize(plan.size());
    cr.up.resize(plan.size());
    for (size_t ip = 0; ip < plan.size(); ip++) {
        const Plan& P = plan[ip];
        for (int dir = 0; dir < 2; dir++) {
            const std::vector<OutSpec>& specs = dir == 0 ? P.dn : P.up;
            std::vector<CrOut> outs;
            for (const OutSpec& o : specs) {
                CrOut d{};
                vref(o.kind, o.level, o.block, d.yb, d.yo);
                for (const auto& kv : o.e) {
                    const int t = d.nt++;
                    vref(std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), d.vb[t], d.vo[t]);
                    if (is_single(kv.second)) {
                        d.s[t] = kv.second[0].s;
                        d.A[t] = kv.second[0].A;
                    } else {
                        CrComp& cc = comps[ic];
                        cc.C = cr.cmat.p + ic * mm;
                        cc.nt = (int)kv.second.size();
                        for (int k = 0; k < cc.nt; k++) {
                            cc.A[k] = kv.second[k].A;
                            cc.B[k] = kv.second[k].B;
                            cc.s[k] = kv.second[k].s;
                        }
                        d.s[t] = 1.0;
                        d.A[t] = cc.C;
                        ic++;
                    }
                }
                outs.push_back(d);
            }
            /* down steps top-first in plan order; up steps applied bottom-first (reverse) */
            CrStep& st = dir == 0 ? cr.down[ip] : cr.up[plan.size() - 1 - ip];
            int rc;
            if ((rc = cr_pack_step(c, cr, outs, st))) return rc;
        }
    }
    if (cr.ncomp) {
        int rc;
        if ((rc = h2d(c, cr.cdesc.p, comps.data(), sizeof(CrComp) * comps.size()))) return rc;
    }
    return 0;
}

/* level sizes, storage offsets and the GEMM descriptors (host, once per grid) */
int cr_init(iemic_ctx* c, SchurCR& cr, int n, int m, int periodic, int tail_max)
{
    if (m > 192) {
        set_error("Schur cyclic reduction: more than 192 latitudes");
        return IEMIC_EINVAL;
    }
    cr.n = n; cr.m = m; cr.periodic = periodic;
    cr.N.clear(); cr.per.clear(); cr.merge.clear();
    int N = n, P = periodic;
    while (N > 1) {
        const int mg = (N == 2 && P) ? 1 : 0;
        if (mg) P = 0;
        cr.N.push_back(N); cr.per.push_back(P); cr.merge.push_back(mg);
        N = (N + 1) / 2;
    }
    cr.N.push_back(1); cr.per.push_back(0); cr.merge.push_back(0);
    cr.nlev = (int)cr.N.size() - 1;
    const size_t mm = (size_t)m * m;
    cr.dlr_off.assign(cr.nlev + 1, 0);
    cr.ap_off.assign(cr.nlev + 1, 0);
    cr.v_off.assign(cr.nlev + 1, 0);
    size_t nd = 0, na = 0, nv = 0;
    for (int l = 0; l <= cr.nlev; l++) {
        cr.dlr_off[l] = nd;
        nd += 3 * (size_t)cr.N[l] * mm;
        cr.ap_off[l] = na;
        na += l < cr.nlev ? (size_t)(2 * ((cr.N[l] + 1) / 2) + 3 * (cr.N[l] / 2)) * mm : mm;
        cr.v_off[l] = nv;
        if (l > 0) nv += (size_t)cr.N[l] * m;
    }
    int rc = 0;
    rc |= cr.dlr.alloc(nd);
    rc |= cr.ap.alloc(na);
    rc |= cr.bv.alloc(std::max<size_t>(nv, 1));
    rc |= cr.xv.alloc(std::max<size_t>(nv, 1));
    rc |= cr.info.alloc(1);
    if (rc) {
        set_error("Schur cyclic reduction: out of device memory");
        return IEMIC_ENOMEM;
    }
    /* descriptors: per level the periodic-pair merge (g0), X/Y products (g1), next level (g2) */
    std::vector<CrGemm> g;
    cr.g_off.assign(3 * cr.nlev, 0);
    cr.g_cnt.assign(3 * cr.nlev, 0);
    auto blk = [&](int l, int which, int b) { return cr.dlr.p + cr.dlr_off[l] + ((size_t)which * cr.N[l] + b) * mm; };
    for (int l = 0; l < cr.nlev; l++) {
        const int Nl = cr.N[l], per = cr.per[l], ne = (Nl + 1) / 2, no = Nl / 2;
        double* ap = cr.ap.p + cr.ap_off[l];
        auto XL = [&](int q) { return ap + (size_t)q * mm; };
        auto XR = [&](int q) { return ap + (size_t)(ne + q) * mm; };
        auto DI = [&](int p) { return ap + (size_t)(2 * ne + p) * mm; };
        auto YL = [&](int p) { return ap + (size_t)(2 * ne + no + p) * mm; };
        auto YR = [&](int p) { return ap + (size_t)(2 * ne + 2 * no + p) * mm; };
        const auto D = [&](int b) { return blk(l, 0, b); };
        const auto Lb = [&](int b) { return blk(l, 1, b); };
        const auto Rb = [&](int b) { return blk(l, 2, b); };
        cr.g_off[3 * l] = (int)g.size();
        if (cr.merge[l]) {
            g.push_back({Rb(0), Lb(0), Rb(0), nullptr, nullptr, nullptr, nullptr, 0.0, 0.0});
            g.push_back({Lb(1), Lb(1), Rb(1), nullptr, nullptr, nullptr, nullptr, 0.0, 0.0});
        }
        cr.g_cnt[3 * l] = (int)g.size() - cr.g_off[3 * l];
        cr.g_off[3 * l + 1] = (int)g.size();
        for (int q = 0; q < ne; q++) {
            const int e = 2 * q;
            const bool lex = e > 0 || per, rex = e + 1 < Nl || per;
            const int lnb = e > 0 ? e - 1 : Nl - 1, rnb = (e + 1) % Nl;
            if (lex && (lnb & 1)) g.push_back({XL(q), nullptr, nullptr, Lb(e), DI(lnb / 2), nullptr, nullptr, 1.0, 0.0});
            if (rex && (rnb & 1)) g.push_back({XR(q), nullptr, nullptr, Rb(e), DI(rnb / 2), nullptr, nullptr, 1.0, 0.0});
        }
        for (int p = 0; p < no; p++) {
            g.push_back({YL(p), nullptr, nullptr, DI(p), Lb(2 * p + 1), nullptr, nullptr, 1.0, 0.0});
            g.push_back({YR(p), nullptr, nullptr, DI(p), Rb(2 * p + 1), nullptr, nullptr, 1.0, 0.0});
        }
        cr.g_cnt[3 * l + 1] = (int)g.size() - cr.g_off[3 * l + 1];
        cr.g_off[3 * l + 2] = (int)g.size();
        for (int q = 0; q < ne; q++) {
            const int e = 2 * q;
            const bool lex = e > 0 || per, rex = e + 1 < Nl || per;
            const int lnb = e > 0 ? e - 1 : Nl - 1, rnb = (e + 1) % Nl;
            const bool lo = lex && (lnb & 1), ro = rex && (rnb & 1);
            CrGemm dg{blk(l + 1, 0, q), D(e), nullptr, nullptr, nullptr, nullptr, nullptr, -1.0, -1.0};
            if (lo) { dg.A1 = XL(q); dg.B1 = Rb(lnb); }
            if (ro) { dg.A2 = XR(q); dg.B2 = Lb(rnb); }
            if (!dg.A1 && dg.A2) { dg.A1 = dg.A2; dg.B1 = dg.B2; dg.A2 = dg.B2 = nullptr; }
            g.push_back(dg);
            if (lo) g.push_back({blk(l + 1, 1, q), nullptr, nullptr, XL(q), Lb(lnb), nullptr, nullptr, -1.0, 0.0});
            else g.push_back({blk(l + 1, 1, q), lex ? Lb(e) : nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.0, 0.0});
            if (ro) g.push_back({blk(l + 1, 2, q), nullptr, nullptr, XR(q), Rb(rnb), nullptr, nullptr, -1.0, 0.0});
            else g.push_back({blk(l + 1, 2, q), rex ? Rb(e) : nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.0, 0.0});
        }
        cr.g_cnt[3 * l + 2] = (int)g.size() - cr.g_off[3 * l + 2];
    }
    if (cr.gd.alloc(std::max<size_t>(g.size(), 1))) {
        set_error("Schur cyclic reduction: out of device memory");
        return IEMIC_ENOMEM;
    }
    if (!g.empty() && (rc = h2d(c, cr.gd.p, g.data(), sizeof(CrGemm) * g.size()))) return rc;
    /* dense tail: the first level of at most 1024 unknowns (2048: no gain) and its
     * descendants become one explicit inverse (built at set-up by solving the tail for the
     * identity), so the apply spends one GEMV launch instead of 2 (nlev - lt) + 1 */
    if (tail_max <= 0) tail_max = CR_TAIL_MAX;
    cr.lt = cr.nlev;
    cr.tM = 0;
    for (int l = 0; l < cr.nlev; l++)
        if (cr.N[l] > 1 && (int64_t)cr.N[l] * m <= tail_max) {
            cr.lt = l;
            cr.tM = cr.N[l] * m;
            break;
        }
    if (cr.tM) {
        cr.tb_off.assign(cr.nlev - cr.lt + 1, 0);
        size_t nt = 0;
        for (int l = cr.lt; l <= cr.nlev; l++) {
            cr.tb_off[l - cr.lt] = nt;
            nt += (size_t)cr.N[l] * m * cr.tM;
        }
        if (cr.tinv.alloc((size_t)cr.tM * cr.tM) || cr.tb.alloc(nt) || cr.tx.alloc(nt)) {
            set_error("Schur cyclic reduction: out of device memory");
            return IEMIC_ENOMEM;
        }
    }
    return cr_build_steps(c, cr);
}

static int cr_inverse(hipStream_t s, int m, int count, const double* src, int s0, int sstep, double* dst,
                      int* info)
{
    if (count <= 0) return 0;
#define CR_INV(TR, RA, RB)                                                                           \
    hipLaunchKernelGGL((k_cr_inv<TR, RA, RB>), dim3(count), dim3(32 * TR), 0, s, src, s0, sstep, dst, m, info)
    if (m <= 32) CR_INV(16, 2, 1);
    else if (m <= 64) CR_INV(16, 4, 2);
    else if (m <= 96) CR_INV(16, 6, 3);
    else if (m <= 128) CR_INV(32, 4, 4);
    else if (m <= 160) CR_INV(32, 5, 5);
    else if (m <= 192) CR_INV(32, 6, 6);
    else {
        set_error("Schur cyclic reduction: more than 192 latitudes");
        return IEMIC_EINVAL;
    }
#undef CR_INV
    HIP_OK(hipGetLastError());
    return 0;
}

/* the inverse of one m x m column-major block (m <= 192) on the device; *info set on a
 * zero pivot */
int cr_inverse_dev(hipStream_t s, int m, const double* src, double* dst, int* info)
{
    return cr_inverse(s, m, 1, src, 0, 1, dst, info);
}

/* set-up from the 9-point rows (stream-ordered, no host synchronisation) */
int cr_factor(iemic_ctx* c, SchurCR& cr, const double* S9, const int* col_of_ij)
{
    hipStream_t s = c->stream;
    const int m = cr.m;
    const size_t mm = (size_t)m * m;
    HIP_OK(hipMemsetAsync(cr.dlr.p, 0, sizeof(double) * 3 * (size_t)cr.n * mm, s));
    const int nm = cr.n * m;
    hipLaunchKernelGGL(k_cr_expand, dim3((nm + 255) / 256), dim3(256), 0, s, S9, col_of_ij, cr.n, m,
                       cr.periodic, cr.dlr.p, cr.dlr.p + (size_t)cr.n * mm, cr.dlr.p + 2 * (size_t)cr.n * mm);
    return cr_factor_blocks(c, cr);
}

/* set-up from level-0 blocks already in cr.dlr (D, L, R: 3 n column-major m x m blocks) */
int cr_factor_blocks(iemic_ctx* c, SchurCR& cr)
{
    hipStream_t s = c->stream;
    int rc;
    const int m = cr.m;
    const size_t mm = (size_t)m * m;
    const int T = (m + 31) / 32;
    HIP_OK(hipMemsetAsync(cr.info.p, 0, sizeof(int), s));
    for (int l = 0; l < cr.nlev; l++) {
        const int Nl = cr.N[l], ne = (Nl + 1) / 2, no = Nl / 2;
        if (cr.g_cnt[3 * l])
            hipLaunchKernelGGL(k_cr_gemm, dim3(T * T, cr.g_cnt[3 * l]), dim3(256), 0, s, cr.gd.p + cr.g_off[3 * l], m);
        if ((rc = cr_inverse(s, m, no, cr.dlr.p + cr.dlr_off[l], 1, 2, cr.ap.p + cr.ap_off[l] + (size_t)2 * ne * mm,
                             cr.info.p)))
            return rc;
        hipLaunchKernelGGL(k_cr_gemm, dim3(T * T, cr.g_cnt[3 * l + 1]), dim3(256), 0, s,
                           cr.gd.p + cr.g_off[3 * l + 1], m);
        hipLaunchKernelGGL(k_cr_gemm, dim3(T * T, cr.g_cnt[3 * l + 2]), dim3(256), 0, s,
                           cr.gd.p + cr.g_off[3 * l + 2], m);
    }
    if ((rc = cr_inverse(s, m, 1, cr.dlr.p + cr.dlr_off[cr.nlev], 0, 1, cr.ap.p + cr.ap_off[cr.nlev], cr.info.p)))
        return rc;
    if (cr.ncomp)                          /* the composite operators of the apply steps */
        hipLaunchKernelGGL(k_cr_comp, dim3(T * T, cr.ncomp), dim3(256), 0, s, cr.cdesc.p, m);
    for (const auto* v : {&cr.down, &cr.up})   /* the apply steps' packed operators */
        for (const CrStep& st : *v)
            if (st.njobs)
                hipLaunchKernelGGL(k_cr_pack, dim3(st.njobs), dim3(256), 0, s, (const CrPack*)st.jobs.p, st.P.p, m,
                                   st.rc);
    if (cr.tM) {                           /* the tail's inverse, column r = tail solve of e_r */
        const int M = cr.tM;
        auto tb = [&](int l) { return cr.tb.p + cr.tb_off[l - cr.lt]; };
        auto tx = [&](int l) { return cr.tx.p + cr.tb_off[l - cr.lt]; };
        hipLaunchKernelGGL(k_cr_eye, dim3((unsigned)(((int64_t)M * M + 255) / 256)), dim3(256), 0, s, tb(cr.lt), M);
        for (int l = cr.lt; l < cr.nlev; l++) cr_down(cr, l, tb(l), tb(l + 1), M, s);
        hipLaunchKernelGGL(k_cr_final, dim3((m + CR_RC - 1) / CR_RC, (M + CR_RB - 1) / CR_RB), dim3(256), 0, s,
                           (const double*)(cr.ap.p + cr.ap_off[cr.nlev]), (const double*)tb(cr.nlev), tx(cr.nlev), m, M);
        for (int l = cr.nlev - 1; l >= cr.lt; l--) cr_up(cr, l, tb(l), tx(l + 1), tx(l), M, s);
        hipLaunchKernelGGL(k_cr_transpose, dim3((M + 31) / 32, (M + 31) / 32), dim3(256), 0, s,
                           (const double*)tx(cr.lt), cr.tinv.p, M);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

int cr_check(iemic_ctx* c, SchurCR& cr)
{
    int info = 0, rc;
    if ((rc = d2h(c, &info, cr.info.p, sizeof(int)))) return rc;
    if (info) {
        set_error("block GS: singular block in the Schur cyclic reduction");
        return IEMIC_EINVAL;
    }
    return 0;
}

/* x = S^-1 b (b, x: n*m, c = i*m + j): the levels above the tail in apply steps of one or
 * two levels each way (k_cr_multi), the tail (levels >= lt, tM = N[lt] m unknowns) one
 * dense GEMV */
static void cr_step(const SchurCR& cr, const CrStep& st, const double* b, double* x, hipStream_t s,
                    double* xT = nullptr)
{
    const int m = cr.m;
    double* bv = const_cast<double*>(cr.bv.p);
    double* xv = const_cast<double*>(cr.xv.p);
    const dim3 g((unsigned)st.nwg), blk(256);
    const int nT = cr.N[0];
#define CR_PK(RC, CPT) hipLaunchKernelGGL((k_cr_pk<RC, CPT>), g, blk, 0, s, (const double*)st.P.p, st.cls, \
                                          (const CrWg*)st.wg.p, m, b, x, bv, xv, xT, nT)
    if (st.rc == 16) {
        if (m <= 80) CR_PK(16, 5);
        else CR_PK(16, 12);
    } else if (st.rc == 8) {
        if (m <= 96) CR_PK(8, 3);
        else CR_PK(8, 6);
    } else {
        if (m <= 128) CR_PK(4, 2);
        else CR_PK(4, 3);
    }
#undef CR_PK
}

int cr_solve(iemic_ctx* c, const SchurCR& cr, const double* b, double* x, hipStream_t s, double* xT)
{
    (void)c;
    auto bvec = [&](int l) { return l == 0 ? b : cr.bv.p + cr.v_off[l]; };
    auto xvec = [&](int l) { return l == 0 ? x : cr.xv.p + cr.v_off[l]; };
    const int le = cr.tM ? cr.lt : cr.nlev;
    for (const CrStep& st : cr.down) cr_step(cr, st, b, x, s);
    if (cr.tM)
        hipLaunchKernelGGL(k_cr_tail, dim3((cr.tM + 3) / 4), dim3(256), 0, s, (const double*)cr.tinv.p, bvec(le),
                           xvec(le), cr.tM, le == 0 ? xT : nullptr, cr.N[0], cr.m);
    else
        hipLaunchKernelGGL(k_cr_final, dim3((cr.m + CR_RC - 1) / CR_RC), dim3(256), 0, s,
                           (const double*)(cr.ap.p + cr.ap_off[cr.nlev]), bvec(le), xvec(le), cr.m, 1);
    for (const CrStep& st : cr.up) cr_step(cr, st, b, x, s, xT);
    if (xT && le == 0 && !cr.tM)           /* one block (n = 1): the transposed order is x's */
        HIP_OK(hipMemcpyAsync(xT, x, sizeof(double) * cr.m, hipMemcpyDeviceToDevice, s));
    HIP_OK(hipGetLastError());
    return 0;
}

}  // namespace iemic
