/*
 * prec_gs.hip -- block Gauss-Seidel preconditioner for the THCM Jacobian (prec = 2).
 *
 * Replaces the reference's TRIOS::BlockPreconditioner with MRILU/ML sub-solves
 * (src/trios/TRIOS_BlockPreconditioner.C, after de Niet & Wubs)
 * by a fully GPU-resident variant of the same block structure.  Unknowns are split into
 *   known   identity rows (land, rigid lid, closed boundaries): z = r
 *   dyn     U/V (horizontal momentum), W (hydrostatic rows), P (continuity rows)
 *   ts      T/S (heat and salt)
 * and solved in the order known -> dyn -> ts (block lower triangular: the buoyancy and
 * momentum couplings from T/S into the dynamics are the dropped upper part):
 *   1. ptil : hydrostatic rows  Gw ptil = r_w, column-wise top-down with p_top = 0
 *   2. uv*  : D^-1 (r_uv - Guv ptil), D = per-point 2x2 U/V (Coriolis) block
 *   3. pbar : depth-integrated continuity per water column, 2-D Schur complement
 *             S = Mz2 Duv D^-1 Guv Mz1^T (9-point, corner-staggered), null space pinned
 *             (one column per checkerboard colour and basin), solved exactly by block
 *             cyclic reduction over longitudes (schur_cr.hip)
 *   4. uv   : uv* - D^-1 Guv Mz1^T pbar,  p = ptil + Mz1^T pbar
 *   5. w    : continuity rows Dw w = r_p - Duv uv, column-wise bottom-up
 *   6. ts   : A_ts ts = r_ts - B_ts,uv uv - B_ts,w w, by symmetric red-black Gauss-Seidel
 *             sweeps with 2x2 T/S cell blocks (parity of i+j+k)
 * Every step is a structured-grid kernel over cells or water columns reading the
 * stencil-ELL Jacobian in place; the only dense objects are the m x m blocks of the
 * Schur cyclic reduction (O(n m^2) doubles, 40 MB at 2 degrees).
 */
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "common.h"

namespace iemic {

namespace {

/* slot indices (see SLOTS in stencil.h) */
constexpr int S_UU0 = 0, S_UV0 = 7;                 /* U row: U self, V self            */
constexpr int S_UP = 20;                            /* U row: P (0,0),(1,0),(0,1),(1,1) */
constexpr int S_VV0 = 24, S_VU0 = 31;               /* V row: V self, U self            */
constexpr int S_VP = 42;                            /* V row: P, same order             */
constexpr int S_WP0 = 47, S_WP1 = 48;               /* W row: P(k), P(k+1)              */
constexpr int S_PU = 54, S_PV = 58;                 /* P row: U/V (0,0),(-1,0),(0,-1),(-1,-1) */
constexpr int S_PW0 = 62, S_PWM = 63;               /* P row: W(k), W(k-1)              */
constexpr int S_TT0 = 64, S_TS0 = 81;               /* T row: T self, S self            */
constexpr int S_SS0 = 84, S_ST0 = 101;              /* S row: S self, T self            */
constexpr int GSL = 10;                             /* gslot doubles per cell           */

/* subdomain layout seen by the kernels (stencil.h ext layout, Decomp2D): n, m global;
 * owned columns [ib0, ib0 + nx), rows from jb0; per-cell arrays are indexed by ext cell,
 * the Jacobian by owned cell (ext cell - own0: the owned cells are one slab) */
struct Lay {
    int n, m, l, periodic, jb0, ib0, nx, hx;
    int64_t nloc, own0, xb;
    int64_t ps;                      /* plane stride of the planar dynamics vectors (next) */
};
/* unknown v of ext cell e in a component-planar vector */
#define PL(e, v) ((e) + (int64_t)(v) * L.ps)
/* ext cell of global (i, j, k) (i in the grid after hnb's wrap; the x halo when split) */
__device__ __forceinline__ int64_t ecell(const Lay& L, int i, int j, int k)
{
    const int64_t r = ((int64_t)j - L.jb0 + HALO) * L.l + k;
    return xcell(r, xlocal(i, L.n, L.ib0, L.nx, L.hx, L.hx ? L.periodic : 0), L.nx, L.hx, L.xb);
}
__device__ __forceinline__ void lc_ijk(const Lay& L, int64_t lc, int& i, int& j, int& k)
{
    i = L.ib0 + (int)(lc % L.nx);
    k = (int)((lc / L.nx) % L.l);
    j = L.jb0 + (int)(lc / ((int64_t)L.nx * L.l));
}
__device__ __forceinline__ SubLay sub_of(const Lay& L)
{
    SubLay X;
    X.n = L.n; X.m = L.m; X.l = L.l; X.periodic = L.periodic;
    X.jb0 = L.jb0; X.ib0 = L.ib0; X.nx = L.nx; X.hx = L.hx; X.xb = L.xb;
    return X;
}
#define LAY_ALIASES const int n = L.n, m = L.m, l = L.l, periodic = L.periodic; (void)n; (void)m; (void)l; (void)periodic
/* thread -> owned cell: lc (Jacobian column), cell (ext), (i, j, k) */
#define OWNED_CELL                                                                       \
    const int64_t lc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;                   \
    if (lc >= L.nloc) return;                                                            \
    const int64_t cell = L.own0 + lc;                                                    \
    const int64_t ncell = L.nloc;                                                        \
    int i, j, k;                                                                         \
    lc_ijk(L, lc, i, j, k);                                                              \
    (void)i; (void)j; (void)k; (void)ncell
/* wrap / reject a horizontal neighbour; returns false when outside the domain */
__device__ __forceinline__ bool hnb(int& i, int& j, int n, int m, int periodic)
{
    if (j < 0 || j >= m) return false;
    if (i < 0 || i >= n) {
        if (!periodic) return false;
        i = (i + n) % n;
    }
    return true;
}

/* ---- structure ------------------------------------------------------------------- */

/* identity rows: diagonal slot exactly 1, every other slot exactly 0 */
__global__ void k_known(const double* __restrict__ val, Lay L, int64_t rowintcon,
                        uint8_t* __restrict__ known)
{
    OWNED_CELL;
    for (int r = 0; r < NUN; r++) {
        bool id = val[(int64_t)ROW_BEGIN[r] * ncell + lc] == 1.0;
        for (int s = ROW_BEGIN[r] + 1; id && s < ROW_BEGIN[r + 1]; s++)
            id = val[(int64_t)s * ncell + lc] == 0.0;
        known[NUN * cell + r] = (id && NUN * cell + r != rowintcon) ? 1 : 0;
    }
}

/* 1 per owned cell (owned index lc) with a non-identity row */
__global__ void k_cell_active(const uint8_t* __restrict__ known, Lay L, uint8_t* __restrict__ act)
{
    OWNED_CELL;
    bool a = false;
#pragma unroll
    for (int r = 0; r < NUN; r++) a |= !known[NUN * cell + r];
    act[lc] = a ? 1 : 0;
}

/* 2x2 inverse of [[a b][c d]] restricted to the active unknowns (ia, ib) */
__device__ __forceinline__ void inv2(double a, double b, double c, double d, bool ia, bool ib,
                                     double* out)
{
    out[0] = out[1] = out[2] = out[3] = 0.0;
    if (ia && ib) {
        const double det = a * d - b * c;
        if (det != 0.0) {
            const double q = 1.0 / det;
            out[0] = d * q; out[1] = -b * q; out[2] = -c * q; out[3] = a * q;
        }
    } else if (ia) {
        if (a != 0.0) out[0] = 1.0 / a;
    } else if (ib) {
        if (d != 0.0) out[3] = 1.0 / d;
    }
}

/* per-cell factors: U/V and T/S 2x2 inverses, depth-integration weight of the P row */
__global__ void k_cell_factors(const double* __restrict__ val, const uint8_t* __restrict__ known,
                               Lay L, int64_t rowintcon, int int_sign,
                               const double* __restrict__ intc, double* __restrict__ uvinv,
                               double* __restrict__ tsinv, double* __restrict__ pw,
                               double* __restrict__ tsdiag, int64_t next)
{
    OWNED_CELL;
    auto V = [&](int s) { return val[(int64_t)s * ncell + lc]; };
    const uint8_t* kn = known + NUN * cell;
    inv2(V(S_UU0), V(S_UV0), V(S_VU0), V(S_VV0), !kn[UU], !kn[VV], uvinv + 4 * cell);
    double sdiag = V(S_SS0), sofft = V(S_ST0);
    if (NUN * cell + SS == rowintcon) {
        sdiag = int_sign * intc[NUN * cell + SS];
        sofft = 0.0;
    }
    inv2(V(S_TT0), V(S_TS0), sofft, sdiag, !kn[TT], !kn[SS], tsinv + 4 * cell);
    {
        /* the 2x2 T/S block the sweeps invert, restricted to the active unknowns */
        const bool ta = !kn[TT], sa = !kn[SS];
        tsdiag[cell] = ta ? V(S_TT0) : 0.0;
        tsdiag[next + cell] = ta && sa ? V(S_TS0) : 0.0;
        tsdiag[2 * next + cell] = ta && sa ? sofft : 0.0;
        tsdiag[3 * next + cell] = sa ? sdiag : 0.0;
    }
    /* depth integral of the continuity rows: weight 1/a_k with a_k the coefficient of
     * the row's own W (or -1/b_k with b_k that of W(k-1) when the own W is an identity) */
    double w = 0.0;
    if (!kn[PP]) {
        const int64_t nm = L.nx;                /* k - 1 is one row of nx cells back */
        const bool w_own = !kn[WW];
        const bool w_below = k > 0 && !known[NUN * (cell - nm) + WW];
        if (w_own && V(S_PW0) != 0.0) w = 1.0 / V(S_PW0);
        else if (w_below && V(S_PWM) != 0.0) w = -1.0 / V(S_PWM);
        else w = 1.0;
    }
    pw[cell] = w;
}

/* Schur entry S[c][c'] for c' = column (i+di, j+dj): S9[c*9 + (dj+1)*3 + (di+1)], c = i*m + j.
 * Only the rows of this band's columns are built (the bands' rows are summed over the
 * ranks afterwards); corner U/V points one latitude row below the band are read from the
 * halo-filled per-cell arrays (known, uvinv, gslot). */
__global__ void k_schur_build(const double* __restrict__ val, const uint8_t* __restrict__ known,
                              const double* __restrict__ uvinv, const double* __restrict__ gslot,
                              const double* __restrict__ pw, const int* __restrict__ col_of_ij,
                              const uint8_t* __restrict__ pinned, Lay L, int jb1,
                              double* __restrict__ S9)
{
    LAY_ALIASES;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)L.nx * (jb1 - L.jb0) * 9) return;
    const int q = (int)(t / 9), o = (int)(t % 9);
    const int di = o % 3 - 1, dj = o / 3 - 1;
    const int i = L.ib0 + q % L.nx, j = L.jb0 + q / L.nx;
    const int c = col_of_ij[j * n + i];
    if (c < 0) return;
    double* row = S9 + (int64_t)c * 9;
    if (pinned[c]) {
        if (o == 4) row[4] = 1.0;
        return;
    }
    int ti = i + di, tj = j + dj;
    if (!hnb(ti, tj, n, m, periodic)) return;
    const int c2 = col_of_ij[tj * n + ti];
    if (c2 < 0 || pinned[c2]) return;
    const int64_t ncell = L.nloc;
    double s = 0.0;
    for (int k = 0; k < l; k++) {
        const int64_t pc = ecell(L, i, j, k);
        if (known[NUN * pc + PP]) continue;
        const int64_t tc = ecell(L, ti, tj, k);
        if (known[NUN * tc + PP]) continue;
        double acc = 0.0;
        /* corners q = (i+a, j+b), a,b in {0,-1}; P row slot index q4 = (0,0),(-1,0),(0,-1),(-1,-1) */
        for (int q4 = 0; q4 < 4; q4++) {
            const int a = -(q4 & 1), b = -((q4 >> 1) & 1);
            const int e = di - a, f = dj - b;
            if (e < 0 || e > 1 || f < 0 || f > 1) continue;
            int qi = i + a, qj = j + b;
            if (!hnb(qi, qj, n, m, periodic)) continue;
            const int64_t qc = ecell(L, qi, qj, k);
            const bool ua = !known[NUN * qc + UU], va = !known[NUN * qc + VV];
            if (!ua && !va) continue;
            const double du = ua ? val[(int64_t)(S_PU + q4) * ncell + (pc - L.own0)] : 0.0;
            const double dv = va ? val[(int64_t)(S_PV + q4) * ncell + (pc - L.own0)] : 0.0;
            const double* Di = uvinv + 4 * qc;
            const double yu = du * Di[0] + dv * Di[2];
            const double yv = du * Di[1] + dv * Di[3];
            const int g4 = e + 2 * f;                      /* (0,0),(1,0),(0,1),(1,1) */
            const double gu = ua ? gslot[GSL * qc + g4] : 0.0;
            const double gv = va ? gslot[GSL * qc + 4 + g4] : 0.0;
            acc += yu * gu + yv * gv;
        }
        s += pw[pc] * acc;
    }
    row[o] = s;
}

/* per owned cell: the U and V rows' couplings to the 4 P corners (slots 20..23, 42..45)
 * and the W row's to P(k), P(k+1) (slots 47, 48) */
__global__ void k_gslot_pack(const double* __restrict__ val, Lay L, double* __restrict__ gslot)
{
    OWNED_CELL;
    for (int g = 0; g < 4; g++) {
        gslot[GSL * cell + g] = val[(int64_t)(S_UP + g) * ncell + lc];
        gslot[GSL * cell + 4 + g] = val[(int64_t)(S_VP + g) * ncell + lc];
    }
    gslot[GSL * cell + 8] = val[(int64_t)S_WP0 * ncell + lc];
    gslot[GSL * cell + 9] = val[(int64_t)S_WP1 * ncell + lc];
}

/* identity-row flags <-> doubles (for the halo exchange of the flags) */
__global__ void k_u8_to_d(const uint8_t* __restrict__ a, double* __restrict__ b, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        b[q] = a[q];
}
__global__ void k_d_to_u8(const double* __restrict__ b, uint8_t* __restrict__ a, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        a[q] = b[q] != 0.0 ? 1 : 0;
}

/* Band LU with partial pivoting (LAPACK gbtrf semantics), one workgroup of 1024 threads,
 * right-looking and blocked by panels of NBP columns: the panel is factorised in LDS
 * (partial pivoting, full panel-row interchanges), row swaps and U12 = L11^-1 A12 follow,
 * and the trailing window is updated once per panel (A22 -= L21 U12) instead of once per
 * column.  U stays in the band (row i holds columns [i-bl, i+bl+bu] at offset
 * j - i + bl); the panel multipliers go to lpan[panel][NBP + bl][NBP], so a solve applies,
 * panel by panel, the panel's interchanges and then its multipliers. */
constexpr int NBP = 16;

__global__ void __launch_bounds__(1024) k_band_lu(double* __restrict__ ab, int ncol, int bl, int bu,
                                                  int* __restrict__ piv, int* __restrict__ info,
                                                  double* __restrict__ lpan, int stage_o)
{
    extern __shared__ double lds[];
    const int W = 2 * bl + bu + 1;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, nwave = nthr >> 6;
    /* panel rows padded to PS = NBP + 1 doubles: lanes walking a column hit distinct banks */
    constexpr int PS = NBP + 1;
    double* P = lds;                              /* (NBP + bl) x PS panel           */
    double* U = lds + (NBP + bl) * PS;            /* NBP x (bl + bu) block row U12   */
    double* Uo = U + NBP * (bl + bu);             /* NBP x (bl + bu) pivot rows below */
    __shared__ int s_lp[NBP], s_slot[NBP];
    __shared__ double s_best;
    __shared__ int s_info;
    if (tid == 0) s_info = 0;
    auto A = [&](int i, int j) -> double& { return ab[(int64_t)i * W + (j - i + bl)]; };
    for (int k0 = 0; k0 < ncol; k0 += NBP) {
        const int nbk = min(NBP, ncol - k0);
        const int pend = min(k0 + nbk - 1 + bl, ncol - 1);
        const int nprow = pend - k0 + 1;
        /* load the panel */
        for (int e = tid; e < nprow * NBP; e += nthr) {
            const int r = e / NBP, t = e % NBP;
            P[r * PS + t] = (t < nbk && r <= t + bl) ? A(k0 + r, k0 + t) : 0.0;
        }
        __syncthreads();
        /* factorise the panel: wavefront 0 finds the pivot and interchanges the panel
         * rows; then one thread per row below scales its multiplier and updates the rest
         * of its row (two workgroup barriers per column) */
        for (int t = 0; t < nbk; t++) {
            const int rlast = min(t + bl, nprow - 1);
            if (wave == 0) {
                double best = -1.0;
                int bi = t;
                for (int r = t + lane; r <= rlast; r += 64) {
                    const double v = fabs(P[r * PS + t]);
                    if (v > best) { best = v; bi = r; }
                }
                for (int off = 32; off > 0; off >>= 1) {
                    const double ob = __shfl_down(best, off, 64);
                    const int oi = __shfl_down(bi, off, 64);
                    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
                }
                best = __shfl(best, 0, 64);
                const int rp = __shfl(bi, 0, 64);
                if (best == 0.0) {
                    if (lane == 0) {
                        s_lp[t] = t;
                        piv[k0 + t] = k0 + t;
                        s_best = 0.0;
                        if (s_info == 0) s_info = k0 + t + 1;
                    }
                } else {
                    if (rp != t && lane < nbk) {
                        const double x = P[t * PS + lane];
                        P[t * PS + lane] = P[rp * PS + lane];
                        P[rp * PS + lane] = x;
                    }
                    if (lane == 0) { s_lp[t] = rp; piv[k0 + t] = k0 + rp; s_best = best; }
                }
            }
            __syncthreads();
            if (s_best == 0.0) {
                __syncthreads();
                continue;
            }
            const double pivot = P[t * PS + t];
            for (int r = t + 1 + tid; r <= rlast; r += nthr) {
                const double l = P[r * PS + t] / pivot;
                P[r * PS + t] = l;
                for (int cc = t + 1; cc < nbk; cc++) P[r * PS + cc] -= l * P[t * PS + cc];
            }
            __syncthreads();
        }
        /* U11 back to the band; the multipliers (L11, L21 with the panel's row
         * interchanges applied, LAPACK getrf convention) go to the panel store */
        double* Lp = lpan + (int64_t)(k0 / NBP) * (NBP + bl) * NBP;
        for (int e = tid; e < (NBP + bl) * NBP; e += nthr) {
            const int r = e / NBP, t = e % NBP;
            const bool in = r < nprow && t < nbk;
            if (in && r <= t) A(k0 + r, k0 + t) = P[r * PS + t];
            Lp[e] = (in && r > t) ? P[r * PS + t] : 0.0;
        }
        /* A12 (the panel rows right of the panel) and the rows below the panel that were
         * chosen as pivots (distinct ones, slot s_slot[t]) are staged in LDS with coalesced
         * loads; per column (one thread each) the interchanges in pivot order and
         * U12 = L11^-1 A12 then run on LDS only, and the pivot rows are written back */
        const int jlo = k0 + nbk, jhi = min(k0 + nbk - 1 + bl + bu, ncol - 1);
        const int ncu = jhi - jlo + 1;
        const int LW = bl + bu;
        if (tid == 0)
            for (int t = 0; t < nbk; t++) {
                int sl = -1;
                if (s_lp[t] >= nbk) {
                    sl = t;
                    for (int u = 0; u < t; u++)
                        if (s_lp[u] == s_lp[t]) { sl = s_slot[u]; break; }
                }
                s_slot[t] = sl;
            }
        for (int e = tid; e < nbk * ncu; e += nthr) {
            const int t = e / ncu, jj = e % ncu, j = jlo + jj;
            U[t * LW + jj] = (j <= k0 + t + bl + bu) ? A(k0 + t, j) : 0.0;
        }
        __syncthreads();
        for (int e = tid; e < nbk * ncu; e += nthr) {
            const int t = e / ncu, jj = e % ncu;
            if (stage_o && s_slot[t] == t) Uo[t * LW + jj] = A(k0 + s_lp[t], jlo + jj);
        }
        __syncthreads();
        for (int jj = tid; jj < ncu; jj += nthr) {
            const int j = jlo + jj;
            for (int t = 0; t < nbk; t++) {
                const int rp = s_lp[t];
                if (rp == t || j > k0 + t + bl + bu) continue;
                double& x = U[t * LW + jj];
                double& y = rp < nbk ? U[rp * LW + jj] : (stage_o ? Uo[s_slot[t] * LW + jj] : A(k0 + rp, j));
                const double tmp = x; x = y; y = tmp;
            }
            double u[NBP];
            for (int t = 0; t < nbk; t++) {
                double v = U[t * LW + jj];
                for (int q = 0; q < t; q++) v -= P[t * PS + q] * u[q];
                u[t] = v;
                U[t * LW + jj] = v;
                if (j <= k0 + t + bl + bu) A(k0 + t, j) = v;
            }
        }
        __syncthreads();
        for (int e = tid; e < nbk * ncu; e += nthr) {
            const int t = e / ncu, jj = e % ncu;
            if (stage_o && s_slot[t] == t) A(k0 + s_lp[t], jlo + jj) = Uo[t * LW + jj];
        }
        __syncthreads();
        /* A22 -= L21 U12 over rows k0+nbk .. pend: 4x4 register tiles (lanes along the
         * columns, so the 16 global loads of a tile are coalesced across the wavefront and
         * issued together before the rank-NBP update) */
        {
            const int nr2 = nprow - nbk;
            const int tr = (nr2 + 3) / 4, tc = (ncu + 3) / 4;
            for (int e = tid; e < tr * tc; e += nthr) {
                const int r0 = nbk + 4 * (e / tc), j0 = 4 * (e % tc);
                double a[4][4];
#pragma unroll
                for (int x = 0; x < 4; x++)
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const int r = r0 + x, jj = j0 + y;
                        a[x][y] = (r < nprow && jj < ncu) ? A(k0 + r, jlo + jj) : 0.0;
                    }
                for (int t = 0; t < nbk; t++) {
                    double lv[4], uv[4];
#pragma unroll
                    for (int x = 0; x < 4; x++) lv[x] = r0 + x < nprow ? P[(r0 + x) * PS + t] : 0.0;
#pragma unroll
                    for (int y = 0; y < 4; y++) uv[y] = j0 + y < ncu ? U[t * (bl + bu) + j0 + y] : 0.0;
#pragma unroll
                    for (int x = 0; x < 4; x++)
#pragma unroll
                        for (int y = 0; y < 4; y++) a[x][y] -= lv[x] * uv[y];
                }
#pragma unroll
                for (int x = 0; x < 4; x++)
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const int r = r0 + x, jj = j0 + y;
                        if (r < nprow && jj < ncu) A(k0 + r, jlo + jj) = a[x][y];
                    }
            }
        }
        __syncthreads();
    }
    if (tid == 0) *info = s_info;
}

/* Columns cols[q0 .. q0+NB) of the inverse, X = U^-1 L^-1 P, one workgroup of 256
 * threads per block of NB right-hand sides (unit vectors); cols ascending.  Column q of
 * the slab is X[row * nq + q] (row-major ncol x nq).  Thread t owns slab column t % NB
 * and every 256/NB-th row of the active window; the window lives in LDS as a ring buffer:
 *   forward  (P, L^-1): rows k..k+bl      y is written to X
 *   backward (U^-1)   : rows i+1..i+bl+bu x overwrites y in X
 * Two barriers per elimination step; the factors are read from L2. */
template <int NB, bool STAGE>
__global__ void __launch_bounds__(256) k_band_inv_pan(const double* __restrict__ ab,
                                                      const double* __restrict__ lpan,
                                                      const int* __restrict__ piv, int ncol,
                                                      int bl, int bu, const int* __restrict__ cols,
                                                      int nq, double* __restrict__ Xs)
{
    extern __shared__ double lds[];
    constexpr int G = 256 / NB;              /* row groups */
    const int W = 2 * bl + bu + 1;
    const int col = threadIdx.x % NB, grp = threadIdx.x / NB;
    const int q0 = blockIdx.x * NB;
    const int q = q0 + col;
    const bool on = q < nq;
    const int c0 = cols[q0];
    const int c = on ? cols[q] : -1;
    const int R1 = bl + NBP + 1, R2 = bl + bu + 1;
    double* red = lds;                       /* NBP x NB panel sums                     */
    double* win = lds + NBP * NB;            /* ring buffer                             */
    /* STAGE: the panel's multipliers (forward) / U rows (backward) are copied to LDS with
     * coalesced loads once per panel, so the inner loops read LDS instead of chains of
     * dependent global loads */
    double* ysh = win + (size_t)max(R1, R2) * NB;   /* NBP x NB forward results of a panel */
    double* stg = ysh + NBP * NB;
    /* ---- forward ---- */
    const int kst = (max(0, c0 - bl - NBP + 1) / NBP) * NBP;
    for (int r = kst + grp; r <= min(kst + NBP - 1 + bl, ncol - 1); r += G)
        win[(r % R1) * NB + col] = (r == c) ? 1.0 : 0.0;
    for (int k0 = kst; k0 < ncol; k0 += NBP) {
        const int nbk = min(NBP, ncol - k0);
        const int pend = min(k0 + nbk - 1 + bl, ncol - 1);
        const int nprow = pend - k0 + 1;
        const double* Lg = lpan + (int64_t)(k0 / NBP) * (NBP + bl) * NBP;
        if (STAGE)
            for (int e = threadIdx.x; e < nprow * NBP; e += 256) stg[e] = Lg[e];
        const double* Lp = STAGE ? stg : Lg;
        const int kb = k0 % R1;                  /* ring slot of row k0 */
        auto slot = [&](int r) { const int v = kb + r; return v >= R1 ? v - R1 : v; };  /* r < R1 */
        __syncthreads();
        if (grp == 0) {
            /* interchanges, then the unit-lower L11 solve, one column per lane */
            for (int t = 0; t < nbk; t++) {
                const int rp = piv[k0 + t] - k0;
                if (rp != t) {
                    double* a = win + slot(t) * NB + col;
                    double* b = win + slot(rp) * NB + col;
                    const double x = *a; *a = *b; *b = x;
                }
            }
            double y[NBP];
#pragma unroll
            for (int t = 0; t < NBP; t++) {
                if (t < nbk) {
                    double v = win[slot(t) * NB + col];
#pragma unroll
                    for (int u = 0; u < t; u++) v -= Lp[t * NBP + u] * y[u];
                    y[t] = v;
                    win[slot(t) * NB + col] = v;
                }
            }
        }
        __syncthreads();
        /* rows below the panel: -= L21 y (panel values held in registers) */
        {
            double y[NBP];
#pragma unroll
            for (int t = 0; t < NBP; t++) y[t] = t < nbk ? win[slot(t) * NB + col] : 0.0;
            for (int r = nbk + grp; r < nprow; r += G) {
                const double* lr = Lp + r * NBP;
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int t = 0; t < NBP; t += 2) {
                    a0 += lr[t] * y[t];
                    a1 += lr[t + 1] * y[t + 1];
                }
                win[slot(r) * NB + col] -= a0 + a1;
            }
        }
        /* panel rows are final: y -> X */
        for (int t = grp; t < nbk; t += G)
            if (on) Xs[(int64_t)(k0 + t) * nq + q] = win[slot(t) * NB + col];
        __syncthreads();
        for (int r = pend + 1 + grp; r <= min(k0 + 2 * NBP - 1 + bl, ncol - 1); r += G)
            win[(r % R1) * NB + col] = (r == c) ? 1.0 : 0.0;
    }
    if (grp == 0 && on)
        for (int r = 0; r < kst; r++) Xs[(int64_t)r * nq + q] = 0.0;
    /* ---- backward, panels from the bottom: ring of R2 = bl + bu + 1 rows ---- */
    __syncthreads();
    const int npan = (ncol + NBP - 1) / NBP;
    const int WU = bl + bu + 1;              /* staged U row: columns i .. i+bl+bu */
    for (int pn = npan - 1; pn >= 0; pn--) {
        const int i0 = pn * NBP, i1 = min(ncol, i0 + NBP);
        const int nr = i1 - i0;
        if (STAGE) {
            for (int e = threadIdx.x; e < nr * WU; e += 256) {
                const int rr = e / WU, jj = e % WU;
                const int i = i0 + rr;
                stg[e] = (i + jj < ncol) ? ab[(int64_t)i * W + bl + jj] : 0.0;
            }
            __syncthreads();
        }
        /* t_i = sum_{j >= i1} U_ij x_j for the panel rows (rows x column per thread);
         * the forward results y_i of the panel rows are fetched alongside */
        for (int e = grp; e < nr; e += G) {
            ysh[e * NB + col] = on ? Xs[(int64_t)(i0 + e) * nq + q] : 0.0;
            const int i = i0 + e;
            const int jend = min(i + bl + bu, ncol - 1);
            double s0 = 0.0, s1 = 0.0;
            const double* ur = STAGE ? stg + e * WU - i : ab + (int64_t)i * W + (bl - i);
            /* x_j sits at ring slot j % R2: walk the slots with a wrap instead of a modulo */
            int js = i1 % R2;
            int j = i1;
            for (; j + 1 <= jend; j += 2) {
                const int js1 = js + 1 == R2 ? 0 : js + 1;
                s0 += ur[j] * win[js * NB + col];
                s1 += ur[j + 1] * win[js1 * NB + col];
                js = js1 + 1 == R2 ? 0 : js1 + 1;
            }
            if (j <= jend) s0 += ur[j] * win[js * NB + col];
            red[e * NB + col] = s0 + s1;
        }
        __syncthreads();
        if (grp == 0) {
            for (int i = i1 - 1; i >= i0; i--) {
                const double* ar = STAGE ? stg + (i - i0) * WU - i : ab + (int64_t)i * W + (bl - i);
                double t = red[(i - i0) * NB + col];
                const int jend = min(i1 - 1, i + bl + bu);
                int js = (i + 1) % R2;
                for (int j = i + 1; j <= jend; j++) {
                    t += ar[j] * win[js * NB + col];
                    js = js + 1 == R2 ? 0 : js + 1;
                }
                const double yv = ysh[(i - i0) * NB + col];
                const double x = (yv - t) / ar[i];
                win[(i % R2) * NB + col] = x;
                if (on) Xs[(int64_t)i * nq + q] = x;
            }
        }
        __syncthreads();
    }
}

/* ---- apply ------------------------------------------------------------------------ */

/* The output z = r on identity rows (zall: and 0 on the others -- the T/S sweeps iterate
 * on z; otherwise the last dynamics pass and the T/S multigrid write every active row);
 * rr = r - A(:, known) r(known) on the others (slot bitmask), to the planar rrP and
 * (rr != null, the T/S sweeps) AoS.  The planar iterate zP is 0 on the identity rows and on
 * T/S (zeroed when the preconditioner is computed, never written there) and the first pass
 * writes its active dynamics rows before reading them, so the apply does not touch it here:
 * the identity rows' couplings are in rr, every kernel of the passes reads zP on the active
 * rows and the dynamics defect is rr - A zP over all its slots */
__global__ void k_gs_rr(const double* __restrict__ val, const uint8_t* __restrict__ known,
                        const uint64_t* __restrict__ kmask, const double* __restrict__ r,
                        double* __restrict__ z, double* __restrict__ rr, int zall,
                        double* __restrict__ rrP, Lay L)
{
    LAY_ALIASES;
    OWNED_CELL;
    double acc[NUN];
    bool kn[NUN];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        const int64_t row = NUN * cell + R;
        acc[R] = r[row];
        kn[R] = known[row] != 0;
        if (kn[R] || zall) z[row] = kn[R] ? acc[R] : 0.0;
    }
    uint64_t b[2] = {kmask[2 * cell], kmask[2 * cell + 1]};
    if (b[0] | b[1]) {
        for (int h = 0; h < 2; h++)
            while (b[h]) {
                const int s = 64 * h + __builtin_ctzll(b[h]);
                b[h] &= b[h] - 1;
                int R = 0;
                while (s >= ROW_BEGIN[R + 1]) R++;
                int ii = i + SLOTS[s].di, jj = j + SLOTS[s].dj;
                const int kk = k + SLOTS[s].dk;
                hnb(ii, jj, n, m, periodic);
                const int64_t col = NUN * ecell(L, ii, jj, kk) + SLOTS[s].var;
                acc[R] -= val[(int64_t)s * ncell + lc] * r[col];
            }
    }
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        const double v = kn[R] ? 0.0 : acc[R];
        if (rr) rr[NUN * cell + R] = v;
        rrP[PL(cell, R)] = v;
    }
}

/* k_gs_rr for a compressed input (FGMRES's Arnoldi vectors, krylov.hip): r is zero on every
 * identity row (land cells are not stored, the identity rows of active cells are 0), so the
 * identity-column couplings vanish and rr = r on the active rows; the output z is 0 on the
 * identity rows (zall: on every row) */
__global__ void k_gs_rr_c(const uint8_t* __restrict__ known, const int* __restrict__ cmap,
                          const double* __restrict__ rc, double* __restrict__ z, double* __restrict__ rr,
                          int zall, double* __restrict__ rrP, Lay L)
{
    LAY_ALIASES;
    OWNED_CELL;
    const int cm = cmap[lc];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        const int64_t row = NUN * cell + R;
        const bool kn = known[row] != 0;
        const double v = (kn || cm < 0) ? 0.0 : rc[(int64_t)NUN * cm + R];
        if (kn || zall) z[row] = 0.0;
        if (rr) rr[row] = v;
        rrP[PL(cell, R)] = v;
    }
}

/* per owned water column (i, j): 1 in flags[j n + i] if a P row of it is active, 1 in
 * flags[n m + j n + i] if a U or V row is (the host's Schur structure input; band_flags did
 * this on a host copy of all the flags) */
__global__ void k_band_flags(const uint8_t* __restrict__ known, Lay L, double* __restrict__ flags)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ncol = L.nloc / L.l;
    if (t >= ncol) return;
    const int il = (int)(t % L.nx), jl = (int)(t / L.nx);
    bool p = false, uv = false;
    for (int k = 0; k < L.l; k++) {
        const int64_t cell = L.own0 + ((int64_t)jl * L.l + k) * L.nx + il;
        p |= !known[NUN * cell + PP];
        uv |= !known[NUN * cell + UU] || !known[NUN * cell + VV];
    }
    const int64_t q = (int64_t)(L.jb0 + jl) * L.n + L.ib0 + il;
    if (p) flags[q] = 1.0;
    if (uv) flags[(int64_t)L.n * L.m + q] = 1.0;
}

/* the identity-row flags in the planar layout */
__global__ void k_known_planar(const uint8_t* __restrict__ known, uint8_t* __restrict__ knP, int64_t next)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= next) return;
#pragma unroll
    for (int R = 0; R < NUN; R++) knP[e + R * next] = known[NUN * e + R];
}

/* per cell: bitmask of the slots (104 bits) through which an active row couples to an
 * identity-row column (coast, sea floor, rigid lid); empty for most interior cells */
__global__ void k_knownmask(const double* __restrict__ val, const uint8_t* __restrict__ known,
                            uint64_t* __restrict__ kmask, Lay L, int jb1)
{
    LAY_ALIASES;
    OWNED_CELL;
    uint64_t b0 = 0, b1 = 0;
    int R = 0;
    for (int s = 0; s < NSLOT; s++) {
        while (s >= ROW_BEGIN[R + 1]) R++;
        if (known[NUN * cell + R] || val[(int64_t)s * ncell + lc] == 0.0) continue;
        int ii = i + SLOTS[s].di, jj = j + SLOTS[s].dj;
        const int kk = k + SLOTS[s].dk;
        if (kk < 0 || kk >= l || !hnb(ii, jj, n, m, periodic)) continue;
        if (jj < L.jb0 - 1 || jj > jb1) continue;   /* beyond the exchanged halo row */
        if (known[NUN * ecell(L, ii, jj, kk) + SLOTS[s].var]) {
            if (s < 64) b0 |= (uint64_t)1 << s;
            else b1 |= (uint64_t)1 << (s - 64);
        }
    }
    kmask[2 * cell] = b0;
    kmask[2 * cell + 1] = b1;
}

/* T/S off-diagonal couplings of active rows to active T/S columns, compacted:
 * per row (T, S) 6 same-variable neighbours (-i,+i,-j,+j,-k,+k) + the other variable at
 * k-1, k+1; zero where the column is an identity row, outside, or the row is inactive. */
constexpr int TS_NC = 16;
__global__ void k_ts_compact(const double* __restrict__ val, const uint8_t* __restrict__ known,
                             double* __restrict__ tsoff, Lay L, int64_t next, int64_t rowintcon)
{
    LAY_ALIASES;
    OWNED_CELL;
    for (int R = TT; R <= SS; R++) {
        const int base = ROW_BEGIN[R];
        const int other = R == TT ? SS : TT;
        const bool act = !known[NUN * cell + R] && NUN * cell + R != rowintcon;
        /* slots base+1..base+6: same var (-i,+i,-j,+j,-k,+k); base+18, base+19: other var k-1, k+1 */
        const int sl[8] = {base + 1, base + 2, base + 3, base + 4, base + 5, base + 6, base + 18, base + 19};
        for (int q = 0; q < 8; q++) {
            double v = 0.0;
            if (act) {
                const int s = sl[q];
                int ii = i + SLOTS[s].di, jj = j + SLOTS[s].dj;
                const int kk = k + SLOTS[s].dk;
                if (kk >= 0 && kk < l && hnb(ii, jj, n, m, periodic) &&
                    !known[NUN * ecell(L, ii, jj, kk) + (q < 6 ? R : other)])
                    v = val[(int64_t)s * ncell + lc];
            }
            tsoff[(int64_t)((R - TT) * 8 + q) * next + cell] = v;
        }
    }
}

__device__ __forceinline__ double duv_uv(const double* __restrict__ val, const uint8_t* __restrict__ knP,
                                         const double* __restrict__ z, int i, int j, int k,
                                         int64_t pl, const Lay& L);
/* Column kernels, transposed: one workgroup of 1024 threads per tile of COL_TI = 1024 / LP
 * consecutive columns of one latitude row (LP = power of two >= l), thread = (column, level)
 * with the column fastest, so every per-cell load of a wave runs along i in 128-byte runs
 * (the slot-major Jacobian rows and the planar dynamics vectors contiguously: with the
 * interleaved AoS vectors at a 48-byte cell stride the U/V and p/w kernels took 12.3 and
 * 12.6 against 7.2 and 6.9 us, scripts/ab/soa_probe.sh);
 * the column recurrences meet in LDS, where each thread composes the affine maps of the
 * levels it depends on (at most l steps of LDS reads).  At 2 degrees (LP = 16) 64-column
 * tiles, 232 workgroups: 16-column tiles (928 of 256 threads) measured 2 ms slower per
 * Newton step (scripts/ab_probe.py). */
template <int LP>
constexpr int col_ti() { return 1024 / LP; }
/* logical workgroup of block b for nwg workgroups launched as xcd_grid(nwg) blocks: the
 * XCDs (blocks dealt round robin, b % 8) get contiguous runs of workgroups, so tiles of
 * neighbouring latitude rows, which read each other's rows, share an L2; -1: idle block */
__device__ __forceinline__ int xcd_block(int nwg)
{
    const int per = (nwg + 7) >> 3;
    const int w = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    return w < nwg ? w : -1;
}
static inline unsigned xcd_grid(int64_t nwg) { return 8u * (unsigned)((nwg + 7) / 8); }

/* hr: the grid also covers the halo rows jl = -1 and jl = mb (latitude bands: the pass
 * recomputes the neighbours' edge values it reads instead of exchanging them) */
template <int LP>
__device__ __forceinline__ bool col_tile(const Lay& L, int& il, int& jl, int& k, bool& on, int hr = 0)
{
    constexpr int TI = col_ti<LP>();
    const int tpr = (L.nx + TI - 1) / TI;
    const int w = xcd_block(tpr * ((int)(L.nloc / ((int64_t)L.l * L.nx)) + 2 * hr));
    if (w < 0) return false;
    jl = w / tpr - hr;
    il = (w % tpr) * TI + (int)threadIdx.x % TI;
    k = (int)threadIdx.x / TI;
    on = k < L.l && il < L.nx;
    return true;
}

/* 4b/5. p = ptil + pbar and the continuity rows bottom-up, w_k = A_k + B_k w_k-1 (the
 * transposed column layout of k_gs_ptil_rcol); zo += omega (p, w) in the correction passes */
template <int LP>
__global__ void __launch_bounds__(1024) k_gs_pw_t(const double* __restrict__ val,
                                                  const uint8_t* __restrict__ knP,
                                                  const double* __restrict__ pbar,
                                                  double* __restrict__ z, Lay L,
                                                  const double* __restrict__ rr,
                                                  double* __restrict__ zo, double omega,
                                                  double* __restrict__ zaos)
{
    constexpr int TI = col_ti<LP>();
    __shared__ double sA[LP][TI], sB[LP][TI];
    int il, jl, k;
    bool on;
    if (!col_tile<LP>(L, il, jl, k, on)) return;    /* whole idle workgroups */
    const int ii = (int)threadIdx.x % TI;
    const int i = L.ib0 + il, j = L.jb0 + jl;
    const int64_t ncell = L.nloc;
    double A = 0.0, B = 0.0, pb = 0.0, zp = 0.0;
    bool pa = false, wa = false;
    int64_t cell = 0;
    if (on) {
        cell = ecell(L, i, j, k);
        const uint8_t kp = knP[PL(cell, PP)], kw = knP[PL(cell, WW)];
        pa = !kp;
        wa = !kw;
    }
    if (pa) {
        /* an inactive P row (land) reads nothing: its (A, B) = (0, 0) */
        const double a = val[(int64_t)S_PW0 * ncell + (cell - L.own0)];
        const double b = val[(int64_t)S_PWM * ncell + (cell - L.own0)];
        const double rhs = rr[PL(cell, PP)] - duv_uv(val, knP, z, i, j, k, cell - L.own0, L);
        pb = pbar[(int64_t)j * L.n + i];
        zp = z[PL(cell, PP)];
        if (wa && a != 0.0) {
            A = rhs / a;
            B = -b / a;
        }
    }
    if (k < LP) {
        sA[k][ii] = A;
        sB[k][ii] = B;
    }
    __syncthreads();
    if (!on) return;
    double w = 0.0;
    for (int kk = 0; kk <= k; kk++) w = sA[kk][ii] + sB[kk][ii] * w;
    const double pn = zp + pb, wn = pa ? w : 0.0;
    if (pa) z[PL(cell, PP)] = pn;
    if (wa) z[PL(cell, WW)] = wn;
    double fp = pn, fw = wn;
    if (zo) {
        if (pa) zo[PL(cell, PP)] = fp = zo[PL(cell, PP)] + omega * pn;
        if (wa) zo[PL(cell, WW)] = fw = zo[PL(cell, WW)] + omega * wn;
    }
    /* the last pass: the final P/W rows into the preconditioner output (AoS) */
    if (zaos) {
        if (pa) zaos[NUN * cell + PP] = fp;
        if (wa) zaos[NUN * cell + WW] = fw;
    }
}

/* Duv uv at a P cell: sum over the 4 U/V corners (P row slots 54..61) */
/* pl: owned index (Jacobian column) of the P cell */
__device__ __forceinline__ double duv_uv(const double* __restrict__ val, const uint8_t* __restrict__ knP,
                                         const double* __restrict__ z, int i, int j, int k,
                                         int64_t pl, const Lay& L)
{
    /* branch-free: a corner outside the domain reads the cell itself with weight 0 */
    const int n = L.n, m = L.m, periodic = L.periodic;
    const int64_t ncell = L.nloc, pc = pl;
    double acc = 0.0;
#pragma unroll
    for (int q4 = 0; q4 < 4; q4++) {
        int qi = i - (q4 & 1), qj = j - ((q4 >> 1) & 1);
        const bool in = hnb(qi, qj, n, m, periodic);
        if (!in) { qi = i; qj = j; }
        const int64_t qc = ecell(L, qi, qj, k);
        const uint8_t ku = knP[PL(qc, UU)], kv = knP[PL(qc, VV)];
        const double au = val[(int64_t)(S_PU + q4) * ncell + pc], av = val[(int64_t)(S_PV + q4) * ncell + pc];
        const double zu = z[PL(qc, UU)], zv = z[PL(qc, VV)];
        acc += (in && !ku) ? au * zu : 0.0;
        acc += (in && !kv) ? av * zv : 0.0;
    }
    return acc;
}

/* ---- the Schur right-hand side as a linear form in rr ----------------------------------
 * Steps 1-3a (ptil, uv*, the depth-weighted continuity defect) are linear in rr, so the
 * Schur right-hand side of water column (i, j) is a fixed combination of rr over its
 * neighbourhood: W rows of the 3 x 3 columns around it (through ptil, which the U/V points
 * of its four corners read), U/V rows of those corners, its own P rows.  The coefficients
 * are formed at set-up (k_rcol_uvp, k_rcol_w), so the apply evaluates ptil and the
 * right-hand side in one column kernel (k_gs_ptil_rcol) and the U/V points only once, after
 * the Schur solve (k_gs_uvp): two launches fewer per dynamics pass.
 * Layout: rcol[(e * l + k) * ncolb + t], t = band column (j - jb0) * nx + (i - ib0);
 * e < 9: rr_W at column (i + e % 3 - 1, j + e / 3 - 1), level k; e = 9 + q4 / 13 + q4: rr_U
 * / rr_V at corner q4 = (i - (q4 & 1), j - (q4 >> 1)); e = 17: rr_P at (i, j, k). */
constexpr int RC_NE = 18;

/* U/V and P coefficients, thread per (band column, level): with w_k the depth weight,
 * a the P row's couplings to its corners and D the corner's 2x2 U/V inverse, the column's
 * entry sum_k w_k (Duv uv* - rr_p) has d/d rr_U(q) = [ua] (cu d0 + cv d2), d/d rr_V(q) =
 * [va] (cu d1 + cv d3), cu = w_k a_U [in, ua], cv = w_k a_V [in, va]; d/d rr_P = -w_k. */
__global__ void k_rcol_uvp(const double* __restrict__ val, const uint8_t* __restrict__ known,
                           const double* __restrict__ uvinv, const double* __restrict__ pw,
                           double* __restrict__ rcol, Lay L)
{
    LAY_ALIASES;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int ncolb = (int)(L.nloc / l);
    if (g >= (int64_t)ncolb * l) return;
    const int t = (int)(g / l), k = (int)(g % l);
    const int i = L.ib0 + t % L.nx, j = L.jb0 + t / L.nx;
    const int64_t cell = ecell(L, i, j, k), pl = cell - L.own0, ncell = L.nloc;
    const bool pa = !known[NUN * cell + PP];
    const double w = pa ? pw[cell] : 0.0;
    /* coefficient e of level k: R[e * l * ncolb] */
    double* R = rcol + (int64_t)k * ncolb + t;
    const int64_t es = (int64_t)l * ncolb;
    for (int q4 = 0; q4 < 4; q4++) {
        int qi = i - (q4 & 1), qj = j - ((q4 >> 1) & 1);
        double cu_r = 0.0, cv_r = 0.0;
        if (pa && hnb(qi, qj, n, m, periodic)) {
            const int64_t qc = ecell(L, qi, qj, k);
            const bool ua = !known[NUN * qc + UU], va = !known[NUN * qc + VV];
            const double cu = ua ? w * val[(int64_t)(S_PU + q4) * ncell + pl] : 0.0;
            const double cv = va ? w * val[(int64_t)(S_PV + q4) * ncell + pl] : 0.0;
            const double* D = uvinv + 4 * qc;
            cu_r = ua ? cu * D[0] + cv * D[2] : 0.0;
            cv_r = va ? cu * D[1] + cv * D[3] : 0.0;
        }
        R[(9 + q4) * es] = cu_r;
        R[(13 + q4) * es] = cv_r;
    }
    R[17 * es] = pa ? -w : 0.0;
}

/* W coefficients, thread per (band column, neighbour column c'): with D_k the entry's
 * derivative in ptil(c', k) (through every corner U/V point of the column that reads
 * P(c', k)), and ptil(c', k) = A_k + B_k ptil(c', k+1), A_k = rr_W / g0, B_k = -g1 / g0 on
 * the active hydrostatic rows (0, 0 elsewhere), the coefficient of rr_W(c', k') is
 * S_k' / g0_k' with S_k' = S_k'-1 B_k'-1 + D_k'.  Reads the U/V coefficients of k_rcol_uvp. */
__global__ void k_rcol_w(const uint8_t* __restrict__ known, const double* __restrict__ gslot,
                         double* __restrict__ rcol, Lay L)
{
    LAY_ALIASES;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int ncolb = (int)(L.nloc / l);
    if (g >= (int64_t)ncolb * 9) return;
    const int t = (int)(g / 9), e = (int)(g % 9);
    const int i = L.ib0 + t % L.nx, j = L.jb0 + t / L.nx;
    const int di = e % 3 - 1, dj = e / 3 - 1;
    /* coefficient e of level k: R[(e * l + k) * ncolb] */
    double* R = rcol + t;
    const int64_t ks = ncolb;
    int gi = i + di, gj = j + dj;
    if (!hnb(gi, gj, n, m, periodic)) {
        for (int k = 0; k < l; k++) R[((int64_t)e * l + k) * ks] = 0.0;
        return;
    }
    double S = 0.0, Bprev = 0.0;
    for (int k = 0; k < l; k++) {
        const int64_t gc = ecell(L, gi, gj, k);
        const bool pa = !known[NUN * gc + PP], wa = !known[NUN * gc + WW];
        double D = 0.0;
        if (pa) {
            for (int q4 = 0; q4 < 4; q4++) {
                const int a = -(q4 & 1), b = -((q4 >> 1) & 1);
                const int ex = di - a, fy = dj - b;          /* c' as a P corner of q */
                if (ex < 0 || ex > 1 || fy < 0 || fy > 1) continue;
                int qi = i + a, qj = j + b;
                if (!hnb(qi, qj, n, m, periodic)) continue;
                const int64_t qc = ecell(L, qi, qj, k);
                const int g4 = ex + 2 * fy;
                D -= R[((int64_t)(9 + q4) * l + k) * ks] * gslot[GSL * qc + g4] +
                     R[((int64_t)(13 + q4) * l + k) * ks] * gslot[GSL * qc + 4 + g4];
            }
        }
        const double g0 = gslot[GSL * gc + 8], g1 = gslot[GSL * gc + 9];
        const bool act = pa && k < l - 1 && wa && g0 != 0.0;
        S = S * Bprev + D;
        R[((int64_t)e * l + k) * ks] = act ? S / g0 : 0.0;
        Bprev = act ? -g1 / g0 : 0.0;
    }
}

/* 1 + 3a. ptil (top-down: p_k = A_k + B_k p_k+1) and the column's Schur right-hand side
 * sum_e rcol_e rr_e (summed over the levels in a fixed order), written as k_gs_pcol wrote it */
/* gsl (latitude bands): the tiles of the halo rows jl = -1, mb (inside the grid) compute
 * ptil there too, with the W row's couplings from the halo-filled gslot (the owned Jacobian
 * has no halo rows), so that the U/V kernel needs no exchange of ptil */
/* RC = false: ptil only (a pass without the Schur solve needs no right-hand side for it) */
template <int LP, bool RC = true>
__global__ void __launch_bounds__(1024) k_gs_ptil_rcol(const double* __restrict__ val,
                                                       const uint8_t* __restrict__ knP,
                                                       const double* __restrict__ rcol,
                                                       const double* __restrict__ rr,
                                                       double* __restrict__ z,
                                                       const int* __restrict__ ocol,
                                                       double* __restrict__ colv_own, Lay L,
                                                       const double* __restrict__ gsl)
{
    LAY_ALIASES;
    constexpr int TI = col_ti<LP>();
    __shared__ double sA[LP][TI], sB[LP][TI], sv[LP][TI];
    int il, jl, k;
    bool on;
    if (!col_tile<LP>(L, il, jl, k, on, gsl ? 1 : 0)) return;    /* whole idle workgroups */
    const int ii = (int)threadIdx.x % TI;
    const int i = L.ib0 + il, j = L.jb0 + jl;
    const int mbl = (int)(L.nloc / ((int64_t)l * L.nx));
    if (jl < 0 || jl >= mbl) {
        /* a halo row: ptil only (rows outside the grid: whole idle workgroups) */
        if (j < 0 || j >= m) return;
        double A = 0.0, B = 0.0;
        bool pa = false;
        int64_t cell = 0;
        if (on) {
            cell = ecell(L, i, j, k);
            pa = !knP[PL(cell, PP)];
            if (pa && k < l - 1 && !knP[PL(cell, WW)]) {
                const double g0 = gsl[GSL * cell + 8], g1 = gsl[GSL * cell + 9];
                if (g0 != 0.0) {
                    A = rr[PL(cell, WW)] / g0;
                    B = -g1 / g0;
                }
            }
        }
        if (k < LP) {
            sA[k][ii] = A;
            sB[k][ii] = B;
        }
        __syncthreads();
        if (!on) return;
        double p = 0.0;
        for (int kk = l - 1; kk >= k; kk--) p = sA[kk][ii] + sB[kk][ii] * p;
        if (pa) z[PL(cell, PP)] = p;
        return;
    }
    const int64_t ncell = L.nloc;
    const int ncolb = (int)(L.nloc / l);
    const int t = jl * L.nx + il;
    double A = 0.0, B = 0.0, v = 0.0;
    bool pa = false;
    int64_t cell = 0;
    if (on) {
        cell = ecell(L, i, j, k);
        const uint8_t kp = knP[PL(cell, PP)], kw = knP[PL(cell, WW)];
        pa = !kp;
        if constexpr (RC) {
            int64_t nc9[9];
#pragma unroll
            for (int e = 0; e < 9; e++) {
                int i2 = i + e % 3 - 1, j2 = j + e / 3 - 1;
                if (!hnb(i2, j2, n, m, periodic)) { i2 = i; j2 = j; }
                nc9[e] = ecell(L, i2, j2, k);
            }
            const double* R = rcol + (int64_t)k * ncolb + t;
            const int64_t es = (int64_t)l * ncolb;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int e = 0; e < 9; e++) a0 += R[e * es] * rr[PL(nc9[e], WW)];
            if (pa) {
                /* the corner and own-P coefficients vanish on an inactive P row (land): not read */
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++) {
                    /* corner q4 = (i - (q4 & 1), j - (q4 >> 1)): neighbour (1 - (q4 >> 1)) * 3 + 1 - (q4 & 1) */
                    const int64_t qc = nc9[(1 - ((q4 >> 1) & 1)) * 3 + 1 - (q4 & 1)];
                    a1 += R[(9 + q4) * es] * rr[PL(qc, UU)];
                    a2 += R[(13 + q4) * es] * rr[PL(qc, VV)];
                }
                a2 += R[17 * es] * rr[PL(cell, PP)];
            }
            v = a0 + (a1 + a2);
        }
        if (pa) {
            if (k < l - 1 && !kw) {
                const double g0 = val[(int64_t)S_WP0 * ncell + (cell - L.own0)];
                const double g1 = val[(int64_t)S_WP1 * ncell + (cell - L.own0)];
                if (g0 != 0.0) {
                    A = rr[PL(cell, WW)] / g0;
                    B = -g1 / g0;
                }
            }
        }
    }
    if (k < LP) {
        sA[k][ii] = A;
        sB[k][ii] = B;
        if constexpr (RC) sv[k][ii] = v;
    }
    __syncthreads();
    if (!on) return;
    double p = 0.0;
    for (int kk = l - 1; kk >= k; kk--) p = sA[kk][ii] + sB[kk][ii] * p;
    if (pa) z[PL(cell, PP)] = p;
    if (RC && k == 0) {
        const int q = ocol[j * n + i];
        double s = 0.0;
        for (int kk = 0; kk < l; kk++) s += sv[kk][ii];
        if (q >= 0) colv_own[q] = s;
        else if (q != -1) colv_own[-2 - q] = 0.0;
    }
}

/* 3b. y = X b (X row-major nr x nc), one wavefront per row */
__global__ void __launch_bounds__(256) k_gemv(const double* __restrict__ X, int nr, int nc,
                                              const double* __restrict__ b, double* __restrict__ y)
{
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nr) return;
    const double* xr = X + (int64_t)row * nc;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int c = lane;
    for (; c + 192 < nc; c += 256) {
        s0 += xr[c] * b[c];
        s1 += xr[c + 64] * b[c + 64];
        s2 += xr[c + 128] * b[c + 128];
        s3 += xr[c + 192] * b[c + 192];
    }
    for (; c < nc; c += 64) s0 += xr[c] * b[c];
    double s = (s0 + s1) + (s2 + s3);
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0) y[row] = s;
}

/* y = X b for a dense row-major N x N inverse (N <= 64 NL), one wave per row: every load
 * of the row is issued before the first multiply, b staged in LDS, eight independent
 * accumulators and a fixed shuffle tree (deterministic) */
template <int NL>
__global__ void __launch_bounds__(256) k_gemv_w(const double* __restrict__ X, int N, const double* __restrict__ b,
                                                double* __restrict__ y)
{
    __shared__ double vb[64 * NL];
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const double* A = X + (size_t)(r < N ? r : 0) * N;
    double a[NL];
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int c = lane + 64 * u;
        a[u] = c < N ? __builtin_nontemporal_load(A + c) : 0.0;
    }
    for (int c = threadIdx.x; c < N; c += 256) vb[c] = b[c];
    __syncthreads();
    if (r >= N) return;
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int c = lane + 64 * u;
        if (c < N) acc[u & 7] += a[u] * vb[c];
    }
    double v = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) y[r] = v;
}

/* Minimal-residual defect correction: with d the defect and q = -A_DD zc the change a
 * full correction zc would make to it, the step w = argmin ||d + w q|| = -(d.q)/(q.q).
 * Block partials in a fixed order (deterministic), summed by one thread. */
constexpr int MR_NB = 256;
/* over the owned cells of the planar U/V/W/P planes (fixed grid-stride order) */
__global__ void __launch_bounds__(256) k_mr_dots(const double* __restrict__ d, const double* __restrict__ q,
                                                 Lay L, double* __restrict__ part)
{
    __shared__ double s0[256], s1[256];
    double a = 0.0, b = 0.0;
    const int64_t n = 4 * L.nloc;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = PL(L.own0 + t % L.nloc, t / L.nloc);
        const double qv = q[e];
        a += d[e] * qv;
        b += qv * qv;
    }
    s0[threadIdx.x] = a;
    s1[threadIdx.x] = b;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s0[threadIdx.x] += s0[threadIdx.x + w];
            s1[threadIdx.x] += s1[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s0[0];
        part[gridDim.x + blockIdx.x] = s1[0];
    }
}
__global__ void k_mr_sum(double* __restrict__ part, int nb)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double a = 0.0, b = 0.0;
    for (int e = 0; e < nb; e++) {
        a += part[e];
        b += part[nb + e];
    }
    part[2 * nb] = a;
    part[2 * nb + 1] = b;
}
/* z += w zc, and (upd) d += w q, on the active U/V/W/P rows (planar); zaos: the final
 * values into the preconditioner output (AoS) */
__global__ void k_mr_update(const uint8_t* __restrict__ knP, const double* __restrict__ sums,
                            const double* __restrict__ zc, const double* __restrict__ q,
                            double* __restrict__ z, double* __restrict__ d, Lay L, int upd,
                            double* __restrict__ zaos)
{
    OWNED_CELL;
    const double w = sums[1] > 0.0 ? -sums[0] / sums[1] : 0.0;
#pragma unroll
    for (int R = UU; R <= PP; R++) {
        const int64_t e = PL(cell, R);
        if (knP[e]) continue;
        const double zn = z[e] + w * zc[e];
        z[e] = zn;
        if (upd) d[e] += w * q[e];
        if (zaos) zaos[NUN * cell + R] = zn;
    }
}

/* 2 + 4. uv = D^-1 (rr_uv - Guv (ptil + Mz1^T pbar)) in one pass once pbar is known (the
 * Schur right-hand side came from rcol, so uv* is never formed); zo += omega uv */
/* gsl (latitude bands): threads past the owned cells compute the south halo row's U/V
 * points too (their P couplings from the halo-filled gslot), into z only, so that the p/w
 * kernel needs no exchange of uv */
/* alist: the threads run over the active cells (nown of them; BlockGS::act), the land
 * cells' U/V points being identity rows */
__global__ void k_gs_uvp(const double* __restrict__ val, const uint8_t* __restrict__ knP,
                         const double* __restrict__ uvinv, const double* __restrict__ rr,
                         const double* __restrict__ pbar, double* __restrict__ z, Lay L,
                         double* __restrict__ zo, double omega, double* __restrict__ zaos,
                         const double* __restrict__ gsl, const int* __restrict__ alist, int64_t nown)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ncell = L.nloc;
    const int n = L.n, m = L.m, periodic = L.periodic;
    int i, j, k;
    int64_t cell, lc = 0;
    const bool halo = t >= nown;
    if (!halo) {
        lc = alist ? (int64_t)alist[t] : t;
        cell = L.own0 + lc;
        lc_ijk(L, lc, i, j, k);
    } else {
        const int64_t q = t - nown;                  /* south halo row, (k, i) */
        if (!gsl || q >= (int64_t)L.l * L.nx || L.jb0 == 0) return;
        i = L.ib0 + (int)(q % L.nx);
        k = (int)(q / L.nx);
        j = L.jb0 - 1;
        cell = ecell(L, i, j, k);
    }
    const uint8_t ku = knP[PL(cell, UU)], kv = knP[PL(cell, VV)];
    const bool ua = !ku, va = !kv;
    if (!ua && !va) return;                 /* land: none of the point's operands is read */
    double gu = 0.0, gv = 0.0;
#pragma unroll
    for (int g4 = 0; g4 < 4; g4++) {
        int pi = i + (g4 & 1), pj = j + ((g4 >> 1) & 1);
        const bool in = hnb(pi, pj, n, m, periodic);
        if (!in) { pi = i; pj = j; }
        const int64_t pc = ecell(L, pi, pj, k);
        const uint8_t kp = knP[PL(pc, PP)];
        const double p = z[PL(pc, PP)] + pbar[(int64_t)pj * n + pi];
        const double au = halo ? gsl[GSL * cell + g4] : val[(int64_t)(S_UP + g4) * ncell + lc];
        const double av = halo ? gsl[GSL * cell + 4 + g4] : val[(int64_t)(S_VP + g4) * ncell + lc];
        const bool use = in && !kp;
        gu += use ? au * p : 0.0;
        gv += use ? av * p : 0.0;
    }
    const double* D = uvinv + 4 * cell;
    const double d0 = D[0], d1 = D[1], d2 = D[2], d3 = D[3];
    const double r0 = rr[PL(cell, UU)], r1 = rr[PL(cell, VV)];
    const double ru = ua ? r0 - gu : 0.0;
    const double rv = va ? r1 - gv : 0.0;
    const double nu = d0 * ru + d1 * rv, nv = d2 * ru + d3 * rv;
    if (ua) z[PL(cell, UU)] = nu;
    if (va) z[PL(cell, VV)] = nv;
    if (halo) {
        /* the pass iterate's south halo row too (the T/S right-hand side reads its U/V) */
        if (zo && ua) zo[PL(cell, UU)] += omega * nu;
        if (zo && va) zo[PL(cell, VV)] += omega * nv;
        return;
    }
    double fu = nu, fv = nv;
    if (zo) {
        if (ua) zo[PL(cell, UU)] = fu = zo[PL(cell, UU)] + omega * nu;
        if (va) zo[PL(cell, VV)] = fv = zo[PL(cell, VV)] + omega * nv;
    }
    /* the last pass: the final U/V rows into the preconditioner output (AoS) */
    if (zaos) {
        if (ua) zaos[NUN * cell + UU] = fu;
        if (va) zaos[NUN * cell + VV] = fv;
    }
}

/* 6a. T/S right-hand side: rr_ts - B_ts,(u,v,w) z;  z_ts = 0 */
__global__ void k_gs_bts(const double* __restrict__ val, const uint8_t* __restrict__ known,
                         const double* __restrict__ rr, double* __restrict__ z, double* __restrict__ bts,
                         Lay L)
{
    LAY_ALIASES;
    OWNED_CELL;
    for (int R = TT; R <= SS; R++) {
        const int64_t row = NUN * cell + R;
        if (known[row]) continue;
        double acc = rr[row];
        for (int s = ROW_BEGIN[R]; s < ROW_BEGIN[R + 1]; s++) {
            const int var = SLOTS[s].var;
            if (var == TT || var == SS) continue;
            const double v = val[(int64_t)s * ncell + lc];
            if (v == 0.0) continue;
            int ii = i + SLOTS[s].di, jj = j + SLOTS[s].dj;
            const int kk = k + SLOTS[s].dk;
            if (kk < 0 || kk >= l || !hnb(ii, jj, n, m, periodic)) continue;
            const int64_t col = NUN * ecell(L, ii, jj, kk) + var;
            if (!known[col]) acc -= v * z[col];
        }
        bts[row] = acc;
        z[row] = 0.0;
    }
}

/* colour of a cell for the T/S sweeps: parity of i+j+k (global j); on a periodic grid with
 * odd n the wrap pairs (n-1, 0) would share a colour, so column i = n-1 gets colours 2/3 */
__device__ __forceinline__ int ts_color(int i, int j, int k, int n, int periodic)
{
    if (periodic && (n & 1) && i == n - 1) return 2 + ((j + k) & 1);
    return (i + j + k) & 1;
}

/* 6b. one red-black half sweep on the T/S block with 2x2 cell blocks (compact couplings;
 * generic layout, used for odd n) */
__global__ void __launch_bounds__(256) k_gs_ts_half(const double* __restrict__ tsoff,
                                                    const uint8_t* __restrict__ known,
                                                    const double* __restrict__ tsinv,
                                                    const double* __restrict__ bts,
                                                    double* __restrict__ z, Lay L, int64_t next,
                                                    int color)
{
    LAY_ALIASES;
    OWNED_CELL;
    if (ts_color(i, j, k, n, periodic) != color) return;
    const bool ta = !known[NUN * cell + TT], sa = !known[NUN * cell + SS];
    if (!ta && !sa) return;
    /* neighbour cells (clamped where the coupling is zero anyway) */
    int im = i - 1, ip = i + 1;
    if (periodic) { if (im < 0) im = n - 1; if (ip >= n) ip = 0; }
    else { if (im < 0) im = i; if (ip >= n) ip = i; }
    const int jm = j > 0 ? j - 1 : j, jp = j < m - 1 ? j + 1 : j;
    const int km = k > 0 ? k - 1 : k, kp = k < l - 1 ? k + 1 : k;
    const int64_t nb[6] = {ecell(L, im, j, k), ecell(L, ip, j, k), ecell(L, i, jm, k),
                           ecell(L, i, jp, k), ecell(L, i, j, km), ecell(L, i, j, kp)};
    double res[2];
#pragma unroll
    for (int R = 0; R < 2; R++) {
        const int var = TT + R, oth = SS - R;
        const double* a = tsoff + (int64_t)(R * 8) * next + cell;
        double acc = bts[NUN * cell + var];
#pragma unroll
        for (int q = 0; q < 6; q++) acc -= a[(int64_t)q * next] * z[NUN * nb[q] + var];
        acc -= a[(int64_t)6 * next] * z[NUN * nb[4] + oth];
        acc -= a[(int64_t)7 * next] * z[NUN * nb[5] + oth];
        res[R] = acc;
    }
    const double* D = tsinv + 4 * cell;
    if (ta) z[NUN * cell + TT] = D[0] * res[0] + D[1] * res[1];
    if (sa) z[NUN * cell + SS] = D[2] * res[0] + D[3] * res[1];
}

/* Even n: the owned cells of one colour are lc = 2q + ((j+k+c)&1) (lc = (row)*n + i with
 * row = (j-jb0)*l + k), so every per-cell T/S array can be stored per colour and read
 * contiguously by a half sweep:  tsc[(c*16 + e)*half + q] couplings,
 * tic[(c*4 + e)*half + q] 2x2 inverses, bc[(c*2 + v)*half + q] right-hand sides;
 * zt / zs: T and S iterates by ext cell (halo entries stay 0). */
__global__ void k_ts_pack(const double* __restrict__ tsoff, const double* __restrict__ tsinv,
                          double* __restrict__ tsc, double* __restrict__ tic, Lay L, int64_t next)
{
    OWNED_CELL;
    const int64_t half = ncell / 2;
    const int c = (i + j + k) & 1;
    const int64_t q = lc >> 1;
    for (int e = 0; e < TS_NC; e++) tsc[(int64_t)(c * TS_NC + e) * half + q] = tsoff[(int64_t)e * next + cell];
    for (int e = 0; e < 4; e++) tic[(int64_t)(c * 4 + e) * half + q] = tsinv[4 * cell + e];
}

/* T/S right-hand side bts = rr_TS - A_TS,D z_D into the colour layout and bts; zt = zs = 0.
 * One wave per (64 cells, T or S row): the row's 10 dynamics slots unrolled at compile
 * time, neighbour indices clamped as in the SpMV (the ELL holds zeros outside the domain),
 * identity-row columns (their couplings are in rr already) skipped by the slot bitmask
 * kmask instead of a byte gather per slot.  Dealt to the XCDs in contiguous runs. */
template <int R>
__device__ __forceinline__ double bts_row(const double* __restrict__ val, const double* __restrict__ z,
                                          int64_t lc, int64_t nloc, const int (*nc)[9],
                                          uint64_t kbits, double acc, int64_t zcell = NUN, int64_t zvar = 1)
{
    /* z(cell, var) = z[zcell cell + zvar var]: (NUN, 1) AoS, (1, plane stride) planar */
    constexpr int B = RowInfo<R>::B, NS = RowInfo<R>::NS;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const Slot sl = SLOTS[B + s];
        if (sl.var == TT || sl.var == SS) continue;
        /* identity-row columns (coupling already in rr) weigh 0: no branch, so the loads of
         * all the row's slots issue together (default load policy: non-temporal loads made
         * the T/S solve 6.5 us slower, scripts/ab_probe.py) */
        const double v = ((kbits >> (B + s - 64)) & 1) ? 0.0 : val[(int64_t)(B + s) * nloc + lc];
        const int cidx = nc[sl.di + 1][(sl.dk + 1) * 3 + (sl.dj + 1)];
        acc -= v * z[zcell * (int64_t)cidx + zvar * sl.var];
    }
    return acc;
}
__global__ void __launch_bounds__(128) k_gs_bts2(const double* __restrict__ val, const uint8_t* __restrict__ known,
                                                 const uint64_t* __restrict__ kmask,
                                                 const double* __restrict__ rr, const double* __restrict__ z,
                                                 double* __restrict__ bc, double* __restrict__ zt,
                                                 double* __restrict__ zs, Lay L, double* __restrict__ bts,
                                                 int nblk)
{
    LAY_ALIASES;
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int64_t lc = (int64_t)tile * 64 + (threadIdx.x & 63);
    if (lc >= L.nloc) return;
    const int R = TT + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int i, j, k;
    lc_ijk(L, lc, i, j, k);
    const int64_t cell = L.own0 + lc;
    int nc[3][9];
    nb_cells(sub_of(L), i - L.ib0, j, k, nc);
    const int64_t row = NUN * cell + R;
    double acc = 0.0;
    if (!known[row]) {
        const uint64_t kb = kmask[2 * cell + 1];
        acc = R == TT ? bts_row<TT>(val, z, lc, L.nloc, nc, kb, rr[row])
                      : bts_row<SS>(val, z, lc, L.nloc, nc, kb, rr[row]);
    }
    const int64_t half = L.nloc / 2;
    const int c = (i + j + k) & 1;
    bc[(int64_t)(c * 2 + (R - TT)) * half + (lc >> 1)] = acc;
    bts[row] = acc;
    if (R == TT) zt[cell] = 0.0;
    else zs[cell] = 0.0;
}

__global__ void __launch_bounds__(256) k_gs_ts_half_c(const double* __restrict__ tsc,
                                                      const double* __restrict__ tic,
                                                      const double* __restrict__ bc,
                                                      double* __restrict__ zt, double* __restrict__ zs,
                                                      Lay L, int c)
{
    LAY_ALIASES;
    const int64_t half = L.nloc / 2;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= half) return;
    const int nx = L.nx;
    const int64_t row = (2 * q) / nx;                /* (j - jb0) * l + k */
    const int k = (int)(row % l), j = L.jb0 + (int)(row / l);
    const int64_t lc = 2 * q + ((j + k + c) & 1);    /* ib0 even: local parity = global */
    const int il = (int)(lc - row * nx);
    const int64_t cell = L.own0 + lc;
    const int64_t r = row + (int64_t)HALO * l;
    const int64_t ln = (int64_t)l * nx;
    const int64_t nb[6] = {xnb_cell(r, il - 1, n, L.ib0, nx, L.hx, periodic, L.xb),
                           xnb_cell(r, il + 1, n, L.ib0, nx, L.hx, periodic, L.xb),
                           j > 0 ? cell - ln : cell, j < m - 1 ? cell + ln : cell,
                           k > 0 ? cell - nx : cell, k < l - 1 ? cell + nx : cell};
    const double* a = tsc + (int64_t)(c * TS_NC) * half + q;
    double rt = bc[(int64_t)(c * 2) * half + q], rs = bc[(int64_t)(c * 2 + 1) * half + q];
#pragma unroll
    for (int e = 0; e < 6; e++) {
        rt -= a[(int64_t)e * half] * zt[nb[e]];
        rs -= a[(int64_t)(8 + e) * half] * zs[nb[e]];
    }
    rt -= a[(int64_t)6 * half] * zs[nb[4]] + a[(int64_t)7 * half] * zs[nb[5]];
    rs -= a[(int64_t)14 * half] * zt[nb[4]] + a[(int64_t)15 * half] * zt[nb[5]];
    const double* D = tic + (int64_t)(c * 4) * half + q;
    zt[cell] = D[0] * rt + D[half] * rs;
    zs[cell] = D[2 * half] * rt + D[3 * half] * rs;
}

/* z(T,S) = zt, zs on the active rows */
__global__ void k_ts_scatter(const uint8_t* __restrict__ known, const double* __restrict__ zt,
                             const double* __restrict__ zs, double* __restrict__ z, Lay L)
{
    OWNED_CELL;
    if (!known[NUN * cell + TT]) z[NUN * cell + TT] = zt[cell];
    if (!known[NUN * cell + SS]) z[NUN * cell + SS] = zs[cell];
}

/* ---- T/S aggregation multigrid ----------------------------------------------------
 * The T/S block is an advection-diffusion operator whose smooth error modes Gauss-Seidel
 * sweeps barely touch.  Its coarse spaces aggregate 2x2 horizontal neighbours over the
 * full depth (each level is again an n x m x l grid with the fine coupling pattern:
 * 6 same-variable face couplings, T<->S at k-1/k+1, a 2x2 cell block), built by Galerkin
 * summation with piecewise-constant transfers.  Aggregates stay inside a latitude band.
 * One V-cycle: z-line relaxation by horizontal colour on every level (colours forward
 * before the coarse correction, backward after it), a dense inverse on the coarsest.
 *
 * Level layout (level 0 included, packed once per Jacobian): columns k-contiguous,
 *     cell = ((jl + hj) * n + i) * l + k,
 * so the P lanes of a column (lane = level k) read one contiguous run of every array and
 * a horizontal neighbour is again one whole run (one 128-B line per array at l = 16);
 * with hj = 1 halo row on each side and hi = 1 halo column (the row width is n + 2 hi) on
 * level 0 when the y / x direction is split over ranks (refreshed by exchanges).
 * The z-lines are factorised at set-up (block Thomas, k_mg_fac: F = -A'^-1 B, A'^-1,
 * Cp = A'^-1 C per cell), so a relaxation is two affine parallel scans over the lanes
 * without a division.  Launch fusion (the apply is latency-bound):
 *   - the T/S right-hand side and the first colour of level 0 (k_mg_entry),
 *   - each restriction and the first colour of the coarse level (k_mg_rc): from a zero
 *     iterate that colour's lines see zero neighbours,
 *   - the prolongation into the first post-smoothing colour (k_mg_zl, corr): a line solve
 *     never reads its own old value, so the coarse correction is only needed on the
 *     neighbours not yet relaxed, and it is added where they are read,
 *   - after one forward sweep from zero with two colours, the residual of the last colour
 *     is zero and that of the first is -H z(last colour) (restriction shortcut: 16 instead
 *     of 72 doubles per fine-cell pair),
 *   - the last colour launches of the final level-0 sweep write z(T, S) straight into the
 *     preconditioner output. */
struct TsLev {
    int n, mb, l, periodic;          /* periodic: the level wraps in x (one x part)        */
    int hj, hi;                      /* halo rows / columns of the layout (level 0, split)  */
    int vis, visi;                   /* halo rows / columns the smoother / residual read    */
    int jpar;                        /* colour parity of (0, 0) (global i + j, level 0)     */
    int64_t cstr;                    /* array stride (mb + 2 hj) (n + 2 hi) l              */
    const double* off;               /* 16 x cstr: T row q 0..7, S row q 8..15            */
    const double* diag;              /* 4 x cstr: 2x2 block (TT, TS, ST, SS)              */
    const double* fac;               /* 12 x cstr: line factors F | A'^-1 | Cp            */
    double* b;                       /* 2 x cstr: right-hand side (T, S)                  */
    double* z;                       /* 2 x cstr: iterate (T, S)                          */
};
__host__ __device__ __forceinline__ int64_t mg_cell(const TsLev& V, int i, int jl, int k)
{
    return (((int64_t)jl + V.hj) * (V.n + 2 * V.hi) + i + V.hi) * V.l + k;
}
/* neighbour q (-i,+i,-j,+j,-k,+k) of (i,jl,k): false outside the level's (visible) band */
__device__ __forceinline__ bool mg_nb(const TsLev& V, int q, int& i, int& jl, int& k)
{
    switch (q) {
    case 0: i--; break;
    case 1: i++; break;
    case 2: jl--; break;
    case 3: jl++; break;
    case 4: k--; break;
    default: k++; break;
    }
    if (jl < -V.vis || jl >= V.mb + V.vis || k < 0 || k >= V.l) return false;
    if (i < -V.visi || i >= V.n + V.visi) {
        if (!V.periodic) return false;
        i = (i + V.n) % V.n;
    }
    return true;
}
/* the same neighbour, branch-free for the apply: outside the level's (visible) band the
 * cell itself (every coupling to outside is 0: k_ts_compact / k_mg_galerkin), so the loads
 * of all neighbours issue together */
__device__ __forceinline__ void mg_nbc(const TsLev& V, int q, int& i, int& jl, int& k)
{
    switch (q) {
    case 0: i = i > -V.visi ? i - 1 : (V.periodic ? V.n - 1 : i); break;
    case 1: i = i < V.n - 1 + V.visi ? i + 1 : (V.periodic ? 0 : i); break;
    case 2: jl = jl > -V.vis ? jl - 1 : jl; break;
    case 3: jl = jl < V.mb - 1 + V.vis ? jl + 1 : jl; break;
    case 4: k = k > 0 ? k - 1 : k; break;
    default: k = k < V.l - 1 ? k + 1 : k; break;
    }
}
/* off-diagonal part of row (T, S) of cell (i,jl,k) applied to the iterate */
__device__ __forceinline__ void mg_offmul(const TsLev& V, int i, int jl, int k, int64_t c,
                                          double& at, double& as)
{
    const int64_t cs = V.cstr;
    at = as = 0.0;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        int ii = i, jj = jl, kk = k;
        mg_nbc(V, q, ii, jj, kk);
        const int64_t nc = mg_cell(V, ii, jj, kk);
        at += V.off[(int64_t)q * cs + c] * V.z[nc];
        as += V.off[(int64_t)(8 + q) * cs + c] * V.z[cs + nc];
        if (q == 4) {
            at += V.off[6 * cs + c] * V.z[cs + nc];
            as += V.off[14 * cs + c] * V.z[nc];
        } else if (q == 5) {
            at += V.off[7 * cs + c] * V.z[cs + nc];
            as += V.off[15 * cs + c] * V.z[nc];
        }
    }
}
/* colour of water column (i, jl): parity of i + j (global j on level 0); on a periodic
 * level with odd n the wrap pair (n-1, 0) would share a colour, so column n-1 gets 2 / 3 */
__host__ __device__ __forceinline__ int mg_ncolour(const TsLev& V) { return (V.periodic && (V.n & 1)) ? 4 : 2; }
__device__ __forceinline__ int mg_lcolour(const TsLev& V, int i, int jl)
{
    if (V.periodic && (V.n & 1) && i == V.n - 1) return 2 + ((jl + V.jpar) & 1);
    return (i + jl + V.jpar) & 1;
}
/* g-th owned column of a colour: row jl holds i = 2h + ((colour + jl + jpar) & 1), h <
 * ceil(n'/2), n' = n - 1 on an odd periodic level (whose last column has colour 2 or 3).
 * hr (bands' level 0): the rows run from -1 to mb, the halo row -1 when hr & 1, mb when
 * hr & 2 (the parity of a negative jl is that of the global row too) */
__device__ __forceinline__ bool mg_column(const TsLev& V, int colour, int g, int& i, int& jl, int hr = 0)
{
    const int np = (V.periodic && (V.n & 1)) ? V.n - 1 : V.n;
    const int rows = V.mb + (hr ? 2 : 0), j0 = hr ? -1 : 0;
    if (colour < 2) {
        const int per_row = (np + 1) / 2;
        if (g >= per_row * rows) return false;
        jl = g / per_row + j0;
        i = 2 * (g % per_row) + ((colour + jl + V.jpar) & 1);
    } else {
        if (g >= rows) return false;
        jl = g + j0;
        i = V.n - 1;
        if (((jl + V.jpar) & 1) != colour - 2) return false;
    }
    if ((jl < 0 && !(hr & 1)) || (jl >= V.mb && !(hr & 2))) return false;
    return i < np || colour >= 2;
}
__host__ __device__ __forceinline__ int64_t mg_columns_of(const TsLev& V, int colour, int hr = 0)
{
    const int np = (V.periodic && (V.n & 1)) ? V.n - 1 : V.n;
    const int rows = V.mb + (hr ? 2 : 0);
    return colour < 2 ? (int64_t)((np + 1) / 2) * rows : rows;
}

/* Line solve of one column, lane = level k (< l when on): g = A'^-1 r, then the forward
 * recurrence dp_k = F_k dp_{k-1} + g_k and the backward x_k = dp_k - Cp_k x_{k+1} as affine
 * Hillis-Steele scans over the P lanes (log2 P shuffle steps of 2x2 algebra each, no
 * division: the pivots were inverted at set-up).  The factor loads are issued first. */
/* the 12 line factors of a lane (0 when !on), loadable ahead of the right-hand side */
struct LineFac {
    double a0, a1, a2, a3, i0, i1, i2, i3, q0, q1, q2, q3;
};
__device__ __forceinline__ LineFac line_fac(const double* __restrict__ f, int64_t cs, bool on)
{
    LineFac F{};
    if (on) {
        F.a0 = f[0]; F.a1 = f[cs]; F.a2 = f[2 * cs]; F.a3 = f[3 * cs];
        F.i0 = f[4 * cs]; F.i1 = f[5 * cs]; F.i2 = f[6 * cs]; F.i3 = f[7 * cs];
        F.q0 = -f[8 * cs]; F.q1 = -f[9 * cs]; F.q2 = -f[10 * cs]; F.q3 = -f[11 * cs];
    }
    return F;
}
template <int P>
__device__ __forceinline__ void line_run(const LineFac& F, int k, double rt, double rs, double& xt, double& xs);
template <int P>
__device__ __forceinline__ void line_solve(const double* __restrict__ f, int64_t cs, bool on, int k,
                                           double rt, double rs, double& xt, double& xs)
{
    line_run<P>(line_fac(f, cs, on), k, rt, rs, xt, xs);
}
template <int P>
__device__ __forceinline__ void line_run(const LineFac& F, int k, double rt, double rs, double& xt, double& xs)
{
    double a0 = F.a0, a1 = F.a1, a2 = F.a2, a3 = F.a3;
    const double i0 = F.i0, i1 = F.i1, i2 = F.i2, i3 = F.i3;
    double q0 = F.q0, q1 = F.q1, q2 = F.q2, q3 = F.q3;
    double ct = i0 * rt + i1 * rs, cv = i2 * rt + i3 * rs;
#pragma unroll
    for (int d = 1; d < P; d <<= 1) {
        const double b0 = __shfl_up(a0, d, P), b1 = __shfl_up(a1, d, P);
        const double b2 = __shfl_up(a2, d, P), b3 = __shfl_up(a3, d, P);
        const double dt = __shfl_up(ct, d, P), dv = __shfl_up(cv, d, P);
        if (k >= d) {
            const double nt = ct + (a0 * dt + a1 * dv), nv = cv + (a2 * dt + a3 * dv);
            const double n0 = a0 * b0 + a1 * b2, n1 = a0 * b1 + a1 * b3;
            const double n2 = a2 * b0 + a3 * b2, n3 = a2 * b1 + a3 * b3;
            ct = nt; cv = nv; a0 = n0; a1 = n1; a2 = n2; a3 = n3;
        }
    }
#pragma unroll
    for (int d = 1; d < P; d <<= 1) {
        const double b0 = __shfl_down(q0, d, P), b1 = __shfl_down(q1, d, P);
        const double b2 = __shfl_down(q2, d, P), b3 = __shfl_down(q3, d, P);
        const double dt = __shfl_down(ct, d, P), dv = __shfl_down(cv, d, P);
        if (k + d < P) {
            const double nt = ct + (q0 * dt + q1 * dv), nv = cv + (q2 * dt + q3 * dv);
            const double n0 = q0 * b0 + q1 * b2, n1 = q0 * b1 + q1 * b3;
            const double n2 = q2 * b0 + q3 * b2, n3 = q2 * b1 + q3 * b3;
            ct = nt; cv = nv; q0 = n0; q1 = n1; q2 = n2; q3 = n3;
        }
    }
    xt = ct;
    xs = cv;
}

/* z-line relaxation of one colour: every column of it solves its 2x2-block tridiagonal T/S
 * system along k with the horizontal couplings taken from the current iterate.  corr: the
 * first post-smoothing colour launch, neighbours not yet relaxed in this sweep (smaller
 * colour) read with their aggregate's coarse correction C.z added.  zout (level 0, final
 * sweep): the active T/S rows of the preconditioner output (ext layout) get the result. */
/* the line solve of column (i, jl) of the given colour from the current iterate (level k of
 * this lane; on: k < l); corr: neighbours of a smaller colour read with their aggregate's
 * coarse correction C.z added.  Returns the cell index (0 when !on). */
template <int P>
__device__ __forceinline__ int64_t zl_col(const TsLev& V, int i, int jl, int k, bool on, int colour,
                                          const TsLev& C, int corr, double& xt, double& xs)
{
    const int64_t cs = V.cstr;
    int64_t c = 0;
    double rt = 0.0, rs = 0.0;
    if (on) {
        c = mg_cell(V, i, jl, k);
        rt = V.b[c];
        rs = V.b[cs + c];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int ii = i, jj = jl, kk = k;
            mg_nbc(V, q, ii, jj, kk);
            const int64_t nc = mg_cell(V, ii, jj, kk);
            double zt = V.z[nc], zs = V.z[cs + nc];
            if (corr && mg_lcolour(V, ii, jj) < colour) {
                const int64_t p = mg_cell(C, ii >> 1, jj >> 1, k);
                zt += C.z[p];
                zs += C.z[C.cstr + p];
            }
            rt -= V.off[(int64_t)q * cs + c] * zt;
            rs -= V.off[(int64_t)(8 + q) * cs + c] * zs;
        }
    }
    line_solve<P>(V.fac + c, cs, on, k, rt, rs, xt, xs);
    return c;
}

template <int P>
__device__ __forceinline__ void zl_one(const TsLev& V, int colour, int g, int k, const TsLev& C, int corr,
                                       double* __restrict__ zout, int hr)
{
    int i, jl;
    if (!mg_column(V, colour, g, i, jl, hr)) return;       /* whole column groups exit */
    const int64_t cs = V.cstr;
    const bool on = k < V.l;
    double xt, xs;
    const int64_t c = zl_col<P>(V, i, jl, k, on, colour, C, corr, xt, xs);
    if (!on) return;
    V.z[c] = xt;
    V.z[cs + c] = xs;
    if (zout && jl >= 0 && jl < V.mb) {
        const int64_t e = NUN * ((((int64_t)jl + HALO) * V.l + k) * V.n + i);
        if (V.diag[c] != 0.0) zout[e + TT] = xt;
        if (V.diag[3 * cs + c] != 0.0) zout[e + SS] = xs;
    }
}
template <int P>
__global__ void __launch_bounds__(256) k_mg_zl(TsLev V, int colour, TsLev C, int corr,
                                              double* __restrict__ zout, int hr)
{
    zl_one<P>(V, colour, (blockIdx.x * blockDim.x + threadIdx.x) / P, threadIdx.x % P, C, corr, zout, hr);
}

/* Restriction F -> C (coarse rhs = sum of the children's residuals, fixed order
 * (c00 + c10) + (c01 + c11)) and, when relax, the coarse level's colour-0 lines from the
 * zero iterate (zero neighbours), the other coarse cells' iterate set to 0.  P lanes per
 * coarse column (lane = level k), every lane reads its four children's level k.
 * shortcut: F was relaxed once, colour 0 then 1, from a zero iterate, so the residual of
 * colour 1 is 0 and that of colour 0 is -H z (its horizontal neighbours). */
template <int P>
__device__ __forceinline__ void rc_one(const TsLev& F, const TsLev& C, int g, int k, int shortcut, int relax)
{
    if (g >= C.n * C.mb) return;
    const int I = g % C.n, J = g / C.n;
    const bool on = k < C.l;
    const int64_t fs = F.cstr, cs = C.cstr;
    const int64_t t = on ? mg_cell(C, I, J, k) : 0;
    double bt = 0.0, bs = 0.0;
    if (shortcut) {
        /* the two colour-0 children (a + b + jpar even), clamped into the level and weighted
         * 0 outside it, so that all their loads issue at once; (c00 + c10) + (c01 + c11)
         * with the colour-1 terms 0 is their plain sum */
        double rr[2][2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int a = h ? 1 - F.jpar : F.jpar, b = h;
            const int i0 = 2 * I + a, j0 = 2 * J + b;
            const bool in = on && i0 < F.n && j0 < F.mb;
            const int i = min(i0, F.n - 1), jl = min(j0, F.mb - 1), kc = on ? k : 0;
            const int64_t c = mg_cell(F, i, jl, kc);
            double at = 0.0, as = 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int ii = i, jj = jl, kk = kc;
                mg_nbc(F, q, ii, jj, kk);
                const int64_t nc = mg_cell(F, ii, jj, kk);
                at += F.off[(int64_t)q * fs + c] * F.z[nc];
                as += F.off[(int64_t)(8 + q) * fs + c] * F.z[fs + nc];
            }
            rr[h][0] = in ? -at : 0.0;
            rr[h][1] = in ? -as : 0.0;
        }
        bt = rr[0][0] + rr[1][0];
        bs = rr[0][1] + rr[1][1];
    } else if (on) {
        double r[4][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
#pragma unroll
        for (int ch = 0; ch < 4; ch++) {
            const int i = 2 * I + (ch & 1), jl = 2 * J + (ch >> 1);
            if (i >= F.n || jl >= F.mb) continue;
            const int64_t c = mg_cell(F, i, jl, k);
            double at, as;
            mg_offmul(F, i, jl, k, c, at, as);
            const double zt = F.z[c], zs = F.z[fs + c];
            at += F.diag[c] * zt + F.diag[fs + c] * zs;
            as += F.diag[2 * fs + c] * zt + F.diag[3 * fs + c] * zs;
            r[ch][0] = F.b[c] - at;
            r[ch][1] = F.b[fs + c] - as;
        }
        bt = (r[0][0] + r[1][0]) + (r[2][0] + r[3][0]);
        bs = (r[0][1] + r[1][1]) + (r[2][1] + r[3][1]);
    }
    if (on) {
        C.b[t] = bt;
        C.b[cs + t] = bs;
    }
    if (!relax) return;
    if (mg_lcolour(C, I, J) == 0) {
        double xt, xs;
        line_solve<P>(C.fac + t, cs, on, k, bt, bs, xt, xs);
        if (on) {
            C.z[t] = xt;
            C.z[cs + t] = xs;
        }
    } else if (on) {
        C.z[t] = 0.0;
        C.z[cs + t] = 0.0;
    }
}
template <int P>
__global__ void __launch_bounds__(256) k_mg_rc(TsLev F, TsLev C, int shortcut, int relax)
{
    rc_one<P>(F, C, (blockIdx.x * blockDim.x + threadIdx.x) / P, threadIdx.x % P, shortcut, relax);
}

/* ---- fused coarse-level visits (two colours, no halos, one sweep): one launch per 2 x 2
 * aggregate instead of two dependent launches, each workgroup recomputing the colour-1
 * lines its aggregate's colour-0 cells border (10 line solves for 2 + 2 outputs; the
 * coarse levels are latency-bound, their arrays L2-resident).  Groups of P lanes: g < 8
 * the line of neighbour q = g & 3 of colour-0 child h = g >> 2, g = 8, 9 the aggregate's
 * own colour-1 children.  The arithmetic is that of the unfused launches, operation for
 * operation (the sums in the same order), so both give the same iterates. */
template <int P>
__device__ __forceinline__ void mg_child0(const TsLev& F, int I, int J, int h, int& i, int& jl, bool& in)
{
    const int a = h ? 1 - F.jpar : F.jpar;          /* (a + h + jpar) even: colour 0 */
    in = 2 * I + a < F.n && 2 * J + h < F.mb;
    i = min(2 * I + a, F.n - 1);
    jl = min(2 * J + h, F.mb - 1);
}

/* down leg at level F (first visit, colour 0 relaxed from zero): colour-1 lines, the
 * restriction of the residual (zero on colour 1, -H z on colour 0: k_mg_rc's shortcut) and,
 * when relax, the coarse level's colour-0 lines from zero -- k_mg_zl(colour 1) + k_mg_rc */
template <int P>
__global__ void __launch_bounds__(10 * P) k_mg_dn(TsLev F, TsLev C, int relax)
{
    __shared__ double xv[8][2][P];
    const int g = threadIdx.x / P, k = threadIdx.x % P;
    const int I = blockIdx.x % C.n, J = blockIdx.x / C.n;
    const bool on = k < F.l;
    const int64_t fs = F.cstr, cs = C.cstr;
    const int64_t t = on ? mg_cell(C, I, J, k) : 0;
    /* group 0's operands of the restriction and the coarse line, loaded before the lines */
    double po[2][8];
    LineFac cf{};
    if (g == 0) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            int i, jl;
            bool in;
            mg_child0<P>(F, I, J, h, i, jl, in);
            const int64_t c = mg_cell(F, i, jl, on ? k : 0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                po[h][q] = F.off[(int64_t)q * fs + c];
                po[h][4 + q] = F.off[(int64_t)(8 + q) * fs + c];
            }
        }
        cf = line_fac(C.fac + t, cs, on && relax && mg_lcolour(C, I, J) == 0);
    }
    if (g < 8) {
        const int h = g >> 2, q = g & 3;
        int i, jl;
        bool in;
        mg_child0<P>(F, I, J, h, i, jl, in);
        double xt = 0.0, xs = 0.0;
        if (in) {
            int ii = i, jj = jl, kk = on ? k : 0;
            mg_nbc(F, q, ii, jj, kk);
            if (ii == i && jj == jl) {                 /* clamped: the child itself, weight 0 */
                if (on) {
                    const int64_t c = mg_cell(F, i, jl, k);
                    xt = F.z[c];
                    xs = F.z[fs + c];
                }
            } else {
                zl_col<P>(F, ii, jj, k, on, 1, F, 0, xt, xs);
            }
        }
        xv[g][0][k] = xt;
        xv[g][1][k] = xs;
    } else {
        const int h = g - 8, a = h ? F.jpar : 1 - F.jpar;   /* colour 1 */
        const int i = 2 * I + a, jl = 2 * J + h;
        if (i < F.n && jl < F.mb) {
            double xt, xs;
            const int64_t c = zl_col<P>(F, i, jl, k, on, 1, F, 0, xt, xs);
            if (on) {
                F.z[c] = xt;
                F.z[fs + c] = xs;
            }
        }
    }
    __syncthreads();
    if (g != 0) return;
    double rr[2][2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        int i, jl;
        bool in;
        mg_child0<P>(F, I, J, h, i, jl, in);
        double at = 0.0, as = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            at += po[h][q] * xv[4 * h + q][0][k];
            as += po[h][4 + q] * xv[4 * h + q][1][k];
        }
        rr[h][0] = (on && in) ? -at : 0.0;
        rr[h][1] = (on && in) ? -as : 0.0;
    }
    const double bt = rr[0][0] + rr[1][0], bs = rr[0][1] + rr[1][1];
    if (on) {
        C.b[t] = bt;
        C.b[cs + t] = bs;
    }
    if (!relax) return;
    if (mg_lcolour(C, I, J) == 0) {
        double xt, xs;
        line_run<P>(cf, k, bt, bs, xt, xs);
        if (on) {
            C.z[t] = xt;
            C.z[cs + t] = xs;
        }
    } else if (on) {
        C.z[t] = 0.0;
        C.z[cs + t] = 0.0;
    }
}

/* up leg at level F (one sweep, colours 1 then 0): the colour-1 lines with the coarse
 * correction C.z added to their colour-0 neighbours, then the colour-0 lines from the new
 * colour-1 values -- k_mg_zl(1, corr) + k_mg_zl(0); the result goes to zu (not F.z, which
 * the neighbouring workgroups still read) */
template <int P>
__global__ void __launch_bounds__(10 * P) k_mg_up(TsLev F, TsLev C, double* __restrict__ zu)
{
    __shared__ double xv[8][2][P];
    const int g = threadIdx.x / P, k = threadIdx.x % P;
    const int I = blockIdx.x % C.n, J = blockIdx.x / C.n;
    const bool on = k < F.l;
    const int64_t fs = F.cstr;
    /* groups 0, 1: their colour-0 child's operands, loaded before the colour-1 lines */
    int64_t c0 = 0;
    bool in0 = false;
    double b0t = 0.0, b0s = 0.0, po[8];
    LineFac ff{};
    if (g < 2) {
        int i, jl;
        mg_child0<P>(F, I, J, g, i, jl, in0);
        if (in0 && on) {
            c0 = mg_cell(F, i, jl, k);
            b0t = F.b[c0];
            b0s = F.b[fs + c0];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                po[q] = F.off[(int64_t)q * fs + c0];
                po[4 + q] = F.off[(int64_t)(8 + q) * fs + c0];
            }
        }
        ff = line_fac(F.fac + c0, fs, in0 && on);
    }
    if (g < 8) {
        const int h = g >> 2, q = g & 3;
        int i, jl;
        bool in;
        mg_child0<P>(F, I, J, h, i, jl, in);
        double xt = 0.0, xs = 0.0;
        if (in) {
            int ii = i, jj = jl, kk = on ? k : 0;
            mg_nbc(F, q, ii, jj, kk);
            if (ii == i && jj == jl) {                 /* clamped: the child's old value, weight 0 */
                if (on) {
                    const int64_t c = mg_cell(F, i, jl, k);
                    xt = F.z[c];
                    xs = F.z[fs + c];
                }
            } else {
                zl_col<P>(F, ii, jj, k, on, 1, C, 1, xt, xs);
            }
        }
        xv[g][0][k] = xt;
        xv[g][1][k] = xs;
    } else {
        const int h = g - 8, a = h ? F.jpar : 1 - F.jpar;
        const int i = 2 * I + a, jl = 2 * J + h;
        if (i < F.n && jl < F.mb) {
            double xt, xs;
            const int64_t c = zl_col<P>(F, i, jl, k, on, 1, C, 1, xt, xs);
            if (on) {
                zu[c] = xt;
                zu[fs + c] = xs;
            }
        }
    }
    __syncthreads();
    if (g >= 2 || !in0) return;                        /* whole groups */
    /* colour-0 child h = g: its line from the four new colour-1 neighbours (k_mg_zl colour 0) */
    const int h = g;
    double rt = b0t, rs = b0s;
    if (on) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            rt -= po[q] * xv[4 * h + q][0][k];
            rs -= po[4 + q] * xv[4 * h + q][1][k];
        }
    }
    double xt, xs;
    line_run<P>(ff, k, rt, rs, xt, xs);
    if (on) {
        zu[c0] = xt;
        zu[fs + c0] = xs;
    }
}

/* Level-0 entry: the T/S right-hand side rr_TS - A_TS,D z_D of a tile of TI columns of one
 * latitude row (Jacobian slots read along i, coalesced; identity-row columns skipped by
 * the slot bitmask), transposed through LDS into the k-contiguous level layout, then the
 * tile's colour-0 lines relaxed from the zero iterate and the other columns' iterate set
 * to 0 (one launch instead of rhs + first colour). */
constexpr int MG_TI = 16;
template <int P>
__global__ void __launch_bounds__(256) k_mg_entry(const double* __restrict__ val, const uint8_t* __restrict__ knP,
                                                 const uint64_t* __restrict__ kmask,
                                                 const double* __restrict__ rr, const double* __restrict__ z,
                                                 Lay L, TsLev V)
{
    LAY_ALIASES;
    __shared__ double sb[2][64][MG_TI + 1];
    const int nx = L.nx;
    const int tiles = (nx + MG_TI - 1) / MG_TI;
    const int jl = blockIdx.x / tiles, i0 = (blockIdx.x % tiles) * MG_TI;
    const int j = L.jb0 + jl;
    const SubLay X = sub_of(L);
    for (int e = threadIdx.x; e < 2 * l * MG_TI; e += blockDim.x) {
        const int R = TT + e / (l * MG_TI);
        const int k = (e / MG_TI) % l, ii = e % MG_TI, i = i0 + ii;
        double acc = 0.0;
        if (i < nx) {
            const int64_t lc = ((int64_t)jl * l + k) * nx + i;
            const int64_t cell = L.own0 + lc;
            const int64_t row = PL(cell, R);
            if (!knP[row]) {
                int nc[3][9];
                nb_cells(X, i, j, k, nc);
                const uint64_t kb = kmask[2 * cell + 1];
                acc = R == TT ? bts_row<TT>(val, z, lc, L.nloc, nc, kb, rr[row], 1, L.ps)
                              : bts_row<SS>(val, z, lc, L.nloc, nc, kb, rr[row], 1, L.ps);
            }
        }
        sb[R - TT][k][ii] = acc;
    }
    __syncthreads();
    const int grp = threadIdx.x / P, k = threadIdx.x % P, ng = blockDim.x / P;
    const bool on = k < l;
    for (int ii = grp; ii < MG_TI; ii += ng) {
        const int i = i0 + ii;
        if (i >= nx) break;
        const int64_t c = on ? mg_cell(V, i, jl, k) : 0;
        const double bt = on ? sb[0][k][ii] : 0.0, bs = on ? sb[1][k][ii] : 0.0;
        if (on) {
            V.b[c] = bt;
            V.b[V.cstr + c] = bs;
        }
        if (mg_lcolour(V, i, jl) == 0) {
            double xt, xs;
            line_solve<P>(V.fac + c, V.cstr, on, k, bt, bs, xt, xs);
            if (on) {
                V.z[c] = xt;
                V.z[V.cstr + c] = xs;
            }
        } else if (on) {
            V.z[c] = 0.0;
            V.z[V.cstr + c] = 0.0;
        }
    }
}

/* fine iterate += coarse correction of its aggregate (active unknowns; level 0 of a band
 * group only, where the first post-smoothing colour reads neighbours across the band edge) */
__global__ void k_mg_prolong(TsLev F, TsLev C)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)F.n * F.mb * F.l) return;
    const int k = (int)(t % F.l), i = (int)((t / F.l) % F.n), jl = (int)(t / ((int64_t)F.l * F.n));
    const int64_t c = mg_cell(F, i, jl, k), p = mg_cell(C, i >> 1, jl >> 1, k);
    if (F.diag[c] != 0.0) F.z[c] += C.z[p];
    if (F.diag[3 * F.cstr + c] != 0.0) F.z[F.cstr + c] += C.z[C.cstr + p];
}

/* level-0 iterate -> z(T, S) of the preconditioner output on the active rows (when the
 * T/S block was solved before the last dynamics pass, whose defects see z(T, S) = 0) */
__global__ void k_mg_out(TsLev V, double* __restrict__ zout)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)V.n * V.mb * V.l) return;
    const int k = (int)(t % V.l), i = (int)((t / V.l) % V.n), jl = (int)(t / ((int64_t)V.l * V.n));
    const int64_t c = mg_cell(V, i, jl, k);
    const int64_t e = NUN * ((((int64_t)jl + HALO) * V.l + k) * V.n + i);
    if (V.diag[c] != 0.0) zout[e + TT] = V.z[c];
    if (V.diag[3 * V.cstr + c] != 0.0) zout[e + SS] = V.z[V.cstr + c];
}

/* level 0: the compact T/S couplings and 2x2 blocks (ext layout) into the level layout */
__global__ void k_mg_pack0(const double* __restrict__ tsoff, const double* __restrict__ tsdiag, Lay L,
                           int64_t next, TsLev V, double* __restrict__ off, double* __restrict__ diag)
{
    OWNED_CELL;
    const int64_t c = mg_cell(V, i - L.ib0, j - L.jb0, k);
#pragma unroll
    for (int e = 0; e < 16; e++) off[(int64_t)e * V.cstr + c] = tsoff[(int64_t)e * next + cell];
#pragma unroll
    for (int e = 0; e < 4; e++) diag[(int64_t)e * V.cstr + c] = tsdiag[(int64_t)e * next + cell];
}

/* Galerkin coarse operator: sum of the children's blocks and couplings; couplings inside
 * the aggregate go to the coarse 2x2 block */
__global__ void k_mg_galerkin(TsLev F, TsLev C, double* __restrict__ off, double* __restrict__ diag)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)C.n * C.mb * C.l) return;
    const int k = (int)(t % C.l), I = (int)((t / C.l) % C.n), J = (int)(t / ((int64_t)C.l * C.n));
    const int64_t fs = F.cstr;
    double o[16], d[4] = {0.0, 0.0, 0.0, 0.0};
    for (int e = 0; e < 16; e++) o[e] = 0.0;
    for (int b = 0; b < 2; b++)
        for (int a = 0; a < 2; a++) {
            const int i = 2 * I + a, jl = 2 * J + b;
            if (i >= F.n || jl >= F.mb) continue;
            const int64_t c = mg_cell(F, i, jl, k);
            for (int e = 0; e < 4; e++) d[e] += F.diag[(int64_t)e * fs + c];
            for (int R = 0; R < 2; R++)
                for (int q = 0; q < 8; q++) {
                    const double v = F.off[(int64_t)(8 * R + q) * fs + c];
                    if (v == 0.0) continue;
                    int ii = i, jj = jl, kk = k;
                    if (!mg_nb(F, q < 6 ? q : q - 2, ii, jj, kk)) continue;
                    if (q < 6 && ii >= 0 && ii < F.n && jj >= 0 && jj < F.mb && (ii >> 1) == I && (jj >> 1) == J &&
                        kk == k)
                        d[3 * R] += v;                    /* same variable, same aggregate */
                    else
                        o[8 * R + q] += v;
                }
        }
    const bool at = d[0] != 0.0, as = d[3] != 0.0;
    if (!at) { d[1] = d[2] = 0.0; for (int q = 0; q < 8; q++) o[q] = 0.0; }
    if (!as) { d[1] = d[2] = 0.0; for (int q = 8; q < 16; q++) o[q] = 0.0; }
    /* the level's layout (a level with an x halo pads its rows) */
    const int64_t cs = C.cstr, cc = mg_cell(C, I, J, k);
    for (int e = 0; e < 16; e++) off[(int64_t)e * cs + cc] = o[e];
    for (int e = 0; e < 4; e++) diag[(int64_t)e * cs + cc] = d[e];
}

/* z-line factors of every owned column (one thread each, serial block Thomas along k, the
 * CPU twin's mg_zline arithmetic): A'_k = A_k - B_k Cp_{k-1}, F_k = -A'_k^-1 B_k, Cp_k =
 * A'_k^-1 C_k; inactive unknowns (zero diagonal) are identity rows whose A'^-1 and F rows
 * are zeroed, so their line values come out 0 whatever the right-hand side */
__global__ void k_mg_fac(TsLev V, double* __restrict__ fac)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= V.n * V.mb) return;
    const int i = t % V.n, jl = t / V.n;
    const int64_t cs = V.cstr;
    double P0 = 0.0, P1 = 0.0, P2 = 0.0, P3 = 0.0;
    for (int k = 0; k < V.l; k++) {
        const int64_t c = mg_cell(V, i, jl, k);
        double Am[4] = {V.diag[c], V.diag[cs + c], V.diag[2 * cs + c], V.diag[3 * cs + c]};
        double Bm[4] = {V.off[4 * cs + c], V.off[6 * cs + c], V.off[14 * cs + c], V.off[12 * cs + c]};
        double Cm[4] = {V.off[5 * cs + c], V.off[7 * cs + c], V.off[15 * cs + c], V.off[13 * cs + c]};
        const bool at = Am[0] != 0.0, as = Am[3] != 0.0;
        if (!at) { Am[0] = 1.0; Am[1] = Am[2] = 0.0; Bm[0] = Bm[1] = 0.0; Cm[0] = Cm[1] = 0.0; }
        if (!as) { Am[3] = 1.0; Am[1] = Am[2] = 0.0; Bm[2] = Bm[3] = 0.0; Cm[2] = Cm[3] = 0.0; }
        if (k == 0) Bm[0] = Bm[1] = Bm[2] = Bm[3] = 0.0;
        else {
            const double a0 = Am[0] - (Bm[0] * P0 + Bm[1] * P2), a1 = Am[1] - (Bm[0] * P1 + Bm[1] * P3);
            const double a2 = Am[2] - (Bm[2] * P0 + Bm[3] * P2), a3 = Am[3] - (Bm[2] * P1 + Bm[3] * P3);
            Am[0] = a0; Am[1] = a1; Am[2] = a2; Am[3] = a3;
        }
        const double det = Am[0] * Am[3] - Am[1] * Am[2];
        const double qd = det != 0.0 ? 1.0 / det : 0.0;
        double I0 = Am[3] * qd, I1 = -Am[1] * qd, I2 = -Am[2] * qd, I3 = Am[0] * qd;
        P0 = I0 * Cm[0] + I1 * Cm[2]; P1 = I0 * Cm[1] + I1 * Cm[3];
        P2 = I2 * Cm[0] + I3 * Cm[2]; P3 = I2 * Cm[1] + I3 * Cm[3];
        double F0 = -(I0 * Bm[0] + I1 * Bm[2]), F1 = -(I0 * Bm[1] + I1 * Bm[3]);
        double F2 = -(I2 * Bm[0] + I3 * Bm[2]), F3 = -(I2 * Bm[1] + I3 * Bm[3]);
        if (!at) { I0 = I1 = F0 = F1 = 0.0; }
        if (!as) { I2 = I3 = F2 = F3 = 0.0; }
        const double v[12] = {F0, F1, F2, F3, I0, I1, I2, I3, P0, P1, P2, P3};
#pragma unroll
        for (int e = 0; e < 12; e++) fac[(int64_t)e * cs + c] = v[e];
    }
}
/* ---- host: structure from the identity-row pattern ------------------------------ */

/* flags[j*n+i] = 1 for an active water column (any active P), flags[n*m + j*n+i] = 1
 * for an active U/V point, over the band's latitude rows */
/* Schur structure of the whole grid from the global flags (identical on every rank) */
int build_structure(iemic_ctx* c, const std::vector<double>& flags)
{
    BlockGS& gs = c->gs;
    const int n = c->n, m = c->m;
    const int periodic = c->cfg.periodic;
    std::vector<int> colid((size_t)n * m, -1);
    std::vector<uint8_t> act((size_t)n * m, 0), uva((size_t)n * m, 0);
    for (size_t q = 0; q < (size_t)n * m; q++) {
        act[q] = flags[q] != 0.0;
        uva[q] = flags[(size_t)n * m + q] != 0.0;
    }
    auto wrap = [&](int& i, int& j) {
        if (j < 0 || j >= m) return false;
        if (i < 0 || i >= n) {
            if (!periodic) return false;
            i = (i + n) % n;
        }
        return true;
    };
    /* band ordering: i folded (periodic: 0, n-1, 1, n-2, ...), j fastest */
    std::vector<int> ipos(n);
    if (periodic) {
        int a = 0, b = n - 1, q = 0;
        while (a <= b) {
            ipos[a] = q++;
            if (a != b) ipos[b] = q++;
            a++; b--;
        }
    } else {
        for (int i = 0; i < n; i++) ipos[i] = i;
    }
    std::vector<std::pair<int64_t, int>> ord;
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++)
            if (act[(size_t)j * n + i]) ord.push_back({(int64_t)ipos[i] * m + j, j * n + i});
    std::sort(ord.begin(), ord.end());
    const int ncol = (int)ord.size();
    /* Schur index of column (i, j): c = i*m + j (the cyclic reduction's block order); the
     * band order above only fixes which column of a null-space set is pinned (its first),
     * the same choice as the CPU twin */
    const int NC = n * m;
    std::vector<int> ij_of_col(NC);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) ij_of_col[(size_t)i * m + j] = j * n + i;
    for (int q = 0; q < ncol; q++) {
        const int ij = ord[q].second;
        colid[ij] = (ij % n) * m + ij / n;
    }
    /* couplings: columns sharing an active U/V corner */
    std::vector<std::vector<int>> adj(NC);
    for (int q = 0; q < ncol; q++) {
        const int ij0 = ord[q].second;
        const int i = ij0 % n, j = ij0 / n, cq = colid[ij0];
        for (int dj = -1; dj <= 1; dj++)
            for (int di = -1; di <= 1; di++) {
                int ti = i + di, tj = j + dj;
                if (!wrap(ti, tj)) continue;
                const int q2 = colid[(size_t)tj * n + ti];
                if (q2 < 0 || q2 == cq) continue;
                bool shared = false;
                for (int a = -1; a <= 0 && !shared; a++)
                    for (int b = -1; b <= 0 && !shared; b++) {
                        /* corner (i+a, j+b) must also be a corner of (ti,tj): e = di-a in {0,1} */
                        const int e = di - a, f = dj - b;
                        if (e < 0 || e > 1 || f < 0 || f > 1) continue;
                        int qi = i + a, qj = j + b;
                        if (!wrap(qi, qj)) continue;
                        if (uva[(size_t)qj * n + qi]) shared = true;
                    }
                if (shared) adj[cq].push_back(q2);
            }
    }
    /* null space of the B-grid pressure Schur: constant on each connected set of
     * same-colour columns linked diagonally through an active U/V corner (checkerboard
     * modes, local ones around islands and straits included) -> one pin per set */
    std::vector<uint8_t> pin(NC, 0);
    std::vector<int> comp(NC, -1);
    for (int q = 0; q < ncol; q++) {
        const int s0 = colid[ord[q].second];       /* band order: first column of its set */
        if (comp[s0] >= 0) continue;
        std::vector<int> stack{s0};
        comp[s0] = s0;
        pin[s0] = 1;
        while (!stack.empty()) {
            const int cq = stack.back();
            stack.pop_back();
            for (int q2 : adj[cq]) {
                int di = q2 / m - cq / m;
                const int dj = q2 % m - cq % m;
                if (di > 1) di -= n;
                if (di < -1) di += n;
                if (di == 0 || dj == 0) continue; /* other colour */
                if (comp[q2] < 0) { comp[q2] = s0; stack.push_back(q2); }
            }
        }
    }
    std::vector<int> own(NC, -1), ocol((size_t)n * m, -1);
    for (int q = 0; q < ncol; q++) {
        const int ij = ord[q].second;
        if (c->su.owns(ij % n, ij / n)) {
            own[colid[ij]] = colid[ij];
            ocol[ij] = pin[colid[ij]] ? -2 - colid[ij] : colid[ij];
        }
    }
    gs.ncol = ncol;
    int rc = 0;
    rc |= gs.col_of_ij.alloc((size_t)n * m);
    rc |= gs.ij_of_col.alloc(NC);
    rc |= gs.pinned.alloc(NC);
    rc |= gs.S9.alloc((size_t)9 * NC);
    rc |= gs.colv2.alloc(NC);
    rc |= gs.colvT.alloc(NC);
    rc |= gs.colvZ.alloc(NC);
    rc |= gs.colv_own.alloc(NC);
    rc |= gs.colv.alloc(NC);
    rc |= gs.own_pos.alloc(NC);
    rc |= gs.ocol.alloc((size_t)n * m);
    if (rc) {
        set_error("block GS: out of device memory");
        return IEMIC_ENOMEM;
    }
    if ((rc = h2d(c, gs.col_of_ij.p, colid.data(), sizeof(int) * colid.size()))) return rc;
    if ((rc = h2d(c, gs.ij_of_col.p, ij_of_col.data(), sizeof(int) * NC))) return rc;
    HIP_OK(hipMemsetAsync(gs.colvZ.p, 0, sizeof(double) * NC, c->stream));
    if ((rc = h2d(c, gs.pinned.p, pin.data(), NC))) return rc;
    if ((rc = h2d(c, gs.own_pos.p, own.data(), sizeof(int) * NC))) return rc;
    if ((rc = h2d(c, gs.ocol.p, ocol.data(), sizeof(int) * ocol.size()))) return rc;
    /* entries of inactive and foreign columns stay 0 (the rhs of the reduced solve) */
    HIP_OK(hipMemsetAsync(gs.colv_own.p, 0, sizeof(double) * NC, c->stream));
    HIP_OK(hipMemsetAsync(gs.colv2.p, 0, sizeof(double) * NC, c->stream));
    if ((rc = cr_init(c, gs.cr, n, m, periodic))) return rc;
    gs.flags_h = flags;
    return 0;
}

}  // namespace

static Lay lay_of(const iemic_ctx* c)
{
    Lay L;
    L.n = c->n; L.m = c->m; L.l = c->l; L.periodic = c->cfg.periodic; L.jb0 = c->jb0;
    L.ib0 = c->ib0; L.nx = c->nx; L.hx = c->hx; L.xb = c->xb;
    L.nloc = c->nloc; L.own0 = c->own0; L.ps = c->next;
    return L;
}
/* colour-compacted T/S sweeps: the owned cells of one colour are every other cell of a
 * row (even n, nx and ib0) */
static bool ts_compact(const iemic_ctx* c) { return (c->n & 1) == 0 && (c->nx & 1) == 0 && (c->ib0 & 1) == 0; }


/* ---- T/S multigrid: host side ------------------------------------------------------ */
/* intermediate levels (1 ..) that carry the x halo under x splits */
constexpr int MG_XHALO_LEVELS = 99;
static TsLev mg_view(iemic_ctx* c, int q)
{
    BlockGS& gs = c->gs;
    TsLev V{};
    V.l = c->l;
    V.n = gs.mg_n[q];
    V.mb = gs.mg_m[q];
    /* subdomains: the level-0 smoother and residual see the neighbours' edge rows and
     * columns (halo rows / columns in the layout, exchanged before every relaxation); with
     * an x split the intermediate levels see the neighbours' edge columns too (a cut across
     * the zonal flow would otherwise make them block Jacobi), the coarsest is
     * the global problem; colours by the global i + j parity of the level's aggregates, so
     * that all subdomains relax the same colour in the same launch and a cell's neighbours
     * across a cut have the other colour; the x wrap only with one x part */
    const int qc = gs.mg_nlev - 1;
    V.periodic = c->cfg.periodic && c->npx == 1;
    V.hj = (q == 0 && c->npy > 1) ? (gs.mg_hr ? 2 : 1) : 0;
    V.hi = (q < qc && q <= MG_XHALO_LEVELS && c->npx > 1) ? 1 : 0;
    V.vis = V.hj;
    V.visi = V.hi;
    V.jpar = gs.mg_par[q];
    V.cstr = (int64_t)(V.mb + 2 * V.hj) * (V.n + 2 * V.hi) * V.l;
    V.off = gs.mg_off[q].p;
    V.diag = gs.mg_diag[q].p;
    V.fac = gs.mg_fac[q].p;
    V.b = gs.mg_b[q].p;
    V.z = gs.mg_z[q].p;
    return V;
}

static unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

/* lanes per z-line (one per level, a power of two >= l; the smoother needs l <= 64) */
static int mg_lanes(int l) { return l <= 16 ? 16 : (l <= 32 ? 32 : 64); }

/* the z-line and restriction launches in 64-thread workgroups (64 / P columns each): a
 * coarse level's few columns spread over 4x the CUs of 256-thread groups (the T/S solve
 * 112 -> 103 us per apply, scripts/ab/mg_wg64.sh) */
#define MG_LAUNCH_P64(P, KERNEL, GRID, ...)                                                \
    do {                                                                                   \
        if ((P) == 16) hipLaunchKernelGGL(KERNEL<16>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \
        else if ((P) == 32) hipLaunchKernelGGL(KERNEL<32>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \
        else hipLaunchKernelGGL(KERNEL<64>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__);     \
    } while (0)
#define MG_LAUNCH_P(P, KERNEL, GRID, ...)                                                  \
    do {                                                                                   \
        if ((P) == 16) hipLaunchKernelGGL(KERNEL<16>, dim3(GRID), dim3(256), 0, s, __VA_ARGS__); \
        else if ((P) == 32) hipLaunchKernelGGL(KERNEL<32>, dim3(GRID), dim3(256), 0, s, __VA_ARGS__); \
        else hipLaunchKernelGGL(KERNEL<64>, dim3(GRID), dim3(256), 0, s, __VA_ARGS__);     \
    } while (0)

/* Gauss-Jordan inverse with partial pivoting (host, large coarsest levels); unknowns
 * without any coupling (inactive) get an identity row */
static void dense_inverse(std::vector<double>& A, int N, std::vector<double>& X)
{
    X.assign((size_t)N * N, 0.0);
    for (int i = 0; i < N; i++) {
        X[(size_t)i * N + i] = 1.0;
        bool any = false;
        for (int j = 0; j < N; j++) any |= A[(size_t)i * N + j] != 0.0;
        if (!any) A[(size_t)i * N + i] = 1.0;
    }
    for (int k = 0; k < N; k++) {
        int p = k;
        for (int i = k + 1; i < N; i++)
            if (std::fabs(A[(size_t)i * N + k]) > std::fabs(A[(size_t)p * N + k])) p = i;
        if (p != k)
            for (int j = 0; j < N; j++) {
                std::swap(A[(size_t)p * N + j], A[(size_t)k * N + j]);
                std::swap(X[(size_t)p * N + j], X[(size_t)k * N + j]);
            }
        const double d = A[(size_t)k * N + k];
        const double q = d != 0.0 ? 1.0 / d : 0.0;
        for (int j = 0; j < N; j++) {
            A[(size_t)k * N + j] *= q;
            X[(size_t)k * N + j] *= q;
        }
        for (int i = 0; i < N; i++) {
            if (i == k) continue;
            const double f = A[(size_t)i * N + k];
            if (f == 0.0) continue;
            for (int j = 0; j < N; j++) {
                A[(size_t)i * N + j] -= f * A[(size_t)k * N + j];
                X[(size_t)i * N + j] -= f * X[(size_t)k * N + j];
            }
        }
    }
}

/* decode of a coarse-level cell index t = (jl n + i) l + k */
static inline void mg_decode(int64_t t, int n, int l, int& i, int& jl, int& k)
{
    k = (int)(t % l);
    i = (int)((t / l) % n);
    jl = (int)(t / ((int64_t)l * n));
}

/* Subdomains: the coarsest T/S level as one global problem.  The ranks' coarsest grids
 * tile a GX x GY coarse grid (rank (px, py) at column offset ioff[px], row offset joff[py]);
 * unknown (J, I, k, var) is 2((J GX + I) l + k) + var, a band matrix of half-width
 * 2 l GX + 1 (+ the periodic wrap inside a row).  Every rank writes its own rows -- its
 * local coarsest operator plus the couplings of its edge aggregates to the neighbours'
 * edge aggregates, taken from the level-0 couplings across the subdomain edges (the
 * Galerkin sum of piecewise-constant aggregates) -- the rows are summed over the ranks,
 * and every rank factorises (k_band_lu) and inverts (k_band_inv_pan) the whole matrix. */
static int mg_global_setup(iemic_ctx* c, const std::vector<double>& off, const std::vector<double>& dg)
{
    BlockGS& gs = c->gs;
    gs.mg_glob = 0;
    if (c->nranks <= 1 || c->l > 64) return 0;
    const int P = c->nranks, l = c->l, qc = gs.mg_nlev - 1;
    const int nc = gs.mg_n[qc], cm = gs.mg_m[qc], mb = c->jb1 - c->jb0;
    const int64_t ncl = (int64_t)nc * cm * l;
    int rc;
    /* coarsest columns / rows of every rank: offsets of its rank column / row */
    std::vector<double> dims(2 * P, 0.0);
    dims[2 * c->rank] = nc;
    dims[2 * c->rank + 1] = cm;
    {
        DevBuf<double> rb;
        if (rb.alloc(2 * P)) return IEMIC_ENOMEM;
        if ((rc = h2d(c, rb.p, dims.data(), sizeof(double) * 2 * P))) return rc;
        if ((rc = allreduce_sum(c, rb.p, 2 * P))) return rc;
        if ((rc = d2h(c, dims.data(), rb.p, sizeof(double) * 2 * P))) return rc;
    }
    std::vector<int> ioff(c->npx + 1, 0), joff(c->npy + 1, 0);
    for (int px = 0; px < c->npx; px++) ioff[px + 1] = ioff[px] + (int)dims[2 * px];
    for (int py = 0; py < c->npy; py++) joff[py + 1] = joff[py] + (int)dims[2 * (py * c->npx) + 1];
    const int GX = ioff[c->npx], GY = joff[c->npy];
    const int I0 = ioff[c->px], J0 = joff[c->py];
    const int NG = 2 * GX * GY * l;
    const int bl = 2 * l * GX + 1, bu = bl, W = 2 * bl + bu + 1;
    {
        /* LDS of the band kernels (same rules as the Schur band) */
        const size_t lb = sizeof(double) * ((size_t)(NBP + bl) * (NBP + 1) + (size_t)NBP * (bl + bu));
        const size_t li = sizeof(double) * (size_t)(std::max(bl + NBP + 1, bl + bu + 1) + 2 * NBP) * 16;
        if (lb > 150 * 1024 || li > 150 * 1024 || (int64_t)NG * W > INT32_MAX) return 0;   /* stay local */
    }
    const bool wrap = c->cfg.periodic != 0;
    auto gidx = [&](int J, int I, int k, int var) { return 2 * ((J * GX + I) * l + k) + var; };
    auto gwrap = [&](int I) { return I < 0 ? I + GX : (I >= GX ? I - GX : I); };
    std::vector<double> H((size_t)NG * W, 0.0);
    auto add = [&](int row, int col, double v) {
        const int d = col - row;
        if (d < -bl || d > bu) return false;
        H[(size_t)row * W + (d + bl)] += v;
        return true;
    };
    bool ok = true;
    const bool lwrap = wrap && c->npx == 1;           /* the local level wraps in x */
    for (int64_t t = 0; t < ncl; t++) {
        int i, jl, k;
        mg_decode(t, nc, l, i, jl, k);
        for (int R = 0; R < 2; R++) {
            const int row = gidx(J0 + jl, I0 + i, k, R);
            ok &= add(row, gidx(J0 + jl, I0 + i, k, R), dg[(3 * R) * ncl + t]);
            ok &= add(row, gidx(J0 + jl, I0 + i, k, 1 - R), dg[(1 + R) * ncl + t]);
            for (int qq = 0; qq < 8; qq++) {
                const double v = off[(8 * R + qq) * ncl + t];
                if (v == 0.0) continue;
                int ii = i, jj = jl, kk = k;
                switch (qq < 6 ? qq : qq - 2) {
                case 0: ii--; break;
                case 1: ii++; break;
                case 2: jj--; break;
                case 3: jj++; break;
                case 4: kk--; break;
                default: kk++; break;
                }
                if (jj < 0 || jj >= cm || kk < 0 || kk >= l) continue;
                if (ii < 0 || ii >= nc) {
                    if (!lwrap) continue;
                    ii = (ii + nc) % nc;
                }
                ok &= add(row, gidx(J0 + jj, I0 + ii, kk, qq < 6 ? R : 1 - R), v);
            }
        }
    }
    /* cross-subdomain couplings: level-0 T/S couplings of the first / last latitude row (-j /
     * +j) and the first / last column (-i / +i), summed into the edge aggregates */
    {
        const int64_t nx = c->nx, slab = (int64_t)l * nx;
        std::vector<double> e((size_t)slab * mb);
        for (int dir = 0; dir < 4; dir++) {
            if (c->nb[dir] < 0) continue;
            const int q = dir == 0 ? 0 : dir == 1 ? 1 : dir == 2 ? 2 : 3;   /* -i, +i, -j, +j */
            for (int R = 0; R < 2; R++) {
                /* the owned rows of coupling q of row R (ext layout: one slab) */
                const double* src = gs.tsoff.p + (int64_t)(R * 8 + q) * c->next + c->own0;
                if ((rc = d2h(c, e.data(), src, sizeof(double) * e.size()))) return rc;
                for (int jl = 0; jl < mb; jl++)
                    for (int k = 0; k < l; k++)
                        for (int il = 0; il < nx; il++) {
                            const bool edge = dir == 0 ? il == 0 : dir == 1 ? il == nx - 1 : dir == 2 ? jl == 0 : jl == mb - 1;
                            if (!edge) continue;
                            const double v = e[((int64_t)jl * l + k) * nx + il];
                            if (v == 0.0) continue;
                            const int Is = I0 + (il >> qc), Js = J0 + (jl >> qc);
                            const int Id = dir == 0 ? gwrap(I0 - 1) : dir == 1 ? gwrap(ioff[c->px + 1]) : Is;
                            const int Jd = dir == 2 ? J0 - 1 : dir == 3 ? joff[c->py + 1] : Js;
                            ok &= add(gidx(Js, Is, k, R), gidx(Jd, Id, k, R), v);
                        }
            }
        }
    }
    if (!ok) return 0;                        /* outside the assumed band: stay local */
    /* own rows without entries (inactive unknowns) become identity rows */
    for (int jl = 0; jl < cm; jl++)
        for (int i = 0; i < nc; i++)
            for (int k = 0; k < l; k++)
                for (int R = 0; R < 2; R++) {
                    const int row = gidx(J0 + jl, I0 + i, k, R);
                    bool any = false;
                    for (int d = 0; d < W; d++) any |= H[(size_t)row * W + d] != 0.0;
                    if (!any) H[(size_t)row * W + bl] = 1.0;
                }
    const size_t npan = (size_t)(NG + NBP - 1) / NBP;
    if (gs.mg_gband.n < (size_t)NG * W) {
        if (gs.mg_gband.alloc((size_t)NG * W) || gs.mg_gX.alloc((size_t)NG * NG) ||
            gs.mg_gvec.alloc(NG) || gs.mg_gtmp.alloc(NG) || gs.mg_gpiv.alloc(NG) ||
            gs.mg_ginfo.alloc(1) || gs.mg_gcols.alloc(NG) ||
            gs.mg_glpan.alloc(npan * (NBP + bl) * NBP))
            return IEMIC_ENOMEM;
        std::vector<int> cols(NG);
        for (int q = 0; q < NG; q++) cols[q] = q;
        if ((rc = h2d(c, gs.mg_gcols.p, cols.data(), sizeof(int) * NG))) return rc;
    }
    if ((rc = h2d(c, gs.mg_gband.p, H.data(), sizeof(double) * H.size()))) return rc;
    if ((rc = allreduce_sum(c, gs.mg_gband.p, (int)((size_t)NG * W)))) return rc;
    {
        const size_t lb = sizeof(double) * ((size_t)(NBP + bl) * (NBP + 1) + (size_t)2 * NBP * (bl + bu));
        const int stage_o = lb <= 150 * 1024 ? 1 : 0;
        const size_t lbu = stage_o ? lb : lb - sizeof(double) * (size_t)NBP * (bl + bu);
        HIP_OK(hipFuncSetAttribute((const void*)k_band_lu, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lbu));
        hipLaunchKernelGGL(k_band_lu, dim3(1), dim3(1024), lbu, c->stream, gs.mg_gband.p, NG, bl, bu,
                           gs.mg_gpiv.p, gs.mg_ginfo.p, gs.mg_glpan.p, stage_o);
        int info = 0;
        HIP_OK(hipGetLastError());
        if ((rc = d2h(c, &info, gs.mg_ginfo.p, sizeof(int)))) return rc;
        if (info != 0) return 0;              /* singular global coarse problem: local */
        const int ring = std::max(bl + NBP + 1, bl + bu + 1);
        const size_t li = (size_t)(ring + 2 * NBP) * 16 * sizeof(double);
        HIP_OK(hipFuncSetAttribute((const void*)k_band_inv_pan<16, false>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)li));
        hipLaunchKernelGGL((k_band_inv_pan<16, false>), dim3((unsigned)((NG + 15) / 16)), dim3(256), li,
                           c->stream, gs.mg_gband.p, gs.mg_glpan.p, gs.mg_gpiv.p, NG, bl, bu,
                           gs.mg_gcols.p, NG, gs.mg_gX.p);
        HIP_OK(hipGetLastError());
    }
    gs.mg_gN = NG;
    gs.mg_gGX = GX;
    gs.mg_gI0 = I0;
    gs.mg_gJ0 = J0;
    gs.mg_glob = 1;
    return 0;
}

/* global index of local coarsest cell t (rank offsets I0, J0 in the GX-wide coarse grid) */
__device__ __forceinline__ int64_t mg_gq(int64_t t, int nc, int l, int GX, int I0, int J0)
{
    const int k = (int)(t % l), i = (int)((t / l) % nc), jl = (int)(t / ((int64_t)l * nc));
    return 2 * ((((int64_t)J0 + jl) * GX + I0 + i) * l + k);
}
/* local coarsest rhs (T block, S block) -> its entries of the global vector */
__global__ void k_mg_gput(const double* __restrict__ b, int64_t ncl, int nc, int l, int GX, int I0, int J0,
                          double* __restrict__ g)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncl) return;
    const int64_t q = mg_gq(t, nc, l, GX, I0, J0);
    g[q] = b[t];
    g[q + 1] = b[ncl + t];
}
/* own rows of the global solution -> local (T block, S block) */
__global__ void k_mg_gget(const double* __restrict__ y, int64_t ncl, int nc, int l, int GX, int I0, int J0,
                          double* __restrict__ z)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncl) return;
    const int64_t q = mg_gq(t, nc, l, GX, I0, J0);
    z[t] = y[q];
    z[ncl + t] = y[q + 1];
}

/* the coarsest level's dense operator, row-major A[row * N + col] (one thread per row; the
 * same entries as the host assembly below), inactive rows -> identity rows */
__global__ void k_mg_coarse_dense(const double* __restrict__ off, const double* __restrict__ dg, int64_t ncl,
                                  int cn, int cm, int l, int periodic, double* __restrict__ A)
{
    const int64_t rowq = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rowq >= 2 * ncl) return;
    const int R = (int)(rowq / ncl);
    const int64_t t = rowq % ncl;
    const int64_t N = 2 * ncl;
    double* Ar = A + rowq * N;
    const int k = (int)(t % l), i = (int)((t / l) % cn), jl = (int)(t / ((int64_t)l * cn));
    Ar[R * ncl + t] += dg[(3 * R) * ncl + t];
    Ar[(1 - R) * ncl + t] += dg[(1 + R) * ncl + t];
    for (int qq = 0; qq < 8; qq++) {
        const double v = off[(8 * R + qq) * ncl + t];
        if (v == 0.0) continue;
        int ii = i, jj = jl, kk = k;
        const int dir = qq < 6 ? qq : qq - 2;
        switch (dir) {
        case 0: ii--; break;
        case 1: ii++; break;
        case 2: jj--; break;
        case 3: jj++; break;
        case 4: kk--; break;
        default: kk++; break;
        }
        if (jj < 0 || jj >= cm || kk < 0 || kk >= l) continue;
        if (ii < 0 || ii >= cn) {
            if (!periodic) continue;
            ii = (ii + cn) % cn;
        }
        const int64_t nb = ((int64_t)jj * cn + ii) * l + kk;
        const int var = qq < 6 ? R : 1 - R;
        Ar[var * ncl + nb] += v;
    }
    bool any = false;
    for (int64_t c = 0; c < N; c++) any |= Ar[c] != 0.0;
    if (!any) Ar[rowq] = 1.0;
}

/* the coarsest level's operator as cyclic-reduction blocks over longitudes (one rank, no
 * halo): block i holds the unknowns (jl l + k) 2 + var of longitude i; D_i couples them
 * within the longitude (2x2 cell block, -+j, -+k, the T/S cross couplings along k), L_i / R_i
 * to longitude i -+ 1 (wrapping when periodic).  Inactive unknowns become identity rows.
 * One thread per (cell, var) row: no write races. */
__global__ void k_mg_cr_expand(TsLev V, int mc, int periodic, double* __restrict__ D, double* __restrict__ Lb,
                               double* __restrict__ Rb)
{
    const int64_t ncl = (int64_t)V.n * V.mb * V.l;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 2 * ncl) return;
    const int R = (int)(q / ncl);
    const int64_t t = q % ncl;
    const int k = (int)(t % V.l), i = (int)((t / V.l) % V.n), jl = (int)(t / ((int64_t)V.l * V.n));
    const int64_t cs = V.cstr, c = mg_cell(V, i, jl, k);
    const size_t mm = (size_t)mc * mc;
    auto idx = [&](int j2, int k2, int var) { return (j2 * V.l + k2) * 2 + var; };
    const int r = idx(jl, k, R);
    double* Di = D + (size_t)i * mm;
    if (V.diag[(int64_t)(3 * R) * cs + c] == 0.0) {
        Di[r + (size_t)r * mc] = 1.0;
        return;
    }
    Di[r + (size_t)r * mc] += V.diag[(int64_t)(3 * R) * cs + c];
    Di[r + (size_t)idx(jl, k, 1 - R) * mc] += V.diag[(int64_t)(1 + R) * cs + c];
    for (int qq = 0; qq < 8; qq++) {
        const double v = V.off[(int64_t)(8 * R + qq) * cs + c];
        if (v == 0.0) continue;
        const int dir = qq < 6 ? qq : qq - 2, var = qq < 6 ? R : 1 - R;
        int jj = jl, kk = k;
        double* B = Di;
        switch (dir) {
        case 0:
            if (i == 0 && !periodic) continue;
            B = Lb + (size_t)i * mm;
            break;
        case 1:
            if (i == V.n - 1 && !periodic) continue;
            B = Rb + (size_t)i * mm;
            break;
        case 2: jj--; break;
        case 3: jj++; break;
        case 4: kk--; break;
        default: kk++; break;
        }
        if (jj < 0 || jj >= V.mb || kk < 0 || kk >= V.l) continue;
        B[r + (size_t)idx(jj, kk, var) * mc] += v;
    }
}

/* the whole-problem inverse of the cyclic reduction (row-major, longitude-block order) in
 * the level's unknown order var ncl + cell, row-major -- what the coarse GEMV applies */
__global__ void k_mg_cr_perm(const double* __restrict__ T, TsLev V, int N, double* __restrict__ X)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)N * N) return;
    const int64_t ncl = N / 2;
    const int rq = (int)(e / N), cq = (int)(e % N);
    auto cr_of = [&](int u) {
        const int var = (int)(u / ncl);
        const int64_t t = u % ncl;
        const int k = (int)(t % V.l), i = (int)((t / V.l) % V.n), jl = (int)(t / ((int64_t)V.l * V.n));
        return (int64_t)i * (2 * V.mb * V.l) + (jl * V.l + k) * 2 + var;
    };
    X[e] = T[cr_of(rq) * N + cr_of(cq)];
}

/* levels, Galerkin operators, z-line factors and the coarsest inverse (once per Jacobian) */
static int mg_setup(iemic_ctx* c)
{
    BlockGS& gs = c->gs;
    const int l = c->l;
    int rc;
    if (l > 64) {                /* the z-line smoother runs one lane per level */
        gs.ts_mg = 0;
        return 0;
    }
    if (gs.mg_nlev == 0) {
        /* latitude bands, one sweep: level 0 keeps 2 halo rows (mg_vcycle) */
        gs.mg_hr = c->npy > 1 && c->npx == 1 && std::max(1, gs.mg_sweeps) == 1;
        /* coarsen 2x2 horizontally until the level has <= 128 cells (<= 256 unknowns); the
         * number of levels is that of the largest subdomain, the same on every rank, so the
         * coarsest grids of the ranks tile the global coarsest problem */
        int N = (c->n + c->npx - 1) / c->npx, M = (c->m + c->npy - 1) / c->npy, q = 0;
        int n = c->nx, m = c->jb1 - c->jb0;
        gs.mg_n[0] = n;
        gs.mg_m[0] = m;
        gs.mg_crd = 0;
        /* one rank: stop at the first level of <= MG_CR_CELLS cells that the whole-problem
         * cyclic reduction takes (blocks of one longitude, 2 m l <= 192 unknowns, >= 2
         * longitudes): an exact coarse solve, one GEMV per V-cycle instead of the last
         * levels' ~9 latency-bound launches */
        auto cr_ok = [&](int nn, int mm) {
            return c->nranks == 1 && (int64_t)nn * mm * l <= BlockGS::MG_CR_CELLS && 2 * mm * l <= 192 && nn >= 2;
        };
        while (q + 1 < BlockGS::MG_MAX && (q == 0 || (int64_t)N * M * l > 128) && (N > 1 || M > 1) &&
               !(q > 0 && cr_ok(n, m))) {
            N = (N + 1) / 2;
            M = (M + 1) / 2;
            n = (n + 1) / 2;
            m = (m + 1) / 2;
            q++;
            gs.mg_n[q] = n;
            gs.mg_m[q] = m;
        }
        if (q == 0) {
            gs.ts_mg = 0;            /* a single water column per band: plain sweeps */
            return 0;
        }
        gs.mg_crd = cr_ok(n, m) && (int64_t)n * m * l > 128 ? 1 : 0;
        if (gs.mg_crd && (rc = cr_init(c, gs.mg_cr, n, 2 * m * l, c->cfg.periodic, 2 * n * m * l))) return rc;
        if ((int64_t)n * m * l > 1024) {
            set_error("block GS: T/S multigrid coarsest level too large");
            return IEMIC_EINVAL;
        }
        gs.mg_nlev = q + 1;
        /* global offsets of this subdomain's aggregates on every level: the x parts to the
         * west / the y parts to the south, each coarsened like this one (decomp.h part_of) */
        for (int lv = 0; lv <= q; lv++) {
            auto coarse = [&](int v) {
                for (int t = 0; t < lv; t++) v = (v + 1) / 2;
                return v;
            };
            int io = 0, jo = 0, off, cnt;
            for (int px = 0; px < c->px; px++) {
                part_of(c->n, c->npx, px, off, cnt);
                io += coarse(cnt);
            }
            for (int py = 0; py < c->py; py++) {
                part_of(c->m, c->npy, py, off, cnt);
                jo += coarse(cnt);
            }
            gs.mg_par[lv] = (io + jo) & 1;
        }
        for (int lv = 0; lv <= q; lv++) {
            const size_t cs = (size_t)mg_view(c, lv).cstr;
            if (gs.mg_off[lv].alloc(16 * cs) || gs.mg_diag[lv].alloc(4 * cs) || gs.mg_fac[lv].alloc(12 * cs) ||
                gs.mg_b[lv].alloc(2 * cs) || gs.mg_z[lv].alloc(2 * cs) || gs.mg_zu[lv].alloc(2 * cs))
                return IEMIC_ENOMEM;
            for (DevBuf<double>* bptr : {&gs.mg_off[lv], &gs.mg_diag[lv], &gs.mg_fac[lv], &gs.mg_b[lv], &gs.mg_z[lv],
                                         &gs.mg_zu[lv]})
                HIP_OK(hipMemsetAsync(bptr->p, 0, sizeof(double) * bptr->n, c->stream));
        }
        const size_t NC = (size_t)2 * n * m * l;
        if (gs.mg_cinv.alloc(NC * NC)) return IEMIC_ENOMEM;
    }
    hipStream_t s = c->stream;
    {
        const TsLev V0 = mg_view(c, 0);
        hipLaunchKernelGGL(k_mg_pack0, dim3(blocks_for(c->nloc)), dim3(256), 0, s, gs.tsoff.p, gs.tsdiag.p,
                           lay_of(c), c->next, V0, gs.mg_off[0].p, gs.mg_diag[0].p);
    }
    for (int q = 1; q < gs.mg_nlev; q++) {
        TsLev F = mg_view(c, q - 1);
        const TsLev C = mg_view(c, q);
        /* the coarse operator keeps the couplings across a cut where the coarse level has a
         * halo there (x splits, intermediate levels); the coarsest stays local (its global
         * problem adds the cross couplings itself, mg_global_setup) */
        F.vis = C.hj;
        F.visi = C.hi;
        hipLaunchKernelGGL(k_mg_galerkin, dim3(blocks_for((int64_t)C.n * C.mb * C.l)), dim3(256), 0, s, F, C,
                           gs.mg_off[q].p, gs.mg_diag[q].p);
    }
    for (int q = 0; q + 1 < gs.mg_nlev; q++) {
        const TsLev V = mg_view(c, q);
        hipLaunchKernelGGL(k_mg_fac, dim3(blocks_for((int64_t)V.n * V.mb)), dim3(256), 0, s, V, gs.mg_fac[q].p);
    }
    HIP_OK(hipGetLastError());
    if (gs.mg_hr) {
        /* level 0's couplings, blocks and line factors of the neighbours' edge rows (the
         * halo-row line solves of mg_vcycle) */
        const TsLev V = mg_view(c, 0);
        const int64_t RW = (int64_t)V.n * V.l;
        const int so = c->nb[2], no = c->nb[3];
        std::vector<Msg> y;
        double* const arr[3] = {gs.mg_off[0].p, gs.mg_diag[0].p, gs.mg_fac[0].p};
        const int ncomp[3] = {16, 4, 12};
        for (int q = 0; q < 3; q++) {
            auto row = [&](int jl) { return Seg{arr[q], (V.hj + jl) * RW, ncomp[q], RW, V.cstr}; };
            if (so >= 0) y.push_back({true, so, row(0)});
            if (no >= 0) y.push_back({false, no, row(V.mb)});
            if (no >= 0) y.push_back({true, no, row(V.mb - 1)});
            if (so >= 0) y.push_back({false, so, row(-1)});
        }
        if ((rc = run_msgs(c, y))) return rc;
    }
    /* coarsest level: its dense operator assembled and inverted on the device (Gauss-Jordan
     * with pivoting in one workgroup, schur_cr.hip, up to 192 unknowns); larger coarsest
     * levels and the bands' global coarsest problem go through the host */
    const int qc = gs.mg_nlev - 1;
    const int64_t ncl = (int64_t)gs.mg_n[qc] * gs.mg_m[qc] * l;
    const int N = (int)(2 * ncl);
    if (gs.mg_crd) {
        /* cyclic reduction over the level's longitudes: blocks of one longitude, unknown
         * (jl l + k) 2 + var; the whole problem is its tail, whose explicit inverse is
         * permuted into the level's (var, cell) order for the coarse GEMV */
        SchurCR& cr = gs.mg_cr;
        const int mc = cr.m;
        const size_t mm = (size_t)mc * mc;
        HIP_OK(hipMemsetAsync(cr.dlr.p, 0, sizeof(double) * 3 * (size_t)cr.n * mm, s));
        const TsLev C = mg_view(c, qc);
        hipLaunchKernelGGL(k_mg_cr_expand, dim3(blocks_for(2 * ncl)), dim3(256), 0, s, C, mc, cr.periodic,
                           cr.dlr.p, cr.dlr.p + (size_t)cr.n * mm, cr.dlr.p + 2 * (size_t)cr.n * mm);
        if ((rc = cr_factor_blocks(c, cr))) return rc;
        if ((rc = cr_check(c, cr))) {
            set_error("block GS: singular coarsest T/S operator");
            return rc;
        }
        hipLaunchKernelGGL(k_mg_cr_perm, dim3(blocks_for((int64_t)N * N)), dim3(256), 0, s,
                           (const double*)cr.tinv.p, C, N, gs.mg_cinv.p);
        HIP_OK(hipGetLastError());
        return 0;
    }
    if (N <= 192 && c->nranks <= 1) {
        DevBuf<double>& A = gs.mg_cdense;
        if (A.n < (size_t)N * N && A.alloc((size_t)N * N)) return IEMIC_ENOMEM;
        if (!gs.mg_cinfo.p && gs.mg_cinfo.alloc(1)) return IEMIC_ENOMEM;
        HIP_OK(hipMemsetAsync(A.p, 0, sizeof(double) * N * N, s));
        HIP_OK(hipMemsetAsync(gs.mg_cinfo.p, 0, sizeof(int), s));
        hipLaunchKernelGGL(k_mg_coarse_dense, dim3((unsigned)((N + 63) / 64)), dim3(64), 0, s,
                           (const double*)gs.mg_off[qc].p, (const double*)gs.mg_diag[qc].p, ncl,
                           gs.mg_n[qc], gs.mg_m[qc], l, c->cfg.periodic && c->npx == 1, A.p);
        /* k_cr_inv reads column-major: it inverts A^T and writes the result column-major,
         * which is A^-1 row-major -- the layout k_gemv applies */
        if ((rc = cr_inverse_dev(s, N, A.p, gs.mg_cinv.p, gs.mg_cinfo.p))) return rc;
        int info = 0;
        if ((rc = d2h(c, &info, gs.mg_cinfo.p, sizeof(int)))) return rc;
        if (info) {
            set_error("block GS: singular coarsest T/S operator");
            return IEMIC_EINVAL;
        }
        return 0;
    }
    std::vector<double> off(16 * ncl), dg(4 * ncl);
    if ((rc = d2h(c, off.data(), gs.mg_off[qc].p, sizeof(double) * off.size()))) return rc;
    if ((rc = d2h(c, dg.data(), gs.mg_diag[qc].p, sizeof(double) * dg.size()))) return rc;
    std::vector<double> A((size_t)N * N, 0.0), X;
    const int cn = gs.mg_n[qc], cm = gs.mg_m[qc];
    for (int64_t t = 0; t < ncl; t++) {
        int i, jl, k;
        mg_decode(t, cn, l, i, jl, k);
        for (int R = 0; R < 2; R++) {
            const int64_t row = R * ncl + t;
            A[row * N + R * ncl + t] += dg[(3 * R) * ncl + t];
            A[row * N + (1 - R) * ncl + t] += dg[(1 + R) * ncl + t];
            for (int qq = 0; qq < 8; qq++) {
                const double v = off[(8 * R + qq) * ncl + t];
                if (v == 0.0) continue;
                int ii = i, jj = jl, kk = k;
                const int dir = qq < 6 ? qq : qq - 2;
                switch (dir) {
                case 0: ii--; break;
                case 1: ii++; break;
                case 2: jj--; break;
                case 3: jj++; break;
                case 4: kk--; break;
                default: kk++; break;
                }
                if (jj < 0 || jj >= cm || kk < 0 || kk >= l) continue;
                if (ii < 0 || ii >= cn) {
                    if (!(c->cfg.periodic && c->npx == 1)) continue;
                    ii = (ii + cn) % cn;
                }
                const int64_t nb = ((int64_t)jj * cn + ii) * l + kk;
                const int var = qq < 6 ? R : 1 - R;
                A[row * N + var * ncl + nb] += v;
            }
        }
    }
    dense_inverse(A, N, X);
    if ((rc = h2d(c, gs.mg_cinv.p, X.data(), sizeof(double) * X.size()))) return rc;
    return mg_global_setup(c, off, dg);
}

/* refresh the level-0 iterate's halo columns (phase x, owned rows) and halo rows (phase
 * y, whole rows with their halo columns) -- the subdomains coupled in the T/S smoother */
static int mg_halo(iemic_ctx* c, const TsLev& V)
{
    if (!V.vis && !V.visi) return 0;
    const int64_t W = V.n + 2 * V.hi, L = V.l;
    const int w = c->nb[0], e = c->nb[1], so = c->nb[2], no = c->nb[3];
    std::vector<Msg> x, y;
    for (double* z : {V.z, V.z + V.cstr}) {
        if (V.visi) {
            auto col = [&](int64_t i) { return Seg{z, (V.hj * W + V.hi + i) * L, V.mb, L, W * L}; };
            if (w >= 0) x.push_back({true, w, col(0)});
            if (e >= 0) x.push_back({false, e, col(V.n)});
            if (e >= 0) x.push_back({true, e, col(V.n - 1)});
            if (w >= 0) x.push_back({false, w, col(-1)});
        }
        if (V.vis) {
            auto row = [&](int64_t jl) { return Seg{z, (V.hj + jl) * W * L, 1, W * L, W * L}; };
            if (so >= 0) y.push_back({true, so, row(0)});
            if (no >= 0) y.push_back({false, no, row(V.mb)});
            if (no >= 0) y.push_back({true, no, row(V.mb - 1)});
            if (so >= 0) y.push_back({false, so, row(-1)});
        }
    }
    int rc = run_msgs(c, x);
    if (rc) return rc;
    return run_msgs(c, y);
}

/* the bands' level 0 (mg_hr): the iterate's 2 rows next to each neighbour band, and with b
 * its right-hand side's edge row -- for the halo-row line solves */
static int mg_halo2(iemic_ctx* c, const TsLev& V, bool with_b)
{
    const int64_t RW = (int64_t)V.n * V.l;
    const int so = c->nb[2], no = c->nb[3];
    std::vector<Msg> y;
    for (double* z : {V.z, V.z + V.cstr}) {
        auto rows = [&](int jl) { return Seg{z, (V.hj + jl) * RW, 1, 2 * RW, 2 * RW}; };
        if (so >= 0) y.push_back({true, so, rows(0)});
        if (no >= 0) y.push_back({false, no, rows(V.mb)});
        if (no >= 0) y.push_back({true, no, rows(V.mb - 2)});
        if (so >= 0) y.push_back({false, so, rows(-2)});
    }
    if (with_b)
        for (double* b : {V.b, V.b + V.cstr}) {
            auto row = [&](int jl) { return Seg{b, (V.hj + jl) * RW, 1, RW, RW}; };
            if (so >= 0) y.push_back({true, so, row(0)});
            if (no >= 0) y.push_back({false, no, row(V.mb)});
            if (no >= 0) y.push_back({true, no, row(V.mb - 1)});
            if (so >= 0) y.push_back({false, so, row(-1)});
        }
    return run_msgs(c, y);
}

/* one colour launch of the z-line smoother (C: first post-smoothing sweep, zout: final;
 * hr: the halo rows' lines too, mg_column) */
static int mg_zl(iemic_ctx* c, const TsLev& V, int colour, const TsLev* C, double* zout, int hr = 0)
{
    hipStream_t s = c->stream;
    const int P = mg_lanes(V.l);
    const unsigned g = (unsigned)((mg_columns_of(V, colour, hr) * P + 63) / 64);
    if (!g) return 0;
    const TsLev Cv = C ? *C : V;
    const int corr = C ? 1 : 0;
    MG_LAUNCH_P64(P, k_mg_zl, g, V, colour, Cv, corr, zout, hr);
    return 0;
}

/* the coarsest level: z = A^-1 b (dense), or the bands' global coarsest problem */
static int mg_coarsest(iemic_ctx* c, int q)
{
    BlockGS& gs = c->gs;
    hipStream_t s = c->stream;
    int rc;
    const int N = 2 * gs.mg_n[q] * gs.mg_m[q] * c->l;
    if (gs.mg_glob) {
        /* gather the bands' right-hand sides, own rows of X b */
        const int64_t ncl = N / 2;
        if ((rc = dev_zero(c, gs.mg_gvec.p, gs.mg_gN))) return rc;
        hipLaunchKernelGGL(k_mg_gput, dim3(blocks_for(ncl)), dim3(256), 0, s, gs.mg_b[q].p, ncl,
                           gs.mg_n[q], c->l, gs.mg_gGX, gs.mg_gI0, gs.mg_gJ0, gs.mg_gvec.p);
        if ((rc = allreduce_sum(c, gs.mg_gvec.p, gs.mg_gN))) return rc;
        hipLaunchKernelGGL(k_gemv, dim3((unsigned)((gs.mg_gN + 3) / 4)), dim3(256), 0, s, gs.mg_gX.p,
                           gs.mg_gN, gs.mg_gN, gs.mg_gvec.p, gs.mg_gtmp.p);
        hipLaunchKernelGGL(k_mg_gget, dim3(blocks_for(ncl)), dim3(256), 0, s, gs.mg_gtmp.p, ncl,
                           gs.mg_n[q], c->l, gs.mg_gGX, gs.mg_gI0, gs.mg_gJ0, gs.mg_z[q].p);
        return 0;
    }
    if (N <= 1024)
        hipLaunchKernelGGL(k_gemv_w<16>, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, (const double*)gs.mg_cinv.p,
                           N, (const double*)gs.mg_b[q].p, gs.mg_z[q].p);
    else if (N <= 2048)
        hipLaunchKernelGGL(k_gemv_w<32>, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, (const double*)gs.mg_cinv.p,
                           N, (const double*)gs.mg_b[q].p, gs.mg_z[q].p);
    else
        hipLaunchKernelGGL(k_gemv, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, gs.mg_cinv.p, N, N,
                           gs.mg_b[q].p, gs.mg_z[q].p);
    return 0;
}

/* One V-cycle from level q.  first: the level's iterate started at 0 and its colour-0 lines
 * were relaxed by the launch that formed its right-hand side (k_mg_entry / k_mg_rc).
 * zout: the last level-0 sweep writes z(T, S) into the preconditioner output. */
/* a coarse level visited by the fused launches (k_mg_dn / k_mg_up): two colours, one
 * sweep, no halo on it or on its coarse level (one rank, or the bands' band-local levels) */
static bool mg_fused(iemic_ctx* c, int q)
{
    BlockGS& gs = c->gs;
    if (q < 1 || q + 1 >= gs.mg_nlev || std::max(1, gs.mg_sweeps) != 1 || !gs.mg_zu[q].p) return false;
    const TsLev V = mg_view(c, q), C = mg_view(c, q + 1);
    return mg_ncolour(V) == 2 && !V.hj && !V.hi && !V.vis && !V.visi && !C.hj && !C.hi && C.l == V.l;
}
/* level q as its coarse-correction source: the iterate after its post-smoothing */
static TsLev mg_final(iemic_ctx* c, int q)
{
    TsLev V = mg_view(c, q);
    if (mg_fused(c, q)) V.z = c->gs.mg_zu[q].p;
    return V;
}

static int mg_vcycle(iemic_ctx* c, int q, bool first, double* zout)
{
    BlockGS& gs = c->gs;
    hipStream_t s = c->stream;
    int rc;
    const TsLev V = mg_view(c, q);
    const int nc = mg_ncolour(V), nu = std::max(1, gs.mg_sweeps);
    if (first && !zout && mg_fused(c, q)) {
        /* one launch down (colour 1 + restriction + the coarse colour 0), one launch up */
        const int qc = gs.mg_nlev - 1;
        const TsLev C = mg_view(c, q + 1);
        const int P = mg_lanes(V.l);
        const unsigned g = (unsigned)(C.n * C.mb);
        const int relax = q + 1 < qc ? 1 : 0;
        if (P == 16) hipLaunchKernelGGL(k_mg_dn<16>, dim3(g), dim3(160), 0, s, V, C, relax);
        else if (P == 32) hipLaunchKernelGGL(k_mg_dn<32>, dim3(g), dim3(320), 0, s, V, C, relax);
        else hipLaunchKernelGGL(k_mg_dn<64>, dim3(g), dim3(640), 0, s, V, C, relax);
        if (q + 1 == qc) {
            if ((rc = mg_coarsest(c, q + 1))) return rc;
        } else if ((rc = mg_vcycle(c, q + 1, true, nullptr))) {
            return rc;
        }
        const TsLev Cf = mg_final(c, q + 1);
        double* zu = gs.mg_zu[q].p;
        if (P == 16) hipLaunchKernelGGL(k_mg_up<16>, dim3(g), dim3(160), 0, s, V, Cf, zu);
        else if (P == 32) hipLaunchKernelGGL(k_mg_up<32>, dim3(g), dim3(320), 0, s, V, Cf, zu);
        else hipLaunchKernelGGL(k_mg_up<64>, dim3(g), dim3(640), 0, s, V, Cf, zu);
        return 0;
    }
    /* the bands' level 0, one sweep of two colours from the entry kernel: one exchange of 2
     * rows before each colour-1 launch, which relaxes the halo rows' colour-1 lines too
     * (the neighbour's own lines, operation for operation), so that the restriction and the
     * last colour-0 launch read them without another exchange (4 -> 2 batches per V-cycle) */
    const bool hrel = q == 0 && gs.mg_hr && V.hj == 2 && nu == 1 && nc == 2 && first;
    const int hr = hrel ? ((c->nb[2] >= 0 ? 1 : 0) | (c->nb[3] >= 0 ? 2 : 0)) : 0;
    for (int sw = 0; sw < nu; sw++)
        for (int h = (sw == 0 && first) ? 1 : 0; h < nc; h++) {
            if ((rc = hrel ? mg_halo2(c, V, true) : mg_halo(c, V))) return rc;
            if ((rc = mg_zl(c, V, h, nullptr, nullptr, hrel && h == 1 ? hr : 0))) return rc;
        }
    const int qc = gs.mg_nlev - 1;
    const TsLev C = mg_view(c, q + 1);
    if (!hrel && (rc = mg_halo(c, V))) return rc;
    {
        const int P = mg_lanes(V.l);
        const int shortcut = (first && nu == 1 && nc == 2) ? 1 : 0;
        const int relax = q + 1 < qc ? 1 : 0;
        MG_LAUNCH_P64(P, k_mg_rc, (unsigned)(((int64_t)C.n * C.mb * P + 63) / 64), V, C, shortcut, relax);
    }
    if (q + 1 == qc) {
        if ((rc = mg_coarsest(c, q + 1))) return rc;
    } else if ((rc = mg_vcycle(c, q + 1, true, nullptr))) {
        return rc;
    }
    const TsLev Cf = mg_final(c, q + 1);
    /* coarse correction: added where the first post-smoothing colours read it, or (level 0
     * of a band group, whose lines also read the neighbour bands' rows) explicitly */
    const bool corr = V.hj == 0 && V.hi == 0;
    if (!corr)
        hipLaunchKernelGGL(k_mg_prolong, dim3(blocks_for((int64_t)V.n * V.mb * V.l)), dim3(256), 0, s, V, Cf);
    for (int sw = 0; sw < nu; sw++)
        for (int h = nc - 1; h >= 0; h--) {
            if (hrel) {
                if (h == 1 && (rc = mg_halo2(c, V, false))) return rc;
            } else if ((rc = mg_halo(c, V))) {
                return rc;
            }
            if ((rc = mg_zl(c, V, h, corr && sw == 0 ? &Cf : nullptr, sw + 1 == nu ? zout : nullptr,
                            hrel && h == 1 ? hr : 0)))
                return rc;
        }
    return 0;
}

/* the T/S block solve: right-hand side rr_TS - A_TS,D z_D from the dynamics iterate zd (the
 * planar zP for the multigrid, the AoS output for the sweeps), then ts_mg V-cycles (or
 * ts_sweeps symmetric red-black sweeps), result into z(T, S) of the output z -- for the
 * multigrid only when out (else later by k_mg_out).  side: the V-cycles (which read and
 * write only the multigrid's own buffers once the entry kernel has formed the right-hand
 * side) run on the side stream, forked after the entry kernel; gs_apply joins before
 * k_mg_out. */
static int ts_solve(iemic_ctx* c, const double* zd, double* z, bool out, bool side = false)
{
    BlockGS& gs = c->gs;
    const Lay L = lay_of(c);
    const int n = c->n;
    hipStream_t s = c->stream;
    const unsigned gc = (unsigned)((c->nloc + 255) / 256);
    int rc;
    if (gs.ts_mg > 0) {
        const TsLev V0 = mg_view(c, 0);
        const int P = mg_lanes(c->l);
        const unsigned ge = (unsigned)(((c->nx + MG_TI - 1) / MG_TI) * V0.mb);
        MG_LAUNCH_P(P, k_mg_entry, ge, gs.vp, gs.knP.p, gs.kmask.p, gs.rrP.p, zd, L, V0);
        if (side) {
            HIP_OK(hipEventRecord(c->ev_fork, s));
            HIP_OK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
            c->stream = c->side;
        }
        rc = 0;
        for (int cyc = 0; cyc < gs.ts_mg && !rc; cyc++)
            rc = mg_vcycle(c, 0, cyc == 0, out && cyc + 1 == gs.ts_mg ? z : nullptr);
        if (side) {
            c->stream = s;
            if (rc) return rc;
            HIP_OK(hipEventRecord(c->ev_join, c->side));
        }
        if (rc) return rc;
        HIP_OK(hipGetLastError());
        return 0;
    }
    const int nsw = std::max(1, gs.ts_sweeps);
    if (ts_compact(c)) {
        /* colour-compacted symmetric red-black sweeps */
        const int nblk = (int)((c->nloc + 63) / 64);
        hipLaunchKernelGGL(k_gs_bts2, dim3(8u * (unsigned)((nblk + 7) / 8)), dim3(128), 0, s, gs.vp,
                           gs.known.p, gs.kmask.p, gs.rr.p, z, gs.bc.p, gs.zt.p, gs.zs.p, L, gs.bts.p, nblk);
        const unsigned gh = (unsigned)((c->nloc / 2 + 255) / 256);
        const int seq[4] = {0, 1, 1, 0};
        for (int sw = 0; sw < nsw; sw++)
            for (int h = 0; h < 4; h++)
                hipLaunchKernelGGL(k_gs_ts_half_c, dim3(gh), dim3(256), 0, s, gs.tsc.p, gs.tic.p, gs.bc.p,
                                   gs.zt.p, gs.zs.p, L, seq[h]);
        hipLaunchKernelGGL(k_ts_scatter, dim3(gc), dim3(256), 0, s, gs.known.p, gs.zt.p, gs.zs.p, z, L);
    } else {
        /* symmetric sweeps: colours forward then backward */
        hipLaunchKernelGGL(k_gs_bts, dim3(gc), dim3(256), 0, s, gs.vp, gs.known.p, gs.rr.p, z,
                           gs.bts.p, L);
        const bool four = c->cfg.periodic && (n & 1);
        const int seq2[4] = {0, 1, 1, 0}, seq4[8] = {0, 1, 2, 3, 3, 2, 1, 0};
        const int* seq = four ? seq4 : seq2;
        const int ns = four ? 8 : 4;
        for (int sw = 0; sw < nsw; sw++)
            for (int h = 0; h < ns; h++)
                hipLaunchKernelGGL(k_gs_ts_half, dim3(gc), dim3(256), 0, s, gs.tsoff.p, gs.known.p,
                                   gs.tsinv.p, gs.bts.p, z, L, c->next, seq[h]);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

/* dvb[(h / 64) 4096 + s 64 + h % 64] = val[s nloc + act[h]] (0 past the last active cell) */
__global__ void k_dyn_pack(const double* __restrict__ val, const int* __restrict__ act, int64_t nact,
                           int64_t nloc, double* __restrict__ dvb, int64_t n)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int64_t blk = t >> 12, s = (t >> 6) & 63, l = t & 63, h = blk * 64 + l;
    dvb[t] = h < nact ? val[s * nloc + act[h]] : 0.0;
}

/* the compressed SpMV's stream (krylov.hip k_spmv7c): the active cells of tile pos (a0 ..
 * a0 + na - 1) hold one contiguous run spc[104 a0 ..), slot s of active cell a at
 * 104 a0 + s na + (a - a0) */
__global__ void k_spmv_pack(const double* __restrict__ val, const int* __restrict__ act,
                                const int* __restrict__ apos, const int4* __restrict__ atl, int64_t nact,
                                int64_t nloc, double* __restrict__ spc)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)NSLOT * nact) return;
    const int64_t s = t / nact, a = t - s * nact;
    const int4 td = atl[2 * apos[a]];
    spc[(int64_t)NSLOT * td.z + s * td.w + (a - td.z)] = val[s * nloc + act[a]];
}

/* gs_refresh: *nd += 1 for every owned row whose identity flag (k_known's rule) in the
 * current Jacobian differs from the set-up's */
__global__ void k_known_diff(const double* __restrict__ val, Lay L, int64_t rowintcon,
                             const uint8_t* __restrict__ known, double* __restrict__ nd)
{
    OWNED_CELL;
    int diff = 0;
    for (int r = 0; r < NUN; r++) {
        bool id = val[(int64_t)ROW_BEGIN[r] * ncell + lc] == 1.0;
        for (int s = ROW_BEGIN[r] + 1; id && s < ROW_BEGIN[r + 1]; s++)
            id = val[(int64_t)s * ncell + lc] == 0.0;
        const uint8_t k = (id && NUN * cell + r != rowintcon) ? 1 : 0;
        diff += k != known[NUN * cell + r];
    }
    if (diff) atomicAdd(nd, (double)diff);
}

/* latitude bands: the U/V/W/P rows' coefficients (slots 0 .. 63) of the two halo rows, from
 * the neighbour bands' first / last owned row (BlockGS::dvh: slot-major, the south row's
 * cells, then the north row's) */
static int dyn_halo_coefs(iemic_ctx* c)
{
    BlockGS& gs = c->gs;
    const int64_t row = (int64_t)c->l * c->nx, nloc = c->nloc;
    constexpr int NDS = 64;
    if (gs.dvh.n < (size_t)(NDS * 2 * row)) {
        if (gs.dvh.alloc((size_t)(NDS * 2 * row))) return IEMIC_ENOMEM;
        HIP_OK(hipMemsetAsync(gs.dvh.p, 0, sizeof(double) * gs.dvh.n, c->stream));
    }
    double* v = c->d_val.p;
    const int so = c->nb[2], no = c->nb[3];
    std::vector<Msg> y;
    if (so >= 0) y.push_back({true, so, Seg{v, 0, NDS, row, nloc}});
    if (no >= 0) y.push_back({false, no, Seg{gs.dvh.p, row, NDS, row, 2 * row}});
    if (no >= 0) y.push_back({true, no, Seg{v, nloc - row, NDS, row, nloc}});
    if (so >= 0) y.push_back({false, so, Seg{gs.dvh.p, 0, NDS, row, 2 * row}});
    return run_msgs(c, y);
}

/* The compressed SpMV's coefficient stream (k_spmv7c): the active cells' 104 slots of the
 * current Jacobian, packed at every set-up and by gs_refresh after every later Jacobian */
static int gs_pack_spc(iemic_ctx* c)
{
    BlockGS& gs = c->gs;
    if (gs.nact <= 0 || !gs.act.p) return 0;
    if (gs.spc.n < (size_t)(NSLOT * gs.nact) && gs.spc.alloc((size_t)(NSLOT * gs.nact))) return IEMIC_ENOMEM;
    hipLaunchKernelGGL(k_spmv_pack, dim3(blocks_for(NSLOT * gs.nact)), dim3(256), 0, c->stream, c->d_val.p,
                       (const int*)gs.act.p, (const int*)gs.apos.p, (const int4*)gs.atl.p, gs.nact, c->nloc,
                       gs.spc.p);
    HIP_OK(hipGetLastError());
    return 0;
}

/* A Jacobian assembled while the block GS is set up (Ocean::solve reuses the preconditioner
 * until preProcess flags a rebuild, Ocean.C:790-801, 1360-1374).  The preconditioner stays the
 * operator of the set-up Jacobian, as TRIOS::BlockPreconditioner's extracted blocks do: the
 * assembly wrote into the second Jacobian buffer (assemble_jacobian) and the apply reads the
 * set-up one through BlockGS::vp, together with the copies made from it (gslot, dvh, dvb).
 * What follows the new Jacobian: the compressed SpMV's stream, and whether the set-up's land
 * cells are still identity rows (else the compressed basis would drop live rows: summed over
 * the ranks, so every rank takes the same branch). */
int gs_refresh(iemic_ctx* c)
{
    BlockGS& gs = c->gs;
    if (!gs.coef_stale || !gs.ready || gs.kind != 2) return 0;
    gs.coef_stale = 0;
    if (gs.chk.n < 1 && gs.chk.alloc(1)) return IEMIC_ENOMEM;
    HIP_OK(hipMemsetAsync(gs.chk.p, 0, sizeof(double), c->stream));
    hipLaunchKernelGGL(k_known_diff, dim3((unsigned)((c->nloc + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_val.p, lay_of(c), (int64_t)c->rowintcon, gs.known.p, gs.chk.p);
    int rc = allreduce_sum(c, gs.chk.p, 1);
    if (rc) return rc;
    double nd = 0.0;
    if ((rc = d2h(c, &nd, gs.chk.p, sizeof(double)))) return rc;
    if (nd != 0.0) gs.cmp_ok = 0;
    return gs_pack_spc(c);
}

int gs_compute(iemic_ctx* c, const iemic_krylov* opt)
{
    BlockGS& gs = c->gs;
    gs.ready = 0;
    gs.ts_sweeps = opt ? std::max(0, opt->ts_sweeps) : 3;
    const int64_t NE = c->nerows, next = c->next;
    if (c->l > 64) {
        set_error("block GS: more than 64 levels per column (the column kernels hold a column in one workgroup)");
        return IEMIC_EINVAL;
    }
    const Lay L = lay_of(c);
    int rc = 0;
    if (gs.known.n < (size_t)NE) {
        /* per-cell arrays span the ext layout; the halo entries stay 0 (and the halo rows
         * are identity rows), which is what makes the bands block-Jacobi coupled */
        rc |= gs.known.alloc(NE);
        rc |= gs.uvinv.alloc((size_t)4 * next);
        rc |= gs.tsinv.alloc((size_t)4 * next);
        rc |= gs.pw.alloc(next);
        rc |= gs.rr.alloc(NE);
        rc |= gs.bts.alloc(NE);
        rc |= gs.kmask.alloc((size_t)2 * next);
        rc |= gs.tsoff.alloc((size_t)TS_NC * next);
        rc |= gs.tsc.alloc((size_t)TS_NC * c->nloc);
        rc |= gs.tic.alloc((size_t)4 * c->nloc);
        rc |= gs.bc.alloc((size_t)2 * c->nloc);
        rc |= gs.zt.alloc(next);
        rc |= gs.zs.alloc(next);
        rc |= gs.tcell.alloc(next);
        rc |= gs.tsdiag.alloc((size_t)4 * next);
        rc |= gs.knP.alloc(NE);
        rc |= gs.zP.alloc(NE);
        rc |= gs.rrP.alloc(NE);
        if (rc) {
            set_error("block GS: out of device memory");
            return IEMIC_ENOMEM;
        }
        for (DevBuf<double>* bptr : {&gs.uvinv, &gs.tsinv, &gs.pw, &gs.rr, &gs.bts, &gs.tsoff, &gs.zt,
                                     &gs.zs, &gs.tcell, &gs.tsdiag, &gs.zP, &gs.rrP})
            HIP_OK(hipMemsetAsync(bptr->p, 0, sizeof(double) * bptr->n, c->stream));
        HIP_OK(hipMemsetAsync(gs.kmask.p, 0, sizeof(uint64_t) * gs.kmask.n, c->stream));
        gs.flags_h.clear();
    }
    const unsigned gc = (unsigned)((c->nloc + 255) / 256);
    const unsigned gN = (unsigned)std::min<int64_t>((NE + 255) / 256, 4096);
    HIP_OK(hipMemsetAsync(gs.known.p, 1, NE, c->stream));     /* outer halo rows: identity */
    /* the planar iterate: 0 on the rows no pass writes (identity rows of this Jacobian, T/S) */
    HIP_OK(hipMemsetAsync(gs.zP.p, 0, sizeof(double) * NE, c->stream));
    hipLaunchKernelGGL(k_known, dim3(gc), dim3(256), 0, c->stream, c->d_val.p, L,
                       (int64_t)c->rowintcon, gs.known.p);
    HIP_OK(hipGetLastError());
    if (c->nranks > 1) {
        /* the neighbours' flags of the adjacent latitude rows */
        hipLaunchKernelGGL(k_u8_to_d, dim3(gN), dim3(256), 0, c->stream, gs.known.p, gs.rr.p, NE);
        if ((rc = halo_exchange_w(c, gs.rr.p, NUN, 1))) return rc;
        hipLaunchKernelGGL(k_d_to_u8, dim3(gN), dim3(256), 0, c->stream, gs.rr.p, gs.known.p, NE);
    }
    hipLaunchKernelGGL(k_known_planar, dim3((unsigned)((next + 255) / 256)), dim3(256), 0, c->stream,
                       gs.known.p, gs.knP.p, next);
    {
        /* the active-cell list of the compressed Arnoldi basis (rebuilt when the flags change) */
        if (gs.actf.n < (size_t)c->nloc && gs.actf.alloc(c->nloc)) return IEMIC_ENOMEM;
        hipLaunchKernelGGL(k_cell_active, dim3(gc), dim3(256), 0, c->stream, gs.known.p, L, gs.actf.p);
        std::vector<uint8_t> h((size_t)c->nloc);
        if ((rc = d2h(c, h.data(), gs.actf.p, h.size()))) return rc;
        if (h != gs.act_h) {
            std::vector<int> list;
            list.reserve(h.size());
            for (int64_t q = 0; q < c->nloc; q++)
                if (h[q]) list.push_back((int)q);
            gs.nact = (int64_t)list.size();
            if (gs.act.n < list.size() + 1 && gs.act.alloc(list.size() + 1)) return IEMIC_ENOMEM;
            if (!list.empty() && (rc = h2d(c, gs.act.p, list.data(), sizeof(int) * list.size()))) return rc;
            std::vector<int> cm((size_t)c->nloc, -1);
            for (size_t q = 0; q < list.size(); q++) cm[list[q]] = (int)q;
            if (gs.cmap.n < cm.size() && gs.cmap.alloc(cm.size())) return IEMIC_ENOMEM;
            if ((rc = h2d(c, gs.cmap.p, cm.data(), sizeof(int) * cm.size()))) return rc;
            gs.ric = -1;
            if (c->rowintcon >= 0) {
                const int64_t cell = c->rowintcon / NUN - c->own0;
                if (cell >= 0 && cell < c->nloc && cm[cell] >= 0) gs.ric = (int64_t)NUN * cm[cell] + c->rowintcon % NUN;
            }
            /* the compressed SpMV's tiles (k_spmv7c): 64 cells along i of one grid row, those
             * holding an active cell: tile, first | last active lane << 8, the first active
             * cell a0, the active cells na, the 64-bit active-lane mask (8 ints each) */
            {
                const int nx = c->nx, tpr = (nx + 63) / 64;
                const int64_t nrow = c->nloc / nx;
                std::vector<int> tl, ap((size_t)gs.nact, 0);
                for (int64_t row = 0; row < nrow; row++)
                    for (int ti = 0; ti < tpr; ti++) {
                        const int i0 = ti * 64, nc = std::min(64, nx - i0);
                        int lo = -1, hi = -1;
                        uint64_t mask = 0;
                        for (int cc = 0; cc < nc; cc++)
                            if (h[row * nx + i0 + cc]) {
                                if (lo < 0) lo = cc;
                                hi = cc;
                                mask |= (uint64_t)1 << cc;
                            }
                        if (lo < 0) continue;
                        const int a0 = cm[row * nx + i0 + lo], na = cm[row * nx + i0 + hi] - a0 + 1;
                        for (int a = a0; a < a0 + na; a++) ap[a] = (int)(tl.size() / 8);
                        tl.insert(tl.end(), {(int)(row * tpr + ti), lo | (hi << 8), a0, na, (int)(uint32_t)mask,
                                             (int)(uint32_t)(mask >> 32), 0, 0});
                    }
                gs.natile = (int)(tl.size() / 8);
                if (gs.atl.n < tl.size() + 8 && gs.atl.alloc(tl.size() + 8)) return IEMIC_ENOMEM;
                if (!tl.empty() && (rc = h2d(c, gs.atl.p, tl.data(), sizeof(int) * tl.size()))) return rc;
                if (gs.apos.n < ap.size() + 1 && gs.apos.alloc(ap.size() + 1)) return IEMIC_ENOMEM;
                if (!ap.empty() && (rc = h2d(c, gs.apos.p, ap.data(), sizeof(int) * ap.size()))) return rc;
            }
            gs.act_h.swap(h);
            /* the defect (k_spmv_dyn) writes the active cells only: the others' rows 0 */
            for (DevBuf<double>* bptr : {&gs.dres, &gs.dq})
                if (bptr->p) HIP_OK(hipMemsetAsync(bptr->p, 0, sizeof(double) * bptr->n, c->stream));
        }
    }
    {
        /* global column / U/V-point flags: the Schur structure is that of the whole grid */
        const size_t nf = (size_t)2 * c->n * c->m;
        if (gs.flags_d.n < nf && gs.flags_d.alloc(nf)) return IEMIC_ENOMEM;
        HIP_OK(hipMemsetAsync(gs.flags_d.p, 0, sizeof(double) * nf, c->stream));
        hipLaunchKernelGGL(k_band_flags, dim3((unsigned)((c->nloc / c->l + 255) / 256)), dim3(256), 0, c->stream,
                           gs.known.p, L, gs.flags_d.p);
        if ((rc = allreduce_sum(c, gs.flags_d.p, (int)nf))) return rc;
        std::vector<double> flags(nf);
        if ((rc = d2h(c, flags.data(), gs.flags_d.p, sizeof(double) * nf))) return rc;
        if (flags != gs.flags_h)
            if ((rc = build_structure(c, flags))) return rc;
    }
    if (gs.gslot.n < (size_t)GSL * next) {
        if (gs.gslot.alloc((size_t)GSL * next)) return IEMIC_ENOMEM;
        HIP_OK(hipMemsetAsync(gs.gslot.p, 0, sizeof(double) * gs.gslot.n, c->stream));
    }
    hipLaunchKernelGGL(k_cell_factors, dim3(gc), dim3(256), 0, c->stream, c->d_val.p, gs.known.p,
                       L, (int64_t)c->rowintcon, c->cfg.int_sign, c->d_intc.p, gs.uvinv.p,
                       gs.tsinv.p, gs.pw.p, gs.tsdiag.p, next);
    hipLaunchKernelGGL(k_gslot_pack, dim3(gc), dim3(256), 0, c->stream, c->d_val.p, L, gs.gslot.p);
    if (c->nranks > 1) {
        if ((rc = halo_exchange_w(c, gs.uvinv.p, 4, 1))) return rc;
        if ((rc = halo_exchange_w(c, gs.gslot.p, GSL, 1))) return rc;
    }
    if (c->nranks > 1 && c->npx == 1 && (rc = dyn_halo_coefs(c))) return rc;
    if (gs.nact > 0 && gs.act.p) {
        /* the defect's coefficient stream: the active cells' 64 U/V/W/P slots, blocked per
         * 64 active cells, so a workgroup reads one contiguous 32 KB run and no land lines */
        const int64_t nb = (gs.nact + 63) / 64;
        if (gs.dvb.n < (size_t)(nb * 64 * 64)) {
            if (gs.dvb.alloc((size_t)(nb * 64 * 64))) return IEMIC_ENOMEM;
        }
        hipLaunchKernelGGL(k_dyn_pack, dim3(blocks_for(nb * 64 * 64)), dim3(256), 0, c->stream, c->d_val.p,
                           (const int*)gs.act.p, gs.nact, c->nloc, gs.dvb.p, nb * 64 * 64);
        HIP_OK(hipGetLastError());
    }
    if ((rc = gs_pack_spc(c))) return rc;
    /* the apply reads this Jacobian (a later one is assembled into the other buffer) */
    gs.vp = c->d_val.p;
    gs.coef_stale = 0;
    gs.cmp_ok = 1;
    /* the staged applies write rrP on the active cells only, and leave z's identity rows */
    HIP_OK(hipMemsetAsync(gs.rrP.p, 0, sizeof(double) * gs.rrP.n, c->stream));
    c->kr.zclean = 0;
    if (c->l <= 64) {
        /* the Schur right-hand side as a linear form in rr (k_gs_ptil_rcol) */
        const int64_t ncolb = c->nloc / c->l;
        if (gs.rcol.n < (size_t)(ncolb * RC_NE * c->l) && gs.rcol.alloc((size_t)(ncolb * RC_NE * c->l)))
            return IEMIC_ENOMEM;
        hipLaunchKernelGGL(k_rcol_uvp, dim3(blocks_for(ncolb * c->l)), dim3(256), 0, c->stream, c->d_val.p,
                           gs.known.p, gs.uvinv.p, gs.pw.p, gs.rcol.p, L);
        hipLaunchKernelGGL(k_rcol_w, dim3(blocks_for(ncolb * 9)), dim3(256), 0, c->stream, gs.known.p,
                           gs.gslot.p, gs.rcol.p, L);
    }
    hipLaunchKernelGGL(k_knownmask, dim3(gc), dim3(256), 0, c->stream, c->d_val.p, gs.known.p,
                       gs.kmask.p, L, c->jb1);
    hipLaunchKernelGGL(k_ts_compact, dim3(gc), dim3(256), 0, c->stream, c->d_val.p, gs.known.p,
                       gs.tsoff.p, L, next, (int64_t)c->rowintcon);
    if (ts_compact(c))
        hipLaunchKernelGGL(k_ts_pack, dim3(gc), dim3(256), 0, c->stream, gs.tsoff.p, gs.tsinv.p,
                           gs.tsc.p, gs.tic.p, L, next);
    const int NC = c->n * c->m;
    HIP_OK(hipMemsetAsync(gs.S9.p, 0, sizeof(double) * 9 * (size_t)NC, c->stream));
    const int64_t nt = (int64_t)c->nx * (c->jb1 - c->jb0) * 9;
    hipLaunchKernelGGL(k_schur_build, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_val.p, gs.known.p, gs.uvinv.p, gs.gslot.p, gs.pw.p, gs.col_of_ij.p,
                       gs.pinned.p, L, c->jb1, gs.S9.p);
    /* every band built the rows of its own columns: the sum is the whole Schur matrix */
    if ((rc = allreduce_sum(c, gs.S9.p, 9 * NC))) return rc;
    if ((rc = cr_factor(c, gs.cr, gs.S9.p, gs.col_of_ij.p))) return rc;
    if ((rc = cr_check(c, gs.cr))) return rc;
    gs.ts_mg = opt ? std::max(0, opt->ts_mg) : 0;
    gs.mg_sweeps = opt ? std::max(1, opt->mg_sweeps) : 1;
    if (gs.ts_mg > 0 && (rc = mg_setup(c))) return rc;
    gs.dyn_iters = opt ? std::max(1, opt->dyn_iters) : 1;
    gs.dyn_mr = opt ? (opt->dyn_mr != 0) : 0;
    gs.dyn_omega = opt && opt->dyn_omega > 0.0 ? opt->dyn_omega : 1.0;
    gs.ts_at = opt ? std::max(0, opt->ts_at) : 0;
    gs.schur_passes = opt ? std::max(0, opt->schur_passes) : 0;
    if (gs.dyn_iters > 1 && gs.dres.n < (size_t)NE) {
        if (gs.dres.alloc(NE) || gs.zc.alloc(NE) || gs.dq.alloc(NE) || gs.dzero.alloc(NE) ||
            gs.dmr.alloc(2 * MR_NB + 2))
            return IEMIC_ENOMEM;
        for (DevBuf<double>* bptr : {&gs.dres, &gs.zc, &gs.dq, &gs.dzero})
            HIP_OK(hipMemsetAsync(bptr->p, 0, sizeof(double) * NE, c->stream));
    }
    HIP_OK(hipGetLastError());
    gs.ready = 1;
    return 0;
}

/* dynamics block: z(U/V/W/P) from the right-hand side rr (steps 1-5 of the header), both
 * component-planar (BlockGS::zP); zo: when given, zo += omega z on the active U/V/W/P rows
 * once z is final (the defect correction's update, fused into the pass's last kernels where
 * the column scans run); zaos: the pass's final values (zo's when given) also into the
 * preconditioner output (AoS), on the last pass */
/* rr_halo: rr's halo rows already hold the neighbours' values (the bands' defect computed
 * them itself, spmv_dyn_defect) */
/* schur = false: pbar = 0 (no Schur right-hand side reduction, no Schur solve; the passes
 * gs_pass_schur leaves out) */
/* does dynamics pass it (0 .. dyn_iters - 1) solve the Schur system?  schur_passes k: the first
 * k - 1 passes and the last (k = 1: the first only; 0 or >= dyn_iters: every pass).  The twin
 * at 2 degrees: every pass 203 FGMRES steps; the first and the last 203; the first two 207;
 * the first and the third 205; the first only 300 (profiles/r06_prec_study.md) */
static bool gs_pass_schur(const BlockGS& gs, int it)
{
    const int k = gs.schur_passes, n = gs.dyn_iters;
    return it == 0 || k <= 0 || k >= n || (k >= 2 && (it < k - 1 || it == n - 1));
}

static int dyn_solve(iemic_ctx* c, const double* rr, double* z, double* zo = nullptr, double omega = 0.0,
                     double* zaos = nullptr, bool rr_halo = false, bool schur = true)
{
    BlockGS& gs = c->gs;
    const Lay L = lay_of(c);
    const unsigned gc = (unsigned)((c->nloc + 255) / 256);
    hipStream_t s = c->stream;
    const bool band = c->nranks > 1;
    int rc = 0;
    const int64_t ncolb = c->nloc / c->l;                        /* water columns of the band */
    const int Pl = c->l <= 16 ? 16 : (c->l <= 32 ? 32 : 64);     /* l <= 64 (gs_compute) */
    /* transposed column kernels: 1024 / Pl columns of one row per workgroup of 1024 threads */
    const int cti = 1024 / Pl;
    const unsigned gct = xcd_grid(((c->nx + cti - 1) / cti) * (ncolb / c->nx));
    const dim3 bct(1024u);
    const int64_t ps = c->next;
    /* ptil and the Schur right-hand side in one column pass (rcol), the U/V points once
     * after the Schur solve, then p and w */
    /* latitude bands: after the one exchange of rr, the pass computes ptil on both halo rows
     * and the U/V points of the south one itself (the halo-filled gslot holds their
     * couplings) instead of exchanging ptil and uv (3 -> 1 exchange batch per pass) */
    const bool hrow = band && c->npx == 1;
    const double* gsl = hrow ? gs.gslot.p : nullptr;
    const unsigned gcth = hrow ? xcd_grid(((c->nx + cti - 1) / cti) * (ncolb / c->nx + 2)) : gct;
    if (band && !rr_halo && (rc = halo_exchange_planar(c, const_cast<double*>(rr), NUN, ps, 1))) return rc;   /* rr around the band */
    {
        auto kp = Pl == 16 ? (schur ? k_gs_ptil_rcol<16, true> : k_gs_ptil_rcol<16, false>)
                : Pl == 32 ? (schur ? k_gs_ptil_rcol<32, true> : k_gs_ptil_rcol<32, false>)
                           : (schur ? k_gs_ptil_rcol<64, true> : k_gs_ptil_rcol<64, false>);
        hipLaunchKernelGGL(kp, dim3(gcth), bct, 0, s, gs.vp, gs.knP.p, gs.rcol.p, rr, z, gs.ocol.p,
                           gs.colv_own.p, L, gsl);
    }
    if (band && !hrow && (rc = halo_exchange_planar(c, z, NUN, ps, 1))) return rc;   /* ptil above the band */
    const double* sb = gs.colv_own.p;
    const double* pbT = schur ? gs.colvT.p : gs.colvZ.p;
    if (band && schur) {
        HIP_OK(hipMemcpyAsync(gs.colv.p, gs.colv_own.p, sizeof(double) * c->n * c->m,
                              hipMemcpyDeviceToDevice, s));
        if ((rc = allreduce_sum(c, gs.colv.p, c->n * c->m))) return rc;
        sb = gs.colv.p;
    }
    if (schur && (rc = cr_solve(c, gs.cr, sb, gs.colv2.p, s, gs.colvT.p))) return rc;
    const bool al = gs.act.p && gs.nact > 0;
    const int64_t nown = al ? gs.nact : c->nloc;
    const unsigned gcu = (unsigned)((nown + (hrow ? (int64_t)c->l * c->nx : 0) + 255) / 256);
    hipLaunchKernelGGL(k_gs_uvp, dim3(gcu), dim3(256), 0, s, gs.vp, gs.knP.p, gs.uvinv.p,
                       rr, pbT, z, L, zo, omega, zaos, gsl, al ? gs.act.p : nullptr, nown);
    if (band && !hrow && (rc = halo_exchange_planar(c, z, NUN, ps, 1))) return rc;   /* uv below the band */
    if (Pl == 16)
        hipLaunchKernelGGL(k_gs_pw_t<16>, dim3(gct), bct, 0, s, gs.vp, gs.knP.p,
                           pbT, z, L, rr, zo, omega, zaos);
    else if (Pl == 32)
        hipLaunchKernelGGL(k_gs_pw_t<32>, dim3(gct), bct, 0, s, gs.vp, gs.knP.p,
                           pbT, z, L, rr, zo, omega, zaos);
    else
        hipLaunchKernelGGL(k_gs_pw_t<64>, dim3(gct), bct, 0, s, gs.vp, gs.knP.p,
                           pbT, z, L, rr, zo, omega, zaos);
    return 0;
}

int spmv_dyn_defect(iemic_ctx* c, const double* z, const double* r, const uint8_t* knP, double* d, bool halo = false);

/* GPU time of the apply's parts (HIP events on the library stream, nrep back-to-back
 * launches each, zero data): us[0] one Schur solve (cyclic reduction), us[1] one T/S block
 * solve (right-hand side + V-cycle), us[2] one dynamics pass (column kernels + Schur solve),
 * us[3] one dynamics defect.  Diagnostics for DESIGN.md's per-part table (one rank). */
int gs_time_parts(iemic_ctx* c, int nrep, double* us)
{
    BlockGS& gs = c->gs;
    if (!gs.ready || gs.kind != 2 || nrep < 1) {
        set_error("gs_time_parts: the block GS preconditioner is not computed");
        return IEMIC_ESTATE;
    }
    if (c->nranks > 1) {   /* parts 2 and 3 exchange halos: not callable on one rank alone */
        set_error("gs_time_parts: one-rank diagnostic, the context has " + std::to_string(c->nranks) + " ranks");
        return IEMIC_EINVAL;
    }
    hipStream_t s = c->stream;
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    double* z = c->d_tmp2.p;
    HIP_OK(hipMemsetAsync(c->d_tmp1.p, 0, sizeof(double) * c->nerows, s));
    HIP_OK(hipMemsetAsync(z, 0, sizeof(double) * c->nerows, s));
    HIP_OK(hipMemsetAsync(gs.rr.p, 0, sizeof(double) * c->nerows, s));
    HIP_OK(hipMemsetAsync(gs.rrP.p, 0, sizeof(double) * c->nerows, s));
    HIP_OK(hipMemsetAsync(gs.zP.p, 0, sizeof(double) * c->nerows, s));
    HIP_OK(hipMemsetAsync(gs.colv_own.p, 0, sizeof(double) * c->n * c->m, s));
    int rc = 0;
    for (int part = 0; part < 4 && !rc; part++) {
        auto once = [&]() -> int {
            switch (part) {
            case 0: return cr_solve(c, gs.cr, gs.colv_own.p, gs.colv2.p, s);
            case 1: return ts_solve(c, gs.ts_mg > 0 ? gs.zP.p : z, z, true);
            case 2: return dyn_solve(c, gs.rrP.p, gs.zP.p);
            default: return spmv_dyn_defect(c, gs.zP.p, c->d_tmp1.p, gs.knP.p, gs.dres.p ? gs.dres.p : c->d_tmp1.p);
            }
        };
        if ((rc = once())) break;                  /* warm */
        HIP_OK(hipEventRecord(e0, s));
        for (int q = 0; q < nrep && !rc; q++) rc = once();
        HIP_OK(hipEventRecord(e1, s));
        HIP_OK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, e0, e1));
        us[part] = 1e3 * ms / nrep;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

static int gs_apply_impl(iemic_ctx* c, const double* r, double* z, bool cmp, bool staged = false);
int gs_apply(iemic_ctx* c, const double* r, double* z) { return gs_apply_impl(c, r, z, false); }
int gs_apply_c(iemic_ctx* c, const double* rc, double* z, bool staged) { return gs_apply_impl(c, rc, z, true, staged); }

static int gs_apply_impl(iemic_ctx* c, const double* r, double* z, bool cmp, bool staged)
{
    BlockGS& gs = c->gs;
    const Lay L = lay_of(c);
    const unsigned gc = (unsigned)((c->nloc + 255) / 256);
    hipStream_t s = c->stream;
    const bool band = c->nranks > 1;
    const int64_t ps = c->next;
    double* zP = gs.zP.p;
    int rc = gs_refresh(c);
    if (rc) return rc;
    /* the T/S block is solved with the right-hand side rr_TS - A_TS,D z_D of the dynamics
     * iterate after ts_at passes (default: after the last; the CPU twin: orc_gs_apply); the
     * later passes neither read nor write the T/S rows */
    const int ts_at = (!gs.dyn_mr && gs.ts_at >= 1 && gs.ts_at < gs.dyn_iters) ? gs.ts_at : gs.dyn_iters;
    /* early T/S on one rank: its V-cycles run on the side stream beside the remaining
     * dynamics passes (both chains are latency-bound, so they overlap) */
    const bool par = ts_at < gs.dyn_iters && !band && gs.ts_mg > 0;
    /* the dynamics passes iterate on the planar zP; the output z (AoS) gets their final
     * values from the last pass (every pass for the T/S sweeps, which read z's AoS rows) */
    const bool aos_all = gs.ts_mg <= 0;
    auto zaos_of = [&](bool last) { return (last || aos_all) ? z : nullptr; };
    /* latitude bands: the last pass also updated the iterate's south halo row U/V (k_gs_uvp),
     * all the T/S right-hand side reads of it beyond the band (A_TS,D couples U/V at j - 1 and
     * W in the column): no exchange (the fixed-step passes only) */
    const bool ts_local = band && c->npx == 1 && gs.ts_mg > 0 && !gs.dyn_mr && ts_at == gs.dyn_iters &&
                          gs.dyn_iters > 1;
    auto ts = [&]() -> int {
        if (band && !ts_local && (ts_at < gs.dyn_iters || gs.dyn_iters > 1)) {
            rc = gs.ts_mg > 0 ? halo_exchange_planar(c, zP, NUN, ps, 1) : halo_exchange(c, z, 1);
            if (rc) return rc;
        }
        return ts_solve(c, gs.ts_mg > 0 ? zP : z, z, ts_at == gs.dyn_iters, par);
    };
    /* the halo rows of r hold the neighbours' identity-row values the couplings need (a
     * compressed r is zero on every identity row: no couplings, no exchange) */
    if (cmp) {
        /* staged: the update pass wrote rrP (its land entries stay 0 since the set-up, the
         * identity rows of z were zeroed per set-up: Krylov::zclean) */
        if (!staged || aos_all)
            hipLaunchKernelGGL(k_gs_rr_c, dim3(gc), dim3(256), 0, s, gs.known.p, gs.cmap.p, r, z,
                               aos_all ? gs.rr.p : nullptr, aos_all ? 1 : 0, gs.rrP.p, L);
    } else {
        if (band && (rc = halo_exchange(c, const_cast<double*>(r), 1))) return rc;
        hipLaunchKernelGGL(k_gs_rr, dim3(gc), dim3(256), 0, s, gs.vp, gs.known.p, gs.kmask.p,
                           r, z, aos_all ? gs.rr.p : nullptr, aos_all ? 1 : 0, gs.rrP.p, L);
    }
    if ((rc = dyn_solve(c, gs.rrP.p, zP, nullptr, 0.0, zaos_of(gs.dyn_iters == 1)))) return rc;
    if (ts_at == 1 && gs.dyn_iters > 1 && (rc = ts())) return rc;
    /* defect correction on the dynamics block: z_D += w M_D^-1 (rr_D - A_DD z_D), with the
     * minimal-residual w (dyn_mr) or the fixed w = dyn_omega */
    if (gs.dyn_mr && gs.dyn_iters > 1) {
        if (band && (rc = halo_exchange_planar(c, zP, NUN, ps, 1))) return rc;
        if ((rc = spmv_dyn_defect(c, zP, gs.rrP.p, gs.knP.p, gs.dres.p))) return rc;
        for (int it = 1; it < gs.dyn_iters; it++) {
            const bool last = it + 1 == gs.dyn_iters;
            if ((rc = dyn_solve(c, gs.dres.p, gs.zc.p))) return rc;
            if (band && (rc = halo_exchange_planar(c, gs.zc.p, NUN, ps, 1))) return rc;
            if ((rc = spmv_dyn_defect(c, gs.zc.p, gs.dzero.p, gs.knP.p, gs.dq.p))) return rc;
            hipLaunchKernelGGL(k_mr_dots, dim3(MR_NB), dim3(256), 0, s, gs.dres.p, gs.dq.p, L, gs.dmr.p);
            hipLaunchKernelGGL(k_mr_sum, dim3(1), dim3(64), 0, s, gs.dmr.p, MR_NB);
            if (band && (rc = allreduce_sum(c, gs.dmr.p + 2 * MR_NB, 2))) return rc;
            hipLaunchKernelGGL(k_mr_update, dim3(gc), dim3(256), 0, s, gs.knP.p, gs.dmr.p + 2 * MR_NB,
                               gs.zc.p, gs.dq.p, zP, gs.dres.p, L, last ? 0 : 1, zaos_of(last));
        }
    }
    /* latitude bands: the defect on the two halo rows too (from a 2-deep halo of the U/V/W/P
     * planes), so that the pass needs no exchange of it (2 -> 1 exchange batch per pass) */
    const bool dhalo = band && c->npx == 1 && gs.dvh.p;
    for (int it = 1; !gs.dyn_mr && it < gs.dyn_iters; it++) {
        const bool last = it + 1 == gs.dyn_iters;
        if (band && (rc = dhalo ? halo_exchange_planar(c, zP, 4, ps, 2) : halo_exchange_planar(c, zP, NUN, ps, 1)))
            return rc;   /* w, p of the neighbours */
        if ((rc = spmv_dyn_defect(c, zP, gs.rrP.p, gs.knP.p, gs.dres.p, dhalo))) return rc;
        const bool schur = gs_pass_schur(gs, it);
        if ((rc = dyn_solve(c, gs.dres.p, gs.zc.p, zP, gs.dyn_omega, zaos_of(last), dhalo, schur)))
            return rc;   /* z += w zc */
        if (it + 1 == ts_at && it + 1 < gs.dyn_iters && (rc = ts())) return rc;
    }
    if (ts_at == gs.dyn_iters && (rc = ts())) return rc;
    if (ts_at < gs.dyn_iters && gs.ts_mg > 0) {
        if (par) HIP_OK(hipStreamWaitEvent(s, c->ev_join, 0));   /* join */
        const TsLev V0 = mg_view(c, 0);
        hipLaunchKernelGGL(k_mg_out, dim3(blocks_for((int64_t)V0.n * V0.mb * V0.l)), dim3(256), 0, s, V0, z);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

}  // namespace iemic
