/*
 * krylov.hip -- stencil-ELL SpMV and the flexible GMRES driver.
 *
 *  - k_spmv7 replaces Epetra_CrsMatrix::Apply (Ocean::applyMatrix, src/ocean/Ocean.C:1352-1357)
 *    on the maximal graph: one workgroup per 64-cell tile of a grid row stages the x values
 *    of the tile's neighbourhood in LDS and four waves share the 104 slot-major coefficient
 *    rows (read non-temporally); columns are implicit in the cell index and slot.  The dense
 *    integral-condition row (SRES = 0, THCM.C:2121-2198) is a separate fused dot.
 *  - k_spmv_dyn: the U/V/W/P rows only (the dynamics defect of the block GS).
 *  - fgmres restates Belos BlockGmresSolMgr as configured by Ocean::initializeBelos
 *    (Ocean.C:961-1020): flexible (right) preconditioning, x0 = 0, residual relative to
 *    ||b|| (the preconditioned initial residual for right preconditioning), classical
 *    Gram-Schmidt with one full re-orthogonalisation pass (DGKS-like), Givens updates of
 *    the least-squares problem, restarts, and the explicit residual check of
 *    Ocean::solve (Ocean.C:1140-1150).
 */
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>

#include <hip/hip_ext.h>

#include "common.h"

namespace iemic {

/* ---- SpMV ------------------------------------------------------------------------ */
/* ---- k_spmv7: LDS-staged x, slot-balanced waves ----------------------------------------
 * One workgroup (4 waves) per tile of up to 64 cells along i of one (j, k) grid row.  The
 * x values of the tile's neighbourhood -- the six (dj, dk) grid rows the slot table reaches
 * ((0,0), (+-1,0), (0,+-1), (+1,-1)), cells i0-1 .. i0+64, all six unknowns -- are copied
 * into LDS with contiguous loads, so the 104 gathers per cell become LDS reads.  The 104
 * slots are split into four runs of 26 (one per wave: U+V, V+W, W+P+T, T+S) instead of one
 * wave per equation (24/22/7/11/20/20), so the waves of a tile finish together; their row
 * partials meet in LDS and the 384 results of the tile are stored contiguously. */
constexpr int SP7_T = 64;
__host__ __device__ constexpr int sp7_row(int s)
{
    return s < 24 ? 0 : s < 46 ? 1 : s < 53 ? 2 : s < 64 ? 3 : s < 84 ? 4 : 5;
}
__host__ __device__ constexpr int sp7_combo(int dj, int dk)
{
    return dk == 0 ? (dj + 1) : (dk == -1 ? (dj == 0 ? 3 : 5) : 4);  /* (-1,0)0 (0,0)1 (1,0)2 (0,-1)3 (0,1)4 (1,-1)5 */
}
/* the coefficient stream is read once per SpMV: non-temporal loads (in-solve 43.4 us vs
 * 45.9 us with the default policy at 2 degrees) */
template <int S0, int S1>
__device__ __forceinline__ void sp7_load(const double* __restrict__ val, int64_t nloc, int64_t lc, bool act,
                                         double* v)
{
    /* an inactive lane's v is left undefined (its sums are never stored): no merge point
     * that would wait for the loads before the staging's are issued */
    if (act) {
#pragma unroll
        for (int s = S0; s < S1; s++) v[s - S0] = __builtin_nontemporal_load(val + (int64_t)s * nloc + lc);
    }
}
template <int S0, int S1>
__device__ __forceinline__ void sp7_compute(const double* v, const double* xs, int c, double* acc)
{
#pragma unroll
    for (int s = S0; s < S1; s++) {
        const Slot sl = SLOTS[s];
        const int q = sp7_combo(sl.dj, sl.dk);
        acc[sp7_row(s) - sp7_row(S0)] += v[s - S0] * xs[(q * (SP7_T + 2) + (c + 1 + sl.di)) * NUN + sl.var];
    }
}
/* the full SpMV (FGMRES's compressed basis uses k_spmv7c below) */
__global__ void __launch_bounds__(256) k_spmv7(SubLay X, const double* __restrict__ val,
                                               const double* __restrict__ x,
                                               double* __restrict__ y, int nloc, int ntile, int tpr)
{
    __shared__ double xs[6 * (SP7_T + 2) * NUN];
    __shared__ double red[4][3][SP7_T];
    const int l = X.l, nx = X.nx;
    const int per = (ntile + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= ntile) return;
    const int row = tile / tpr, i0 = (tile - row * tpr) * SP7_T;
    const int k = row % l, jl = row / l, j = X.jb0 + jl;
    const int nc = min(SP7_T, nx - i0);
    const int lc0 = row * nx + i0;
    const int t = threadIdx.x, c = t & 63;
    const int g = __builtin_amdgcn_readfirstlane(t >> 6);   /* wave-uniform: scalar branches */
    const bool act = c < nc;
    const int64_t lc = lc0 + c;
    double acc[3] = {0.0, 0.0, 0.0};
    double v[26];
    /* the coefficient loads first (one predicated block), then the x staging's loads, all
     * issued before the first LDS store: one memory latency per tile instead of one per
     * staging round (the staging loop waited for each load before its store) */
    if (g == 0) sp7_load<0, 26>(val, nloc, lc, act, v);
    else if (g == 1) sp7_load<26, 52>(val, nloc, lc, act, v);
    else if (g == 2) sp7_load<52, 78>(val, nloc, lc, act, v);
    else sp7_load<78, 104>(val, nloc, lc, act, v);
    /* stage x: 6 grid rows x (nc + 2) cells x 6 unknowns, contiguous runs (the two end
     * cells: the neighbour columns, from the x halo when the x direction is split) */
    {
        const int jm = j > 0 ? j - 1 : j, jp = j < X.m - 1 ? j + 1 : j;
        const int km = k > 0 ? k - 1 : k, kp = k < l - 1 ? k + 1 : k;
        const int rj[6] = {jm, j, jp, j, j, jp}, rk[6] = {k, k, k, km, kp, km};
        /* element e of the LDS image is (q (SP7_T + 2) + p) NUN + var: constant divisors */
        constexpr int PR = (SP7_T + 2) * NUN;
        constexpr int SPT = (6 * PR + 255) / 256;
        const int lim = (nc + 2) * NUN;
        double xv[SPT];
        int xo[SPT];
#pragma unroll
        for (int u = 0; u < SPT; u++) {
            const int e = t + 256 * u;
            const int q = e / PR, w = e - q * PR;
            xo[u] = -1;
            if (e < 6 * PR && w < lim) {
                const int p = w / NUN, var = w - p * NUN;
                const int64_t r = (int64_t)(rj[q] - X.jb0 + HALO) * l + rk[q];
                const int64_t cell = (p == 0 || p == nc + 1)
                                         ? xnb_cell(r, i0 + p - 1, X.n, X.ib0, nx, X.hx, X.periodic, X.xb)
                                         : r * nx + i0 + p - 1;
                xo[u] = e;
                xv[u] = x[NUN * cell + var];
            }
        }
#pragma unroll
        for (int u = 0; u < SPT; u++)
            if (xo[u] >= 0) xs[xo[u]] = xv[u];
    }
    __syncthreads();
    if (g == 0) sp7_compute<0, 26>(v, xs, c, acc);
    else if (g == 1) sp7_compute<26, 52>(v, xs, c, acc);
    else if (g == 2) sp7_compute<52, 78>(v, xs, c, acc);
    else sp7_compute<78, 104>(v, xs, c, acc);
#pragma unroll
    for (int q = 0; q < 3; q++) red[g][q][c] = acc[q];
    __syncthreads();
    /* rows of the groups: g0 {U,V} g1 {V,W} g2 {W,P,T} g3 {T,S}; first row of group g */
    for (int o = t; o < nc * NUN; o += 256) {
        const int cc = o / NUN, R = o - cc * NUN;
        double v;
        switch (R) {
        case 0: v = red[0][0][cc]; break;
        case 1: v = red[0][1][cc] + red[1][0][cc]; break;
        case 2: v = red[1][1][cc] + red[2][0][cc]; break;
        case 3: v = red[2][1][cc]; break;
        case 4: v = red[2][2][cc] + red[3][0][cc]; break;
        default: v = red[3][1][cc]; break;
        }
        y[NUN * ((int64_t)HALO * l * nx + lc0) + o] = v;
    }
}

/* k_spmv7c: the in-solve SpMV of FGMRES's compressed basis (round 6).  k_spmv7 reads the
 * slot-major Jacobian, whose 128-byte coefficient lines hold 16 cells: the lines of mixed land /
 * water runs are fetched whole (at 2 degrees 128.9 MB of coefficient lines for 100.7 MB of
 * active coefficients; round 5's land-skipping variant moved 147 MB per launch, 1.25x).
 *  - Coefficients: BlockGS::spc holds the active cells' 104 slots blocked per tile -- the na
 *    active cells of a tile (consecutive in the compressed order, from a0) as one contiguous
 *    run of 104 na doubles, slot s of the tile's r-th active cell at 104 a0 + s na + r -- so a
 *    workgroup streams one run that no land cell and no other tile shares (PMC: 117.1 MB per
 *    launch against 117.7 MB algorithmic; slot-major packing over the active list: 124.9 MB,
 *    3.4 us slower).
 *  - Tiles: only the 64-cell tiles (one grid row) that hold an active cell are launched
 *    (BlockGS::atl: tile, first / last active lane, a0, na and the 64-bit active-lane mask, so
 *    a lane finds its compressed index by a popcount instead of a dependent load), dealt to
 *    the 8 XCDs in contiguous runs.
 *  - x: the six (dj, dk) neighbour rows' interior cells are contiguous runs in x and in the
 *    LDS image, copied by LDS-DMA (global_load_lds_dwordx4, no VGPR destination: 94 instead
 *    of 104 VGPRs, 5 waves per SIMD instead of 4; 32.5 -> 29.2 us), pieces beyond the active
 *    cells' reach skipped; the two end cells of each row by plain loads.
 * Same sums in the same order as k_spmv7: the compressed rows are bitwise its rows. */
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;
__global__ void __launch_bounds__(256) k_spmv7c(SubLay X, const double* __restrict__ spc,
                                                const double* __restrict__ x, double* __restrict__ y,
                                                const int4* __restrict__ atl, int natile, int tpr)
{
    __shared__ double xs[6 * (SP7_T + 2) * NUN];
    __shared__ double red[4][3][SP7_T];
    __shared__ int lof[SP7_T];
    const int l = X.l, nx = X.nx;
    const int per = (natile + 7) >> 3;
    const int pos = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (pos >= natile) return;
    const int4 td = atl[2 * pos], tm = atl[2 * pos + 1];
    const int tile = td.x, clo = td.y & 255, chi = td.y >> 8, a0 = td.z;
    /* the tile's active lanes: a 64-bit mask, so a lane finds its compressed index without a
     * dependent load (cm = a0 + active lanes below it) */
    const uint64_t amask = (uint64_t)(uint32_t)tm.x | ((uint64_t)(uint32_t)tm.y << 32);
    const int row = tile / tpr, i0 = (tile - row * tpr) * SP7_T;
    const int k = row % l, jl = row / l, j = X.jb0 + jl;
    const int nc = min(SP7_T, nx - i0);
    const int t = threadIdx.x, c = t & 63;
    const int g = __builtin_amdgcn_readfirstlane(t >> 6);   /* wave-uniform: scalar branches */
    const bool act = (amask >> c) & 1;
    const int cm = act ? a0 + __builtin_popcountll(amask & ((1ull << c) - 1)) : -1;
    if (g == 0 && act) lof[cm - a0] = c;                    /* active cell -> its lane */
    double acc[3] = {0.0, 0.0, 0.0};
    double v[26];
    /* coefficient loads, then the staging loads, all issued before the first LDS store */
    const double* vb = spc + (int64_t)NSLOT * a0;
    const int64_t vs = td.w, vo = cm - a0;
    if (g == 0) sp7_load<0, 26>(vb, vs, vo, act, v);
    else if (g == 1) sp7_load<26, 52>(vb, vs, vo, act, v);
    else if (g == 2) sp7_load<52, 78>(vb, vs, vo, act, v);
    else sp7_load<78, 104>(vb, vs, vo, act, v);
    {
        /* the interior cells i0 .. i0 + nc - 1 of each of the six grid rows are one contiguous
         * run of nc * 48 bytes in x and in the LDS image: copied by LDS-DMA in 1 KiB pieces (a
         * wave-instruction of 16 bytes per lane, no VGPR destination), the pieces outside the
         * active cells' reach skipped; the two end cells of each row (the neighbour columns,
         * from the x halo when the x direction is split) by 72 plain loads */
        const int jm = j > 0 ? j - 1 : j, jp = j < X.m - 1 ? j + 1 : j;
        const int km = k > 0 ? k - 1 : k, kp = k < l - 1 ? k + 1 : k;
        const int rj[6] = {jm, j, jp, j, j, jp}, rk[6] = {k, k, k, km, kp, km};
        const int lane = t & 63, nb = nc * NUN * 8;
        const int blo = max(0, (clo - 1) * NUN * 8), bhi = min(nb, (chi + 2) * NUN * 8);
        for (int u = g; u < 18; u += 4) {
            const int q = u / 3, h = u - 3 * q;
            if (h * 1024 >= bhi || (h + 1) * 1024 <= blo) continue;        /* wave-uniform */
            const int byte = h * 1024 + lane * 16;
            const int64_t r = (int64_t)(rj[q] - X.jb0 + HALO) * l + rk[q];
            if (byte < nb)
                __builtin_amdgcn_global_load_lds((glb_void*)(x + NUN * (r * nx + i0) + byte / 8),
                                                 (lds_void*)(xs + (q * (SP7_T + 2) + 1) * NUN + h * 128), 16, 0, 0);
    }
        if (t < 72) {
            const int q = t / 12, side = (t / NUN) & 1, var = t - NUN * (t / NUN);
            const int p = side ? nc + 1 : 0;
            const int64_t r = (int64_t)(rj[q] - X.jb0 + HALO) * l + rk[q];
            const int64_t cell = xnb_cell(r, i0 + p - 1, X.n, X.ib0, nx, X.hx, X.periodic, X.xb);
            xs[(q * (SP7_T + 2) + p) * NUN + var] = x[NUN * cell + var];
    }
    }
    __syncthreads();
    if (act) {
        if (g == 0) sp7_compute<0, 26>(v, xs, c, acc);
        else if (g == 1) sp7_compute<26, 52>(v, xs, c, acc);
        else if (g == 2) sp7_compute<52, 78>(v, xs, c, acc);
        else sp7_compute<78, 104>(v, xs, c, acc);
    }
#pragma unroll
    for (int q = 0; q < 3; q++) red[g][q][c] = acc[q];
    __syncthreads();
    /* rows of the groups: g0 {U,V} g1 {V,W} g2 {W,P,T} g3 {T,S}; the tile's active cells are
     * consecutive in the compressed vector, so its rows [6 cm(clo), 6 cm(chi) + 6) are one
     * contiguous run: thread o writes entry o of it */
    const int na = td.w;
    for (int o = t; o < na * NUN; o += 256) {
        const int ac = o / NUN, R = o - ac * NUN;
        const int cc = lof[ac];
        double vv;
        switch (R) {
        case 0: vv = red[0][0][cc]; break;
        case 1: vv = red[0][1][cc] + red[1][0][cc]; break;
        case 2: vv = red[1][1][cc] + red[2][0][cc]; break;
        case 3: vv = red[2][1][cc]; break;
        case 4: vv = red[2][2][cc] + red[3][0][cc]; break;
        default: vv = red[3][1][cc]; break;
        }
        y[(int64_t)NUN * a0 + o] = vv;
    }
}

/* Dynamics defect of the block GS (prec_gs.hip): d = rr - A z on the active U/V/W/P rows,
 * 0 on the others.  z is the pass iterate, 0 on the identity rows (whose couplings are in
 * rr, the block right-hand side) and on T/S, so rr - A z equals rr_D - A_DD z_D of the
 * block iteration.  One workgroup per 64 cells; the 64 slots of the four rows are split
 * evenly over the waves (U | U+V | V+W | W+P, 16 each), the gathers read z directly, and
 * the rows' partials meet in LDS.  z, rr, the flags and d are all component-planar (plane
 * stride ps: unit-stride along i; round 4 read r as 48-byte AoS records).  Skipping the W
 * row's four T/S slots (z(T, S) = 0) measured slower (24.7 against 22.5 us: the waves'
 * balance), so they are read. */
/* on[q]: row sp7_row(S0) + q of the cell is active; an identity row's coefficients are
 * neither loaded nor used (about half the cells are land at 2 degrees).  (Non-temporal
 * coefficient loads measured 35.6 against 26.1 us per defect, scripts/ab_probe.py.) */
/* The loads of each row are issued in one predicated block (per-slot predicates made the
 * compiler wait for every load before the next: 64 vmcnt(0) per wave), then the products
 * are summed in slot order. */
template <int S0, int S1>
__device__ __forceinline__ void dyn_partial(const double* __restrict__ val, const double* __restrict__ z,
                                            int64_t vs, const int (*nc)[9], const bool* on,
                                            int64_t ps, double* acc)
{
    constexpr int NS = S1 - S0;
    double v[NS], zz[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) v[s] = zz[s] = 0.0;
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if (!on[q]) continue;
#pragma unroll
        for (int s = S0; s < S1; s++) {
            const Slot sl = SLOTS[s];
            if (sp7_row(s) - sp7_row(S0) != q) continue;
            const int cidx = nc[sl.di + 1][(sl.dk + 1) * 3 + (sl.dj + 1)];
            v[s - S0] = val[(int64_t)s * vs];
            zz[s - S0] = z[(int64_t)cidx + ps * sl.var];
        }
    }
#pragma unroll
    for (int s = S0; s < S1; s++) {
        const int q = sp7_row(s) - sp7_row(S0);
        if (on[q]) acc[q] += v[s - S0] * zz[s - S0];
    }
}
/* hv (latitude bands): tiles past the owned ones compute the defect on the two halo rows
 * too (their coefficients exchanged once per Jacobian, BlockGS::dvh; z with a 2-deep halo),
 * so that the next dynamics pass needs no exchange of d.  hs / hn: the south / north halo row
 * exists (a neighbour band).  alist: the owned tiles run over the active cells only (the
 * compressed basis' list, BlockGS::act; about half the cells are land at 2 degrees): d of the
 * other cells stays 0 (gs_compute zeroes it whenever the list changes). */
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) k_spmv_dyn(SubLay X, const double* __restrict__ val,
                                                  const double* __restrict__ z,
                                                  const double* __restrict__ r,
                                                  const uint8_t* __restrict__ knP,
                                                  double* __restrict__ d, int64_t nloc, int nblk, int64_t ps,
                                                  const double* __restrict__ hv, int nhb, int hs, int hn,
                                                  const int* __restrict__ alist, int64_t nown,
                                                  const double* __restrict__ vb)
{
    __shared__ double red[4][2][64];
    __shared__ int64_t us[64];
    __shared__ int oks[64];
    const int ntot = nblk + nhb;
    const int per = (ntot + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= ntot) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t row = (int64_t)X.l * X.nx;             /* cells of one latitude row */
    const int64_t e0 = (int64_t)HALO * row;              /* ext cell of owned cell 0 */
    /* u: the cell relative to owned cell 0 (the halo rows at -row .. -1 and nloc .. nloc + row - 1) */
    const bool halo = tile >= nblk;
    int64_t h, u;
    bool act;
    if (!halo) {
        h = (int64_t)tile * 64 + c;
        act = h < nown;
        u = !act ? 0 : (alist ? (int64_t)alist[h] : h);
    } else {
        h = (int64_t)(tile - nblk) * 64 + c;             /* halo index: south row, then north */
        const bool south = h < row;
        act = h < 2 * row && (south ? hs : hn);
        u = south ? h - row : nloc + h - row;
    }
    if (g == 0) {
        us[c] = u;
        oks[c] = act ? 1 : 0;
    }
    double acc[2] = {0.0, 0.0};
    if (act) {
        const int64_t q = u + row;                       /* >= 0 */
        const int il = (int)(q % X.nx), k = (int)((q / X.nx) % X.l);
        const int j = X.jb0 - 1 + (int)(q / row);
        int nc[3][9];
        nb_cells(X, il, j, k, nc);
        /* the wave's two rows: g0 {U, -} g1 {U, V} g2 {V, W} g3 {W, P} */
        const int64_t cell = e0 + u;
        const int v0 = g == 0 ? 0 : g - 1;
        const bool on[2] = {!knP[cell + ps * v0], g > 0 && !knP[cell + ps * (v0 + 1)]};
        /* vb: the active cells' coefficients blocked per tile (h = tile 64 + c) */
        const double* vp = halo ? hv + h : (vb ? vb + (int64_t)tile * 4096 + c : val + u);
        const int64_t vs = halo ? 2 * row : (vb ? 64 : nloc);
        if (g == 0) dyn_partial<0, 16>(vp, z, vs, nc, on, ps, acc);
        else if (g == 1) dyn_partial<16, 32>(vp, z, vs, nc, on, ps, acc);
        else if (g == 2) dyn_partial<32, 48>(vp, z, vs, nc, on, ps, acc);
        else dyn_partial<48, 64>(vp, z, vs, nc, on, ps, acc);
    }
    red[g][0][c] = acc[0];
    red[g][1][c] = acc[1];
    __syncthreads();
    /* rows of the waves: g0 {U} g1 {U,V} g2 {V,W} g3 {W,P}; thread = (row, cell), the
     * cell fastest (planar stores) */
    const int R = threadIdx.x >> 6, cc = threadIdx.x & 63;
    if (!oks[cc]) return;
    const double sum = R == 0 ? red[0][0][cc] + red[1][0][cc]
                     : R == 1 ? red[1][1][cc] + red[2][0][cc]
                     : R == 2 ? red[2][1][cc] + red[3][0][cc]
                              : red[3][1][cc];
    const int64_t cell = e0 + us[cc], e = cell + ps * R;
    d[e] = knP[e] ? 0.0 : r[e] - sum;
}

int spmv_dyn_defect(iemic_ctx* c, const double* z, const double* r, const uint8_t* knP, double* d, bool halo)
{
    const BlockGS& gs = c->gs;
    const bool al = gs.act.p && gs.nact > 0;
    const int64_t nown = al ? gs.nact : c->nloc;
    const int nblk = (int)((nown + 63) / 64);
    const int64_t row = (int64_t)c->l * c->nx;
    const bool hv = halo && gs.dvh.p;
    const int nhb = hv ? (int)((2 * row + 63) / 64) : 0;
    const unsigned grid = 8u * (unsigned)((nblk + nhb + 7) / 8);
    hipLaunchKernelGGL(k_spmv_dyn, dim3(grid), dim3(256), 0, c->stream, sub_lay(c), gs.vp, z, r, knP, d,
                       c->nloc, nblk, (int64_t)c->next, hv ? gs.dvh.p : nullptr, nhb,
                       hv && c->nb[2] >= 0 ? 1 : 0, hv && c->nb[3] >= 0 ? 1 : 0, al ? gs.act.p : nullptr, nown,
                       al && gs.dvb.p ? gs.dvb.p : nullptr);
    return 0;
}

/* ---- reductions / BLAS-1 ------------------------------------------------------------ */
__global__ void k_zero(double* __restrict__ p, int64_t n)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        p[q] = 0.0;
}


__device__ __forceinline__ double block_sum(double v, double* sm)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sm[wid] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += sm[w];
    return t;
}

/* partial[i * gridDim.x + blk] = sum over the block's range of V_i . w, i < nvec;
 * with extra != null, row i == nvec is extra . w (or extra . extra_w) in the same launch */
__global__ void __launch_bounds__(256) k_mdot(const double* __restrict__ V, int64_t ldv, int nvec,
                                              const double* __restrict__ w, int64_t N,
                                              double* __restrict__ partial,
                                              const double* __restrict__ extra = nullptr,
                                              const double* __restrict__ extra_w = nullptr)
{
    __shared__ double sm[8];
    const int i = blockIdx.y;
    if (i > nvec || (i == nvec && !extra)) return;
    const double* vi = i == nvec ? extra : V + (int64_t)i * ldv;
    const double* wi = (i == nvec && extra_w) ? extra_w : w;
    double s = 0.0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        s += vi[q] * wi[q];
    double t = block_sum(s, sm);
    if (threadIdx.x == 0) partial[(int64_t)i * gridDim.x + blockIdx.x] = t;
}
/* out[i] = sum_b partial[i*nb + b]  (fixed order: deterministic) */
__global__ void k_mdot_final(const double* __restrict__ partial, int nb, int nvec,
                             double* __restrict__ out)
{
    __shared__ double sm[8];
    const int i = blockIdx.x;
    if (i >= nvec) return;
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) s += partial[(int64_t)i * nb + b];
    double t = block_sum(s, sm);
    if (threadIdx.x == 0) out[i] = t;
}
/* w -= sum_i h_i V_i */
__global__ void __launch_bounds__(256) k_mupdate(const double* __restrict__ V, int64_t ldv, int nvec,
                                                 const double* __restrict__ h,
                                                 double* __restrict__ w, int64_t N)
{
    __shared__ double hs[1024];
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) hs[i] = h[i];
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x) {
        double acc = w[q];
        for (int i = 0; i < nvec; i++) acc -= hs[i] * V[(int64_t)i * ldv + q];
        w[q] = acc;
    }
}
/* w -= sum_i h_i V_i and partial[blk] = block's sum of the new w^2 (grid = RED_BLOCKS) */
__global__ void __launch_bounds__(256) k_mupdate_norm(const double* __restrict__ V, int64_t ldv,
                                                      int nvec, const double* __restrict__ h,
                                                      double* __restrict__ w, int64_t N,
                                                      double* __restrict__ partial)
{
    __shared__ double hs[1024];
    __shared__ double sm[8];
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) hs[i] = h[i];
    __syncthreads();
    double ss = 0.0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x) {
        double acc = w[q];
        int i = 0;
        for (; i + 4 <= nvec; i += 4) {
            const double* v = V + (int64_t)i * ldv + q;
            acc -= hs[i] * v[0];
            acc -= hs[i + 1] * v[ldv];
            acc -= hs[i + 2] * v[2 * ldv];
            acc -= hs[i + 3] * v[3 * ldv];
        }
        for (; i < nvec; i++) acc -= hs[i] * V[(int64_t)i * ldv + q];
        w[q] = acc;
        ss += acc * acc;
    }
    const double t = block_sum(ss, sm);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

/* sum NV values over the block; result valid in thread 0 (sm: NV*(blockDim/64) doubles) */
template <int NV>
__device__ __forceinline__ void block_sum_n(double* v, double* sm)
{
#pragma unroll
    for (int q = 0; q < NV; q++)
        for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_down(v[q], o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) sm[q * nw + wid] = v[q];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) {
            double t = 0.0;
            for (int w = 0; w < nw; w++) t += sm[q * nw + w];
            v[q] = t;
        }
}

/* DCGS2 dot pass: rows 2i, 2i+1 = Q_i.u, Q_i.w (i < nvec); rows 2nvec..2nvec+2 = u.u, u.w,
 * w.w.  Block (bx, by), by < ceil(nvec / DG), handles DG basis vectors against u and w over
 * chunk bx; by == nq the three self products.  The group index varies fastest in the block
 * order, so the groups of one chunk run together on one XCD and u, w come from its L2
 * after the first;
 * every lane reads two consecutive elements (16-byte loads; N even, 16-byte aligned).
 * partial[row * nbx + bx].  (scripts/orth_probe.hip: DG = 4 in this order 5.5 TB/s at 89
 * vectors against 4.5 for DG = 8 with the group index slowest.) */
constexpr int DCGS_DG = 4;
static_assert(RED_BLOCKS % 8 == 0, "k_dcgs_dot deals chunks to the 8 XCDs");
__global__ void __launch_bounds__(256) k_dcgs_dot(const double* __restrict__ V, int64_t ldv, int nvec,
                                                  const double* __restrict__ u,
                                                  const double* __restrict__ w, int64_t N,
                                                  double* __restrict__ partial, int nbx)
{
    constexpr int DG = DCGS_DG;
    __shared__ double sm[4 * 2 * DG];
    const int nq = (nvec + DG - 1) / DG;
    /* XCD-aware order (workgroups are dealt to the 8 XCDs round robin): the nq + 1 groups of
     * chunk bx run on XCD bx % 8, launched together, so u and w of the chunk are read from
     * HBM once and from that XCD's L2 by the other groups (nbx % 8 == 0) */
    const int G = nq + 1, sb = blockIdx.x / (8 * G), rem = blockIdx.x % (8 * G);
    const int by = rem / 8, bx = sb * 8 + rem % 8;
    const int64_t N2 = N / 2;
    const int64_t stride = (int64_t)nbx * blockDim.x;
    const int64_t e0 = (int64_t)bx * blockDim.x + threadIdx.x;
    const double2* u2 = reinterpret_cast<const double2*>(u);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    if (by < nq) {
        const int i0 = DG * by;
        const int nv = min(DG, nvec - i0);
        double acc[2 * DG];
#pragma unroll
        for (int t = 0; t < 2 * DG; t++) acc[t] = 0.0;
        const double* q0 = V + (int64_t)i0 * ldv;
        for (int64_t e = e0; e < N2; e += stride) {
            const double2 ue = u2[e], we = w2[e];
#pragma unroll
            for (int t = 0; t < DG; t++) {
                if (t < nv) {
                    const double2 qe = reinterpret_cast<const double2*>(q0 + (int64_t)t * ldv)[e];
                    acc[2 * t] += qe.x * ue.x + qe.y * ue.y;
                    acc[2 * t + 1] += qe.x * we.x + qe.y * we.y;
                }
            }
        }
        block_sum_n<2 * DG>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 2 * nv; t++) partial[(int64_t)(2 * i0 + t) * nbx + bx] = acc[t];
    } else {
        double acc[3] = {0, 0, 0};
        for (int64_t e = e0; e < N2; e += stride) {
            const double2 ue = u2[e], we = w2[e];
            acc[0] += ue.x * ue.x + ue.y * ue.y;
            acc[1] += ue.x * we.x + ue.y * we.y;
            acc[2] += we.x * we.x + we.y * we.y;
        }
        block_sum_n<3>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 3; t++) partial[(int64_t)(2 * nvec + t) * nbx + bx] = acc[t];
    }
}

/* DCGS2 dot pass, one read of everything: a workgroup holds its chunk of u and w in
 * registers (DOT1_E 16-byte elements per lane) and streams every basis vector past them once;
 * each vector's two sums are reduced across the wave and accumulated per wave in LDS
 * (4 x (2 nvec + 3) doubles, dynamic).  Chunks are dealt to the nbx <= RED_BLOCKS workgroups
 * round robin.  partial[row * nbx + bx] as k_dcgs_dot. */
/* 16-byte non-temporal load: the DCGS2 passes stream the basis (up to 1 GB at 2 degrees,
 * past the Infinity Cache) once per pass, and keeping it out of the caches leaves them to
 * u, w and the partial sums (dot pass 84.2 -> 73.7 us, update 84.0 -> 81.7 us,
 * scripts/ab/dcgs_nt.sh) */
__device__ __forceinline__ double2 ldnt2(const double2* p)
{
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
constexpr int DOT1_E = 4;
__device__ __forceinline__ double wave_sum(double v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__global__ void __launch_bounds__(256) k_dcgs_dot1(const double* __restrict__ V, int64_t ldv, int nvec,
                                                   const double* __restrict__ u,
                                                   const double* __restrict__ w, int64_t N,
                                                   double* __restrict__ partial, int nbx)
{
    constexpr int E = DOT1_E;
    extern __shared__ double acc_s[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int R = 2 * nvec + 3;
    double* my = acc_s + wid * R;
    for (int t = lane; t < R; t += 64) my[t] = 0.0;
    __syncthreads();
    const int64_t N2 = N / 2, CH = 256 * E;
    const int64_t nch = (N2 + CH - 1) / CH;
    const double2* u2 = reinterpret_cast<const double2*>(u);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double suu = 0.0, suw = 0.0, sww = 0.0;
    for (int64_t ch = blockIdx.x; ch < nch; ch += nbx) {
        const int64_t e0 = ch * CH + threadIdx.x;
        double2 ue[E], we[E];
#pragma unroll
        for (int k = 0; k < E; k++) {
            const int64_t e = e0 + (int64_t)k * 256;
            ue[k] = e < N2 ? u2[e] : make_double2(0.0, 0.0);
            we[k] = e < N2 ? w2[e] : make_double2(0.0, 0.0);
            suu += ue[k].x * ue[k].x + ue[k].y * ue[k].y;
            suw += ue[k].x * we[k].x + ue[k].y * we[k].y;
            sww += we[k].x * we[k].x + we[k].y * we[k].y;
        }
        /* out-of-range lanes read element 0 of the vector (their u, w are zero) */
        int64_t ex[E];
#pragma unroll
        for (int k = 0; k < E; k++) {
            const int64_t e = e0 + (int64_t)k * 256;
            ex[k] = e < N2 ? e : 0;
        }
        double2 qn[E];
        if (nvec > 0) {
#pragma unroll
            for (int k = 0; k < E; k++) qn[k] = ldnt2(reinterpret_cast<const double2*>(V) + ex[k]);
        }
        for (int i = 0; i < nvec; i++) {
            double2 q[E];
#pragma unroll
            for (int k = 0; k < E; k++) q[k] = qn[k];
            if (i + 1 < nvec) {
                const double2* qv = reinterpret_cast<const double2*>(V + (int64_t)(i + 1) * ldv);
#pragma unroll
                for (int k = 0; k < E; k++) qn[k] = ldnt2(qv + ex[k]);
            }
            double a = 0.0, b = 0.0;
#pragma unroll
            for (int k = 0; k < E; k++) {
                a += q[k].x * ue[k].x + q[k].y * ue[k].y;
                b += q[k].x * we[k].x + q[k].y * we[k].y;
            }
            a = wave_sum(a);
            b = wave_sum(b);
            if (lane == 0) {
                my[2 * i] += a;
                my[2 * i + 1] += b;
            }
        }
    }
    suu = wave_sum(suu);
    suw = wave_sum(suw);
    sww = wave_sum(sww);
    if (lane == 0) {
        my[2 * nvec] += suu;
        my[2 * nvec + 1] += suw;
        my[2 * nvec + 2] += sww;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < R; t += blockDim.x)
        partial[(int64_t)t * nbx + blockIdx.x] = acc_s[t] + acc_s[R + t] + acc_s[2 * R + t] + acc_s[3 * R + t];
}

/* DCGS2 coefficients on the device (no host round trip before the update pass): from the
 * summed dot rows hb = [Q^T u, Q^T w interleaved | u.u, u.w, w.w], beta = sqrt(u.u - |a|^2),
 * h_jj = (u.w - a.b) / beta, gamma = h_jj / beta; coef = [a | b - gamma a], coef[DCGS_SCAL..] =
 * 1/beta, gamma; beta, h_jj appended to hb (rows 2nv+3, 2nv+4) for the host's Hessenberg
 * column.  A breakdown (beta = 0) gives zero scales; the host stops on it. */
__global__ void __launch_bounds__(256) k_dcgs_coef(double* __restrict__ hb, int nv, double* __restrict__ coef,
                                                   double* __restrict__ hrows)
{
    __shared__ double sm[2 * 4];
    __shared__ double tot[2];
    double v[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
        const double a = hb[2 * i], b = hb[2 * i + 1];
        v[0] += a * a;
        v[1] += a * b;
    }
    block_sum_n<2>(v, sm);
    if (threadIdx.x == 0) {
        tot[0] = v[0];
        tot[1] = v[1];
    }
    __syncthreads();
    const double beta2 = hb[2 * nv] - tot[0];
    const double bt = beta2 > 0.0 ? sqrt(beta2) : 0.0;
    const bool ok = bt > 0.0 && bt <= 1.79e308;
    const double hjj = ok ? (hb[2 * nv + 1] - tot[1]) / bt : 0.0;
    const double gamma = ok ? hjj / bt : 0.0;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
        const double a = hb[2 * i], b = hb[2 * i + 1];
        coef[i] = a;
        coef[nv + i] = b - a * gamma;
    }
    if (threadIdx.x == 0) {
        coef[DCGS_SCAL] = ok ? 1.0 / bt : 0.0;
        coef[DCGS_SCAL + 1] = gamma;
        hb[2 * nv + 3] = bt;
        hb[2 * nv + 4] = hjj;
    }
    /* the rows for the host's Hessenberg column, straight into its pinned (coherent) slot:
     * no device-to-host copy launch per Arnoldi step */
    if (hrows) {
        __syncthreads();
        for (int i = threadIdx.x; i < 2 * nv + 5; i += blockDim.x) hrows[i] = hb[i];
    }
}

/* DCGS2 update pass, one read of Q:  q_j = (u - Q a) * inv_beta,
 * w = (w - Q c - gamma * u) * inv_beta  (coef = [a (nvec) | c (nvec)], inv_beta and gamma at
 * coef[DCGS_SCAL..]); u is overwritten by q_j.  Scaling the next candidate w by the same
 * 1/beta (lagged normalisation) keeps every candidate at the scale of a normalised Arnoldi
 * vector, so its norm never compounds the earlier subdiagonals (no overflow / false breakdown
 * over long cycles). */
/* rrP (the compressed basis with the block GS): the new candidate w -- the next step's
 * preconditioner input -- also goes straight into the block GS's planar right-hand side
 * (rows 2e, 2e + 1 of w are unknowns R, R + 1 of active cell act[2e / 6]), so the apply
 * skips its entry kernel k_gs_rr_c */
__global__ void __launch_bounds__(256) k_dcgs_update(const double* __restrict__ V, int64_t ldv,
                                                     int nvec, const double* __restrict__ coef,
                                                     double* __restrict__ u, double* __restrict__ w,
                                                     int64_t N, const int* __restrict__ act = nullptr,
                                                     int64_t own0 = 0, int64_t ps = 0,
                                                     double* __restrict__ rrP = nullptr)
{
    /* two consecutive elements per lane (16-byte loads; N even), four basis vectors per step */
    constexpr int UN = 4;
    __shared__ double cs[2 * 1024];
    for (int i = threadIdx.x; i < 2 * nvec; i += blockDim.x) cs[i] = coef[i];
    __syncthreads();
    const double inv_beta = coef[DCGS_SCAL], gamma = coef[DCGS_SCAL + 1];
    const double* a = cs;
    const double* cc = cs + nvec;
    const int64_t N2 = N / 2;
    double2* u2 = reinterpret_cast<double2*>(u);
    double2* w2 = reinterpret_cast<double2*>(w);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N2;
         e += (int64_t)gridDim.x * blockDim.x) {
        double sux = 0.0, suy = 0.0, swx = 0.0, swy = 0.0;
        int i = 0;
        for (; i + UN <= nvec; i += UN) {
            double2 q[UN];
#pragma unroll
            for (int k = 0; k < UN; k++) q[k] = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)(i + k) * ldv) + e);
#pragma unroll
            for (int k = 0; k < UN; k++) {
                sux += a[i + k] * q[k].x;
                suy += a[i + k] * q[k].y;
                swx += cc[i + k] * q[k].x;
                swy += cc[i + k] * q[k].y;
            }
        }
        for (; i < nvec; i++) {
            const double2 q = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)i * ldv) + e);
            sux += a[i] * q.x;
            suy += a[i] * q.y;
            swx += cc[i] * q.x;
            swy += cc[i] * q.y;
        }
        const double2 ue = u2[e], we = w2[e];
        u2[e] = make_double2((ue.x - sux) * inv_beta, (ue.y - suy) * inv_beta);
        const double2 wn = make_double2((we.x - swx - gamma * ue.x) * inv_beta, (we.y - swy - gamma * ue.y) * inv_beta);
        w2[e] = wn;
        if (rrP) {
            const int64_t a = e / 3, R = 2 * e - 6 * a, cell = own0 + act[a];
            rrP[cell + R * ps] = wn.x;
            rrP[cell + (R + 1) * ps] = wn.y;
        }
    }
}

/* x += sum_i y_i Z_i */
__global__ void __launch_bounds__(256) k_mupdate_add(const double* __restrict__ Z, int64_t ldz, int nvec,
                                                     const double* __restrict__ y,
                                                     double* __restrict__ x, int64_t N)
{
    __shared__ double ys[1024];
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) ys[i] = y[i];
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x) {
        double acc = x[q];
        for (int i = 0; i < nvec; i++) acc += ys[i] * Z[(int64_t)i * ldz + q];
        x[q] = acc;
    }
}
__global__ void k_scale_copy(const double* __restrict__ a, double s, double* __restrict__ b, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        b[q] = s * a[q];
}
__global__ void k_axpby(double a, const double* __restrict__ x, double b, const double* __restrict__ y,
                        double* __restrict__ out, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        out[q] = a * x[q] + b * y[q];
}

static inline unsigned grid_for(int64_t N)
{
    int64_t b = (N + 255) / 256;
    return (unsigned)std::min<int64_t>(b, 2048);
}

static int spmv_intcond(iemic_ctx* c, const double* x, double* yr);
/* the SpMV kernel(s) alone: x's halo rows must be current */
int spmv_kernel(iemic_ctx* c, const double* x, double* y)
{
    if (!c->jac_valid) {
        set_error("spmv: no Jacobian assembled");
        return IEMIC_ESTATE;
    }
    hipStream_t s = c->stream;
    if (c->nloc >= INT32_MAX) {
        set_error("spmv: more than 2^31 cells per rank");
        return IEMIC_EINVAL;
    }
    const int tpr = (c->nx + SP7_T - 1) / SP7_T;
    const int ntile = (int)(c->nloc / c->nx) * tpr;
    const unsigned grid = 8u * (unsigned)((ntile + 7) / 8);
    hipLaunchKernelGGL(k_spmv7, dim3(grid), dim3(256), 0, s, sub_lay(c), c->d_val.p, x, y, (int)c->nloc, ntile,
                       tpr);
    return spmv_intcond(c, x, c->rowintcon >= 0 ? y + c->rowintcon : nullptr);
}

/* the dense integral-condition row: *yr = intSign * coeff . x (summed over the ranks; yr its
 * entry of this rank's output, if it owns it) */
static int spmv_intcond(iemic_ctx* c, const double* x, double* yr)
{
    hipStream_t s = c->stream;
    if (c->su.rowintcon_ref >= 0) {
        /* dense intcond row: y[rowintcon] = intSign * coeff . x (summed over the ranks) */
        const int64_t o = NUN * c->own0;
        hipLaunchKernelGGL(k_mdot, dim3(RED_BLOCKS, 1), dim3(256), 0, s, c->d_intc.p + o, (int64_t)0, 1,
                           x + o, c->nlrows, c->d_red.p);
        hipLaunchKernelGGL(k_mdot_final, dim3(1), dim3(256), 0, s, c->d_red.p, RED_BLOCKS, 1,
                           c->d_red.p + RED_BLOCKS);
        int rc = allreduce_sum(c, c->d_red.p + RED_BLOCKS, 1);
        if (rc) return rc;
        if (c->rowintcon >= 0)
            hipLaunchKernelGGL(k_scale_copy, dim3(1), dim3(1), 0, s, c->d_red.p + RED_BLOCKS,
                               (double)c->cfg.int_sign, yr, (int64_t)1);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

/* ev0 / ev1 (optional): the kernel's own start and end (hipExtLaunchKernelGGL records them
 * from the dispatch itself, so FGMRES times the SpMV kernel alone, as the trace does) */
int spmv_kernel_c(iemic_ctx* c, const double* x, double* yc, hipEvent_t ev0, hipEvent_t ev1)
{
    const BlockGS& gs = c->gs;
    if (!c->jac_valid || !gs.cmap.p || !gs.spc.p || !gs.atl.p || gs.coef_stale) {
        set_error("spmv: no Jacobian, no active-cell map or stale packed coefficients");
        return IEMIC_ESTATE;
    }
    hipStream_t s = c->stream;
    const int tpr = (c->nx + SP7_T - 1) / SP7_T;
    const unsigned grid = 8u * (unsigned)((gs.natile + 7) / 8);
    if (gs.natile > 0)
        hipExtLaunchKernelGGL(k_spmv7c, dim3(grid), dim3(256), 0, s, ev0, ev1, 0, sub_lay(c), (const double*)gs.spc.p,
                              x, yc, (const int4*)gs.atl.p, gs.natile, tpr);
    double* yr = nullptr;
    if (c->rowintcon >= 0) {
        if (c->gs.ric < 0) {
            set_error("spmv: the integral-condition row lies in an inactive cell");
            return IEMIC_EINVAL;
        }
        yr = yc + c->gs.ric;
    }
    return spmv_intcond(c, x, yr);
}

int spmv(iemic_ctx* c, double* x, double* y, hipStream_t)
{
    int rc = halo_exchange(c, x, 1);
    if (rc) return rc;
    return spmv_kernel(c, x, y);
}

/* dot products of nvec vectors V_i (stride ldv) with w, and (ea != null) ea . eb as
 * out[nvec], in one launch pair and one host synchronisation */
/* V, w, ea, eb point at the first owned row; length nlrows; sums over the ranks */
static int mdot_host(iemic_ctx* c, const double* V, int64_t ldv, int nvec, const double* w,
                     double* out, const double* ea = nullptr, const double* eb = nullptr)
{
    const int64_t N = c->nlrows;
    const int nout = nvec + (ea ? 1 : 0);
    hipLaunchKernelGGL(k_mdot, dim3(RED_BLOCKS, nout), dim3(256), 0, c->stream, V, ldv, nvec, w, N,
                       c->d_part.p, ea, eb);
    hipLaunchKernelGGL(k_mdot_final, dim3(nout), dim3(256), 0, c->stream, c->d_part.p, RED_BLOCKS,
                       nout, c->d_hbuf.p);
    int rc = allreduce_sum(c, c->d_hbuf.p, nout);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(c->h_red, c->d_hbuf.p, sizeof(double) * nout, hipMemcpyDeviceToHost,
                          c->stream));
    DEV_SYNC(c);
    for (int i = 0; i < nout; i++) out[i] = c->h_red[i];
    return 0;
}

/* a . b over the owned rows of two ext vectors, summed over the ranks (error code) */
int dot_owned(iemic_ctx* c, const double* a, const double* b, double* out)
{
    const int64_t o = NUN * c->own0;
    return mdot_host(c, a + o, 0, 1, b + o, out);
}

/* a . b over the owned rows of two ext vectors, summed over the ranks */
double dot(iemic_ctx* c, const double* a, const double* b, int64_t)
{
    const int64_t o = NUN * c->own0;
    double r = 0.0;
    if (mdot_host(c, a + o, 0, 1, b + o, &r)) return NAN;
    return r;
}

/* One Gram-Schmidt pass over the nvec basis vectors: h = V^T w, ww0 = w.w (before),
 * w -= V h, ww1 = w.w (after).  The coefficients stay on the device between the two
 * launches; one device-to-host copy + synchronisation returns h, ww0, ww1. */
static int orth_pass(iemic_ctx* c, const double* V, int64_t ldv, int nvec, double* w, double* h,
                     double* ww0, double* ww1)
{
    const int64_t N = c->nlrows;
    hipLaunchKernelGGL(k_mdot, dim3(RED_BLOCKS, nvec + 1), dim3(256), 0, c->stream, V, ldv, nvec,
                       w, N, c->d_part.p, (const double*)w);
    hipLaunchKernelGGL(k_mdot_final, dim3(nvec + 1), dim3(256), 0, c->stream, c->d_part.p,
                       RED_BLOCKS, nvec + 1, c->d_hbuf.p);
    int rc = allreduce_sum(c, c->d_hbuf.p, nvec + 1);   /* coefficients summed before use */
    if (rc) return rc;
    hipLaunchKernelGGL(k_mupdate_norm, dim3(RED_BLOCKS), dim3(256), 0, c->stream, V, ldv, nvec,
                       c->d_hbuf.p, w, N, c->d_part.p);
    hipLaunchKernelGGL(k_mdot_final, dim3(1), dim3(256), 0, c->stream, c->d_part.p, RED_BLOCKS, 1,
                       c->d_hbuf.p + nvec + 1);
    if ((rc = allreduce_sum(c, c->d_hbuf.p + nvec + 1, 1))) return rc;
    HIP_OK(hipMemcpyAsync(c->h_red, c->d_hbuf.p, sizeof(double) * (nvec + 2), hipMemcpyDeviceToHost,
                          c->stream));
    DEV_SYNC(c);
    for (int i = 0; i < nvec; i++) h[i] = c->h_red[i];
    *ww0 = c->h_red[nvec];
    *ww1 = c->h_red[nvec + 1];
    return 0;
}

/* the Krylov work space: Z (m x N) and w, r always; the full-length basis V ((m+1) x N) unless
 * the basis is compressed, then Vc ((m+1) x nc) and the full-length t, b' */
static int ensure_krylov(iemic_ctx* c, int m, int64_t nc = 0)
{
    Krylov& k = c->kr;
    const int64_t N = c->nerows;
    int rc = 0;
    if (k.m < m || !k.Z.p) {
        k.zclean = 0;
        k.V.free();                  /* sized by m: reallocated below when needed */
        rc |= k.Z.alloc((size_t)m * N);
        rc |= k.w.alloc(N);
        rc |= k.r.alloc(N);
        if (rc) {
            set_error("fgmres: out of device memory for the Krylov basis");
            return IEMIC_ENOMEM;
        }
        k.m = m;
    }
    if (!nc && !k.V.p) {
        if (k.V.alloc((size_t)(k.m + 1) * N)) {
            set_error("fgmres: out of device memory for the Krylov basis");
            return IEMIC_ENOMEM;
        }
    }
    if (nc && (k.mc < m || k.nc < nc || !k.Vc.p)) {
        rc |= k.Vc.alloc((size_t)(m + 1) * nc);
        if (!k.t.p) rc |= k.t.alloc(N) | k.bp.alloc(N);
        if (rc) {
            set_error("fgmres: out of device memory for the Krylov basis");
            return IEMIC_ENOMEM;
        }
        k.mc = m;
        k.nc = nc;
    }
    return 0;
}

/* the compressed Arnoldi basis: rows of the active cells act[] (6 per cell), in order */
__global__ void k_cgather(const double* __restrict__ full, const int* __restrict__ act, int64_t nc,
                          int64_t own0, double s, double* __restrict__ cmp)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nc;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t cl = q / NUN;
        cmp[q] = s * full[NUN * (own0 + act[cl]) + (q - NUN * cl)];
    }
}
/* t = v on the identity rows (known), 0 elsewhere (owned rows) */
__global__ void k_known_part(const double* __restrict__ v, const uint8_t* __restrict__ known, int64_t n0,
                             int64_t nl, double* __restrict__ t)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nl;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = n0 + q;
        t[r] = known[r] ? v[r] : 0.0;
    }
}

/* coefficients -> device through the pinned staging area (the previous use of the area
 * has completed: every caller synchronised the stream since) */
static int upload_coeffs(iemic_ctx* c, const double* h, int n)
{
    if (n > RED_ROWS) {
        set_error("upload_coeffs: too many coefficients");
        return IEMIC_EINVAL;
    }
    double* st = c->h_red + RED_ROWS;
    for (int i = 0; i < n; i++) st[i] = h[i];
    HIP_OK(hipMemcpyAsync(c->d_hbuf.p + RED_ROWS, st, sizeof(double) * n,
                          hipMemcpyHostToDevice, c->stream));
    return 0;
}

static double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

/* sqrt of a squared norm that rounding may have driven below zero; NaN stays NaN */
static inline double sqrt0(double v) { return v > 0.0 ? std::sqrt(v) : (v == v ? 0.0 : v); }

/* a NaN/Inf reaching the Hessenberg column would pass for a breakdown (res = 0): stop loudly */
static int nonfinite()
{
    set_error("FGMRES: non-finite value in the Krylov basis (operator or preconditioner output)");
    return IEMIC_ERANGE;
}

int prec_safeguard(iemic_ctx* c);

/* a restart cycle of at least STAG_MIN steps that cut the true residual by less than
 * 1 / STAG_RATIO counts as stagnation (a converging cycle at the 2-degree bench state cuts it
 * by ~1e-3, one at the 1-degree continuation tolerance by ~30) */
constexpr double STAG_RATIO = 0.25;
constexpr int STAG_MIN = 20;

int fgmres(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt, iemic_solve_info* info)
{
    /* vectors are ext-layout (stride NE); kernels touch the owned rows [o, o + NL) */
    const int m = std::max(1, std::min(opt->krylov_dim, MAX_KRYLOV));
    const int64_t NE = c->nerows, o = NUN * c->own0, NL = c->nlrows;
    /* DCGS2 with the block GS: the Arnoldi basis on the active cells only.  Identity rows of J
     * (all rows of a land cell, some of an ocean cell) are identity rows of the preconditioner
     * too, so with a right-hand side that is zero on them every Krylov vector is exactly zero
     * there: the basis skips the land cells (48 % of the rows at 2 degrees), the block GS
     * reads it without the identity-column couplings and the SpMV writes only the active
     * cells.  A right-hand side with identity-row entries is first reduced: x_k = b_k,
     * b' = b - J t (t = b on the identity rows), zero on them. */
    const BlockGS& gs = c->gs;
    int rc = opt->prec > 0 ? gs_refresh(c) : 0;
    if (rc) return rc;
    const bool cmp = opt->orth == 0 && opt->prec == 2 && gs.ready && gs.kind == 2 && gs.nact > 0 && gs.cmap.p &&
                     gs.cmp_ok && gs.spc.p && gs.atl.p;
    const int64_t NC = cmp ? NUN * gs.nact : 0;
    rc = ensure_krylov(c, m, NC);
    if (rc) return rc;
    /* the staged applies (gs_apply_c after an update pass) leave the identity rows of the
     * preconditioned vectors Z alone: zero them once per set-up (kr.zclean), the other
     * solvers may have left values there */
    if (cmp && !c->kr.zclean) {
        if ((rc = dev_zero(c, c->kr.Z.p, (int64_t)m * NE))) return rc;
        c->kr.zclean = 1;
    } else if (!cmp) {
        c->kr.zclean = 0;
    }
    iemic_solve_info inf{};
    auto T0 = std::chrono::steady_clock::now();
    double* V = cmp ? nullptr : c->kr.V.p;
    double* Vc = cmp ? c->kr.Vc.p : nullptr;
    double* Z = c->kr.Z.p;
    double* w = c->kr.w.p;
    double* r = c->kr.r.p;
    const unsigned G = grid_for(NL);
    const unsigned GC = grid_for(NC);
    std::vector<double> H((size_t)(m + 1) * m), cs(m), sn(m), g(m + 1), h(m + 1), h2(m + 1), y(m);
    std::vector<double> zs(m + 1, 1.0);   /* DCGS2: scale of the stored z_j (1 for DGKS) */
    if (2 * m + 5 > RED_ROWS) {
        set_error("fgmres: Krylov dimension too large");
        return IEMIC_EINVAL;
    }
    int inf_reorth = 0;
    /* prec / SpMV timing events (two sets: the DCGS2 loop runs one iteration ahead) and the
     * DCGS2 row-copy events */
    struct Events {
        hipEvent_t e[8] = {};
        ~Events() { for (auto& x : e) if (x) (void)hipEventDestroy(x); }
    } evs;
    hipEvent_t* ev = evs.e;
    hipEvent_t* evr = evs.e + 6;
    for (int q = 0; q < 6; q++) HIP_OK(hipEventCreate(&ev[q]));
    for (int q = 6; q < 8; q++) HIP_OK(hipEventCreateWithFlags(&evs.e[q], hipEventDisableTiming));

    if ((rc = dev_zero(c, x, NE))) return rc;
    double bnorm = sqrt0(dot(c, b, b, 0));
    if (!std::isfinite(bnorm)) return nonfinite();
    if (!(bnorm > 0)) {
        inf.converged = 1;
        if (info) *info = inf;
        return 0;
    }
    const double* b_orig = b;
    bool known_rhs = false;
    if (cmp) {
        double* t = c->kr.t.p;
        hipLaunchKernelGGL(k_known_part, dim3(G), dim3(256), 0, c->stream, b, gs.known.p, o, NL, t);
        if (dot(c, t, t, 0) > 0.0) {
            known_rhs = true;
            if ((rc = spmv(c, t, w, c->stream))) return rc;
            hipLaunchKernelGGL(k_axpby, dim3(G), dim3(256), 0, c->stream, 1.0, b + o, -1.0, w + o,
                               c->kr.bp.p + o, NL);
            b = c->kr.bp.p;
        }
    }
    /* r = b (x0 = 0) */
    HIP_OK(hipMemcpyAsync(r, b, sizeof(double) * NE, hipMemcpyDeviceToDevice, c->stream));
    double beta = known_rhs ? sqrt0(dot(c, b, b, 0)) : bnorm, res = beta / bnorm, res_c0 = res;
    int it = 0;
    /* the safeguard's switch lasts for this solve only */
    struct Restore {
        iemic_ctx* c;
        int mr;
        ~Restore() { c->gs.dyn_mr = mr; }
    } restore{c, c->gs.dyn_mr};
    /* beta = 0: a right-hand side on the land rows only, solved by x = t below */
    for (int cycle = 0; beta > 0.0 && cycle <= opt->max_restarts; cycle++) {
        const int it_c0 = it;
        if (cmp)
            hipLaunchKernelGGL(k_cgather, dim3(GC), dim3(256), 0, c->stream, r, gs.act.p, NC, c->own0, 1.0 / beta, Vc);
        else
            hipLaunchKernelGGL(k_scale_copy, dim3(G), dim3(256), 0, c->stream, r + o, 1.0 / beta, V + o, NL);
        std::fill(g.begin(), g.end(), 0.0);
        g[0] = beta;
        int j = 0;
        if (opt->orth == 1) {
            for (; j < m; j++) {
                double* vj = V + (int64_t)j * NE;
                double* zj = Z + (int64_t)j * NE;
                double* vn = V + (int64_t)(j + 1) * NE;
                /* prec and SpMV are timed with events (no extra host synchronisation) */
                HIP_OK(hipEventRecord(ev[0], c->stream));
                if (opt->prec > 0) {
                    rc = prec_apply(c, vj, zj);
                    if (rc) return rc;
                } else {
                    HIP_OK(hipMemcpyAsync(zj, vj, sizeof(double) * NE, hipMemcpyDeviceToDevice, c->stream));
                }
                HIP_OK(hipEventRecord(ev[1], c->stream));
                rc = spmv(c, zj, vn, c->stream);
                if (rc) return rc;
                HIP_OK(hipEventRecord(ev[2], c->stream));

                /* DGKS (Belos' default orthogonalisation): one classical Gram-Schmidt pass
                 * h = V^T w (with ||w||^2 in the same launch), w -= V h (with ||w||^2 fused),
                 * and a second pass only when the norm dropped below 1/sqrt(2) of its value
                 * (dep_tol, BelosDGKSOrthoManager).  One host synchronisation per pass. */
                double hn2 = 0.0;
                {
                    double ww0 = 0.0;
                    rc = orth_pass(c, V + o, NE, j + 1, vn + o, h.data(), &ww0, &hn2);
                    if (rc) return rc;
                    if (hn2 < 0.5 * ww0) {
                        double dummy = 0.0;
                        rc = orth_pass(c, V + o, NE, j + 1, vn + o, h2.data(), &dummy, &hn2);
                        if (rc) return rc;
                        for (int i = 0; i <= j; i++) h[i] += h2[i];
                        inf_reorth++;
                    }
                }
                if (!std::isfinite(hn2)) return nonfinite();
                double hn = sqrt0(hn2);
                if (hn > 0)
                    hipLaunchKernelGGL(k_scale_copy, dim3(G), dim3(256), 0, c->stream, vn + o, 1.0 / hn,
                                       vn + o, NL);
                {
                    float a1 = 0.f, a2 = 0.f;
                    (void)hipEventElapsedTime(&a1, ev[0], ev[1]);
                    (void)hipEventElapsedTime(&a2, ev[1], ev[2]);
                    inf.t_prec_ms += a1;
                    inf.t_spmv_ms += a2;
                    inf.n_spmv++;
                }
                for (int i = 0; i <= j; i++) H[(size_t)i * m + j] = h[i];
                H[(size_t)(j + 1) * m + j] = hn;
                for (int i = 0; i < j; i++) {
                    double a = H[(size_t)i * m + j], bb = H[(size_t)(i + 1) * m + j];
                    H[(size_t)i * m + j] = cs[i] * a + sn[i] * bb;
                    H[(size_t)(i + 1) * m + j] = -sn[i] * a + cs[i] * bb;
                }
                double a = H[(size_t)j * m + j], bb = H[(size_t)(j + 1) * m + j];
                double d = std::sqrt(a * a + bb * bb);
                cs[j] = d > 0 ? a / d : 1.0;
                sn[j] = d > 0 ? bb / d : 0.0;
                H[(size_t)j * m + j] = d;
                H[(size_t)(j + 1) * m + j] = 0.0;
                g[j + 1] = -sn[j] * g[j];
                g[j] = cs[j] * g[j];
                res = std::fabs(g[j + 1]) / bnorm;
                it++;
                if (res <= opt->tol || hn == 0.0) {
                    j++;
                    break;
                }
            }
        } else {
            /* DCGS2 (delayed classical Gram-Schmidt with reorthogonalisation): the new
             * vector u_j is orthogonalised once when produced and re-orthogonalised one step
             * later in the same pass over the basis that orthogonalises the next candidate;
             * normalisation is folded in.  One read pass (k_dcgs_dot) + one update pass
             * (k_dcgs_update) over the basis per iteration; the Hessenberg column j-1 is final
             * (and the residual known) at iteration j.
             * Pipelined: the update coefficients come from the device (k_dcgs_coef), so the
             * host enqueues iteration jj+1 (update, preconditioner, SpMV, dot pass) before it
             * waits for iteration jj's dot rows; the queue never drains on a host round trip.
             * The one speculative iteration past convergence only touches columns the
             * solution update does not read. */
            std::vector<double> htent(m + 1), col(m + 1);
            int ncolf = 0;                 /* finalised columns */
            /* the basis: compressed (Vc, stride NC, from row 0) or the ext vectors' owned rows */
            double* const Q = cmp ? Vc : V + o;
            const int64_t LQ = cmp ? NC : NE, NQ = cmp ? NC : NL;
            const int nbx1 = (int)std::min<int64_t>(RED_BLOCKS, (NQ / 2 + 256 * DOT1_E - 1) / (256 * DOT1_E));
            /* z_jj = M u_jj with u_jj of norm bt_jj: the Hessenberg column of z_jj / bt_jj is
             * the one assembled below, so the solution update divides y_jj by bt_jj */
            std::fill(zs.begin(), zs.end(), 1.0);
            /* iteration jj: [update of jj-1 enqueued before] prec, SpMV, dot pass, coefficients,
             * rows -> pinned slot jj % 2, update */
            auto enqueue = [&](int jj) -> int {
                double* u = Q + (int64_t)jj * LQ;
                double* wv = jj < m ? Q + (int64_t)(jj + 1) * LQ : nullptr;
                hipEvent_t* e = ev + 3 * (jj & 1);
                int rc2;
                if (jj < m) {
                    double* zj = Z + (int64_t)jj * NE;
                    HIP_OK(hipEventRecord(e[0], c->stream));
                    if (cmp) {
                        /* the block GS reads the compressed u (staged into its planar right-hand
                         * side by the previous update pass, jj > 0), the SpMV writes the
                         * compressed w */
                        if ((rc2 = gs_apply_c(c, u, zj, jj > 0))) return rc2;
                    } else if (opt->prec > 0) {
                        if ((rc2 = prec_apply(c, u - o, zj))) return rc2;
                    } else {
                        HIP_OK(hipMemcpyAsync(zj, u - o, sizeof(double) * NE, hipMemcpyDeviceToDevice,
                                              c->stream));
                    }
                    if (cmp) {
                        /* e[1] .. e[2]: the SpMV kernel alone (bench.py's roofline.launch_us) */
                        if ((rc2 = halo_exchange(c, zj, 1))) return rc2;
                        if ((rc2 = spmv_kernel_c(c, zj, wv, e[1], e[2]))) return rc2;
                    } else {
                        HIP_OK(hipEventRecord(e[1], c->stream));
                        if ((rc2 = spmv(c, zj, wv - o, c->stream))) return rc2;
                        HIP_OK(hipEventRecord(e[2], c->stream));
                    }
                }
                /* dot pass: a = Q^T u, b = Q^T w, u.u, u.w, w.w (Q = V_0..jj-1), summed over ranks */
                const int nv = jj;
                const double* wd = wv ? wv : u;
                hipLaunchKernelGGL(k_dcgs_dot1, dim3(nbx1), dim3(256), sizeof(double) * 4 * (2 * nv + 3),
                                   c->stream, Q, LQ, nv, u, wd, NQ, c->d_part.p, nbx1);
                hipLaunchKernelGGL(k_mdot_final, dim3(2 * nv + 3), dim3(256), 0, c->stream, c->d_part.p,
                                   nbx1, 2 * nv + 3, c->d_hbuf.p);
                if ((rc2 = allreduce_sum(c, c->d_hbuf.p, 2 * nv + 3))) return rc2;
                hipLaunchKernelGGL(k_dcgs_coef, dim3(1), dim3(256), 0, c->stream, c->d_hbuf.p, nv,
                                   c->d_hbuf.p + RED_ROWS, c->h_red + (size_t)RED_ROWS * (jj & 1));
                HIP_OK(hipEventRecord(evr[jj & 1], c->stream));
                if (jj < m)
                    hipLaunchKernelGGL(k_dcgs_update, dim3((unsigned)std::min<int64_t>(4096, (NQ / 2 + 255) / 256)), dim3(256), 0, c->stream, Q, LQ, nv,
                                       c->d_hbuf.p + RED_ROWS, u, wv, NQ, cmp ? (const int*)gs.act.p : nullptr,
                                       c->own0, (int64_t)c->next, cmp ? gs.rrP.p : nullptr);
                return 0;
            };
            if ((rc = enqueue(0))) return rc;
            for (int jj = 0; jj <= m; jj++) {
                if (jj < m && (rc = enqueue(jj + 1))) return rc;
                DEV_WAIT_EVENT(c, evr[jj & 1]);
                if (jj < m) {
                    float a1 = 0.f, a2 = 0.f;
                    hipEvent_t* e = ev + 3 * (jj & 1);
                    (void)hipEventElapsedTime(&a1, e[0], e[1]);
                    (void)hipEventElapsedTime(&a2, e[1], e[2]);
                    inf.t_prec_ms += a1;
                    inf.t_spmv_ms += a2;
                    inf.n_spmv++;
                }
                const int nv = jj;
                const double* hr = c->h_red + (size_t)RED_ROWS * (jj & 1);
                const double uu = hr[2 * nv], uw = hr[2 * nv + 1];
                if (!std::isfinite(uu) || !std::isfinite(uw)) {
                    (void)dev_wait(c, nullptr, "fgmres");
                    return nonfinite();
                }
                const double bt = hr[2 * nv + 3], hjj = hr[2 * nv + 4];
                bool stop = false;
                if (jj >= 1) {
                    /* finalise column jj-1: tentative + reorthogonalisation coefficients */
                    const int q = jj - 1;
                    for (int i = 0; i < jj; i++) col[i] = htent[i] + hr[2 * i];
                    col[jj] = bt;
                    for (int i = 0; i <= jj; i++) H[(size_t)i * m + q] = col[i];
                    for (int i = 0; i < q; i++) {
                        const double x0 = H[(size_t)i * m + q], x1 = H[(size_t)(i + 1) * m + q];
                        H[(size_t)i * m + q] = cs[i] * x0 + sn[i] * x1;
                        H[(size_t)(i + 1) * m + q] = -sn[i] * x0 + cs[i] * x1;
                    }
                    const double x0 = H[(size_t)q * m + q], x1 = H[(size_t)(q + 1) * m + q];
                    const double d = std::sqrt(x0 * x0 + x1 * x1);
                    cs[q] = d > 0 ? x0 / d : 1.0;
                    sn[q] = d > 0 ? x1 / d : 0.0;
                    H[(size_t)q * m + q] = d;
                    H[(size_t)(q + 1) * m + q] = 0.0;
                    g[q + 1] = -sn[q] * g[q];
                    g[q] = cs[q] * g[q];
                    res = std::fabs(g[q + 1]) / bnorm;
                    ncolf = jj;
                    it++;
                    stop = res <= opt->tol || !(bt > 0.0);
                }
                if (stop || jj == m || !(bt > 0.0)) break;
                /* the update pass (already enqueued): q_jj = (u - Q a)/bt,  w -= Q c + gamma u */
                for (int i = 0; i < nv; i++) htent[i] = hr[2 * i + 1] / bt;
                htent[nv] = hjj / bt;
                zs[jj] = bt;
            }
            /* the speculative iteration and its copy into the pinned slots finish before the
             * slots are reused as the staging area of the solution update */
            DEV_SYNC(c);
            j = ncolf;
        }
        /* y = H \ g ; x += Z y */
        int k = j;
        for (int i = k - 1; i >= 0; i--) {
            double t = g[i];
            for (int q = i + 1; q < k; q++) t -= H[(size_t)i * m + q] * y[q];
            y[i] = t / H[(size_t)i * m + i];
        }
        if (k > 0) {
            for (int i = 0; i < k; i++) y[i] /= zs[i];
            if ((rc = upload_coeffs(c, y.data(), k))) return rc;
            hipLaunchKernelGGL(k_mupdate_add, dim3(G), dim3(256), 0, c->stream, Z + o, NE, k,
                               c->d_hbuf.p + RED_ROWS, x + o, NL);
        }
        if (cycle == opt->max_restarts) break;
        /* r = b - J x; a cycle that converged on the implicit (Givens) estimate restarts
         * only if the true residual has not reached the tolerance */
        rc = spmv(c, x, r, c->stream);
        if (rc) return rc;
        hipLaunchKernelGGL(k_axpby, dim3(G), dim3(256), 0, c->stream, 1.0, b + o, -1.0, r + o, r + o, NL);
        beta = sqrt0(dot(c, r, r, 0));
        res = beta / bnorm;
        if (res <= opt->tol) break;
        /* stagnation: switch the preconditioner to its safe variant (FGMRES is flexible) */
        if (opt->prec == 2 && it - it_c0 >= STAG_MIN && res > STAG_RATIO * res_c0 && prec_safeguard(c))
            inf.safeguard++;
        res_c0 = res;
    }
    /* the identity-row part of a reduced right-hand side: x = x' + t */
    if (known_rhs)
        hipLaunchKernelGGL(k_axpby, dim3(G), dim3(256), 0, c->stream, 1.0, x + o, 1.0, c->kr.t.p + o, x + o, NL);
    b = b_orig;
    /* explicit residual (Ocean.C:1140-1150) */
    rc = spmv(c, x, w, c->stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_axpby, dim3(G), dim3(256), 0, c->stream, 1.0, b + o, -1.0, w + o, w + o, NL);
    double e2 = dot(c, w, w, 0);
    inf.iters = it;
    inf.reorth = inf_reorth;
    inf.implicit_rel_res = res;
    inf.explicit_rel_res = sqrt0(e2) / bnorm;
    /* converged: the Givens estimate reached the tolerance and the true residual agrees
     * with it (a loss of orthogonality shows up as a gap between the two) */
    inf.converged = res <= opt->tol && inf.explicit_rel_res <= 2.0 * opt->tol;
    inf.t_total_ms = ms_since(T0);
    /* everything that is not the (event-timed) preconditioner or SpMV: Gram-Schmidt
     * passes, reductions, host synchronisation and the Hessenberg work */
    inf.t_orth_ms = std::max(0.0, inf.t_total_ms - inf.t_prec_ms - inf.t_spmv_ms);
    HIP_OK(hipGetLastError());
    if (info) *info = inf;
    return 0;
}

}  // namespace iemic

/* ---- IDR(s) (src/idrsolver/IDRSolver.H:109-340, van Gijzen & Sonneveld) -------------- */
namespace iemic {

/* y = a y + sum_i c_i X_i (i < nv <= 16), coefficients by value */
struct LinComb {
    int nv;
    double a;
    double c[16];
    const double* X[16];
};
/* y may also be one of the X (the IDR update of U(:,k) reads U(:,k)): no __restrict__ */
__global__ void __launch_bounds__(256) k_lincomb(LinComb L, double* y, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x) {
        double acc = L.a == 0.0 ? 0.0 : L.a * y[q];
        for (int i = 0; i < L.nv; i++) acc += L.c[i] * L.X[i][q];
        y[q] = acc;
    }
}

/* the IDR shadow space P: s vectors uniform in [-1, 1] from splitmix64 over the global
 * row index (identical for every band split), orthonormalised (IDRSolver::createP) */
__global__ void k_idr_random(double* __restrict__ P, int64_t ldp, int s, int64_t NL, int64_t row0,
                             int n, int m, int l, int jb0, int ib0, int nx)
{
    const int64_t lr = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lr >= NL) return;
    /* owned row -> global reference row 6((k m + j) n + i) + v */
    const int64_t lc = lr / NUN;
    const int v = (int)(lr % NUN);
    const int i = ib0 + (int)(lc % nx), k = (int)((lc / nx) % l), j = jb0 + (int)(lc / ((int64_t)nx * l));
    const uint64_t g = (uint64_t)(NUN * (((int64_t)k * m + j) * n + i) + v);
    for (int q = 0; q < s; q++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * (g * 16 + (uint64_t)q + 1) + 20261015ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        P[(int64_t)q * ldp + row0 + lr] = 2.0 * ((double)(z >> 11) * (1.0 / 9007199254740992.0)) - 1.0;
    }
}

/* two independent combinations in one pass (y1 = a1 y1 + sum c_i X_i, y2 likewise) */
__global__ void __launch_bounds__(256) k_lincomb2(LinComb L1, double* y1, LinComb L2, double* y2, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x) {
        double a1 = L1.a == 0.0 ? 0.0 : L1.a * y1[q];
        for (int i = 0; i < L1.nv; i++) a1 += L1.c[i] * L1.X[i][q];
        double a2 = L2.a == 0.0 ? 0.0 : L2.a * y2[q];
        for (int i = 0; i < L2.nv; i++) a2 += L2.c[i] * L2.X[i][q];
        y1[q] = a1;
        y2[q] = a2;
    }
}
static LinComb make_lc(double a, const std::vector<double>& cs, const std::vector<const double*>& xs, int64_t o)
{
    LinComb L{};
    L.a = a;
    for (size_t q = 0; q < cs.size() && q < 16; q++) {
        L.c[L.nv] = cs[q];
        L.X[L.nv] = xs[q] + o;
        L.nv++;
    }
    return L;
}
static void lincomb2(iemic_ctx* c, double a1, double* y1, const std::vector<double>& c1,
                     const std::vector<const double*>& x1, double a2, double* y2, const std::vector<double>& c2,
                     const std::vector<const double*>& x2, int64_t o, int64_t NL)
{
    hipLaunchKernelGGL(k_lincomb2, dim3(grid_for(NL)), dim3(256), 0, c->stream, make_lc(a1, c1, x1, o), y1 + o,
                       make_lc(a2, c2, x2, o), y2 + o, NL);
}

static void lincomb(iemic_ctx* c, double a, double* y, std::initializer_list<std::pair<double, const double*>> terms,
                    int64_t o, int64_t NL)
{
    LinComb L{};
    L.a = a;
    for (auto& t : terms) {
        if (L.nv == 16) break;
        L.c[L.nv] = t.first;
        L.X[L.nv] = t.second + o;
        L.nv++;
    }
    hipLaunchKernelGGL(k_lincomb, dim3(grid_for(NL)), dim3(256), 0, c->stream, L, y + o, NL);
}
static void lincomb_v(iemic_ctx* c, double a, double* y, const std::vector<double>& cs,
                      const std::vector<const double*>& xs, int64_t o, int64_t NL)
{
    LinComb L{};
    L.a = a;
    for (size_t q = 0; q < cs.size() && q < 16; q++) {
        L.c[L.nv] = cs[q];
        L.X[L.nv] = xs[q] + o;
        L.nv++;
    }
    hipLaunchKernelGGL(k_lincomb, dim3(grid_for(NL)), dim3(256), 0, c->stream, L, y + o, NL);
}

int idrs(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt, iemic_solve_info* info)
{
    const int s = std::max(1, std::min(opt->idr_s > 0 ? opt->idr_s : 4, 8));
    const double angle = opt->idr_angle > 0.0 ? opt->idr_angle : 0.7;
    const double mp = 1e-13;
    const int maxit = std::max(1, opt->krylov_dim * (opt->max_restarts + 1));
    const int64_t NE = c->nerows, o = NUN * c->own0, NL = c->nlrows;
    /* vectors: P (s) | U (s) | G (s) | t | r | v  in the Krylov basis storage */
    int rc = ensure_krylov(c, 3 * s + 3);
    if (rc) return rc;
    iemic_solve_info inf{};
    auto T0 = std::chrono::steady_clock::now();
    double* base = c->kr.V.p;
    double* P = base;
    double* U = base + (int64_t)s * NE;
    double* G = base + (int64_t)2 * s * NE;
    double* t = base + (int64_t)3 * s * NE;
    double* r = t + NE;                          /* t, r adjacent: one multi-dot for omega */
    double* v = r + NE;
    auto Ui = [&](int i) { return U + (int64_t)i * NE; };
    auto Gi = [&](int i) { return G + (int64_t)i * NE; };
    auto Pi = [&](int i) { return P + (int64_t)i * NE; };
    const unsigned GR = grid_for(NL);
    /* shadow space (createP: random, orthonormalised in order) */
    hipLaunchKernelGGL(k_idr_random, dim3((unsigned)((NL + 255) / 256)), dim3(256), 0, c->stream, P, NE, s, NL,
                       o, c->n, c->m, c->l, c->jb0, c->ib0, c->nx);
    for (int j = 0; j < s; j++) {
        std::vector<double> al(j + 1);
        if (j > 0 && (rc = mdot_host(c, P + o, NE, j, Pi(j) + o, al.data()))) return rc;
        std::vector<double> cs;
        std::vector<const double*> xs;
        for (int k = 0; k < j; k++) { cs.push_back(-al[k]); xs.push_back(Pi(k)); }
        if (j > 0) lincomb_v(c, 1.0, Pi(j), cs, xs, o, NL);
        const double nn = sqrt0(dot(c, Pi(j), Pi(j), 0));
        if (!(nn > 0.0)) return nonfinite();
        hipLaunchKernelGGL(k_scale_copy, dim3(GR), dim3(256), 0, c->stream, Pi(j) + o, 1.0 / nn, Pi(j) + o, NL);
    }
    if ((rc = dev_zero(c, x, NE))) return rc;
    HIP_OK(hipMemcpyAsync(r, b, sizeof(double) * NE, hipMemcpyDeviceToDevice, c->stream));
    const double normb = sqrt0(dot(c, b, b, 0));
    if (!std::isfinite(normb)) return nonfinite();
    if (!(normb > 0.0)) {
        inf.converged = 1;
        if (info) *info = inf;
        return 0;
    }
    const double tolb = opt->tol * normb;
    double normr = normb;
    std::vector<double> f(s, 0.0), gamma(s, 0.0), d(s + 2, 0.0);
    std::vector<std::vector<double>> M(s, std::vector<double>(s, 0.0));
    double om = 1.0;
    int jj = 0, iter = 0;
    bool trueres = false;
    hipEvent_t e0, e1, e2;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventCreate(&e2));
    struct Ev { hipEvent_t a, b, c2; ~Ev() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); (void)hipEventDestroy(c2); } } evg{e0, e1, e2};
    auto prec = [&](const double* in, double* out) -> int {
        HIP_OK(hipEventRecord(e0, c->stream));
        int r2 = 0;
        if (opt->prec > 0) r2 = prec_apply(c, in, out);
        else HIP_OK(hipMemcpyAsync(out, in, sizeof(double) * NE, hipMemcpyDeviceToDevice, c->stream));
        HIP_OK(hipEventRecord(e1, c->stream));
        return r2;
    };
    /* one host synchronisation per inner step: the multi-dot after the matvec also returns
     * r.r of the previous update, whose convergence check therefore comes one matvec late
     * (wasted only on the final step: the pending step's updates are not applied) */
    auto matvec = [&](double* in, double* out) -> int {
        int r2 = spmv(c, in, out, c->stream);
        HIP_OK(hipEventRecord(e2, c->stream));
        return r2;
    };
    auto times = [&]() {                          /* after a synchronisation: e2 is done */
        float a1 = 0.f, a2 = 0.f;
        (void)hipEventElapsedTime(&a1, e0, e1);
        (void)hipEventElapsedTime(&a2, e1, e2);
        inf.t_prec_ms += a1;
        inf.t_spmv_ms += a2;
        inf.n_spmv++;
    };
    auto set_normr = [&](double rr) -> int {
        normr = sqrt0(rr);
        return std::isfinite(normr) ? 0 : nonfinite();
    };
    bool done = false;
    while (!done && iter < maxit) {
        {
            std::vector<double> fr(s + 1);
            if ((rc = mdot_host(c, P + o, NE, s, r + o, fr.data(), r + o, r + o))) return rc;  /* f = P' r */
            for (int k = 0; k < s; k++) f[k] = fr[k];
            if ((rc = set_normr(fr[s]))) return rc;
            if (normr <= tolb) break;
        }
        for (int k = 0; k < s; k++) {
            if (jj > 0) {
                /* gamma from the lower-triangular M(k:s, k:s); v = r - G(:, k:s) gamma */
                std::vector<double> cs{1.0};
                std::vector<const double*> xs{r};
                for (int i = k; i < s; i++) {
                    double gi = f[i];
                    for (int j = k; j < i; j++) gi -= M[i][j] * gamma[j];
                    gamma[i] = gi / M[i][i];
                    cs.push_back(-gamma[i]);
                    xs.push_back(Gi(i));
                }
                lincomb_v(c, 0.0, v, cs, xs, o, NL);                             /* v = r - G gamma */
                if ((rc = prec(v, t))) return rc;
                /* U(:,k) = om t + U(:, k:s) gamma */
                cs.clear();
                xs.clear();
                cs.push_back(om);
                xs.push_back(t);
                for (int i = k; i < s; i++) { cs.push_back(gamma[i]); xs.push_back(Ui(i)); }
                lincomb_v(c, 0.0, Ui(k), cs, xs, o, NL);
            } else {
                if ((rc = prec(r, Ui(k)))) return rc;                           /* initial space */
            }
            if ((rc = matvec(Ui(k), Gi(k)))) return rc;                          /* G(:,k) = A U(:,k) */
            /* bi-orthogonalise against P(:, 0:k) (the modified Gram-Schmidt of the reference
             * restated as one multi-dot + forward substitution) and the new column of M; the
             * same launch returns r.r after the previous step's update */
            if ((rc = mdot_host(c, P + o, NE, s, Gi(k) + o, d.data(), r + o, r + o))) return rc;
            times();
            if (k > 0) {
                if ((rc = set_normr(d[s]))) return rc;
                if (normr <= tolb) {
                    done = true;
                    break;
                }
            }
            std::vector<double> al(k, 0.0);
            for (int i = 0; i < k; i++) {
                double a = d[i];
                for (int j = 0; j < i; j++) a -= al[j] * M[i][j];
                al[i] = a / M[i][i];
            }
            for (int i = k; i < s; i++) {
                double mik = d[i];
                for (int j = 0; j < k; j++) mik -= al[j] * M[i][j];
                M[i][k] = mik;
            }
            if (k > 0) {
                std::vector<double> cs;
                std::vector<const double*> xg, xu;
                for (int i = 0; i < k; i++) { cs.push_back(-al[i]); xg.push_back(Gi(i)); xu.push_back(Ui(i)); }
                lincomb2(c, 1.0, Gi(k), cs, xg, 1.0, Ui(k), cs, xu, o, NL);
            }
            if (!std::isfinite(M[k][k])) return nonfinite();
            if (M[k][k] == 0.0) {
                set_error("IDR(s): breakdown (M[k][k] == 0)");
                return IEMIC_ERANGE;
            }
            const double beta = f[k] / M[k][k];
            lincomb2(c, 1.0, r, {-beta}, {Gi(k)}, 1.0, x, {beta}, {Ui(k)}, o, NL);   /* r -= beta G, x += beta U */
            if (opt->idr_replace) {
                if ((rc = set_normr(dot(c, r, r, 0)))) return rc;
                if (normr > tolb / mp) trueres = true;
            }
            for (int i = k + 1; i < s; i++) f[i] -= beta * M[i][k];
            iter++;
            if (iter >= maxit) break;
        }
        if (done || iter >= maxit) break;
        jj++;
        /* first residual of G_{j+1}: v = M^-1 r, t = A v, omega, r -= om t, x += om v */
        if ((rc = prec(r, v))) return rc;
        if ((rc = matvec(v, t))) return rc;
        double tt_tr[3];
        if ((rc = mdot_host(c, t + o, NE, 2, t + o, tt_tr, r + o, r + o))) return rc;   /* t.t, r.t, r.r */
        times();
        if ((rc = set_normr(tt_tr[2]))) return rc;
        if (normr <= tolb) break;
        const double nt = sqrt0(tt_tr[0]), ts = tt_tr[1];
        if (!(nt > 0.0) || !std::isfinite(ts)) return nonfinite();
        const double rho = std::fabs(ts / (nt * normr));
        om = ts / (nt * nt);
        if (rho < angle) om = om * angle / rho;                                 /* calc_omega */
        lincomb2(c, 1.0, r, {-om}, {t}, 1.0, x, {om}, {v}, o, NL);
        if (opt->idr_replace) {
            if ((rc = set_normr(dot(c, r, r, 0)))) return rc;
            if (normr > tolb / mp) trueres = true;
            if (trueres && normr < normb) {
                /* residual replacement: r = b - A x */
                if ((rc = spmv(c, x, r, c->stream))) return rc;
                hipLaunchKernelGGL(k_axpby, dim3(GR), dim3(256), 0, c->stream, 1.0, b + o, -1.0, r + o, r + o, NL);
                trueres = false;
                inf.reorth++;
            }
        }
        iter++;
    }
    if (!done && (rc = set_normr(dot(c, r, r, 0)))) return rc;                  /* the final r */
    /* explicit residual */
    if ((rc = spmv(c, x, t, c->stream))) return rc;
    hipLaunchKernelGGL(k_axpby, dim3(GR), dim3(256), 0, c->stream, 1.0, b + o, -1.0, t + o, t + o, NL);
    const double e2v = dot(c, t, t, 0);
    inf.iters = iter;
    inf.implicit_rel_res = normr / normb;
    inf.explicit_rel_res = sqrt0(e2v) / normb;
    inf.converged = normr <= tolb && inf.explicit_rel_res <= 2.0 * opt->tol;
    inf.t_total_ms = ms_since(T0);
    inf.t_orth_ms = std::max(0.0, inf.t_total_ms - inf.t_prec_ms - inf.t_spmv_ms);
    HIP_OK(hipGetLastError());
    if (info) *info = inf;
    return 0;
}

}  // namespace iemic

namespace iemic {
int krylov_solve(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt, iemic_solve_info* info)
{
    if (opt->method == 1) return idrs(c, b, x, opt, info);
    if (opt->method != 0) {
        set_error("krylov: unknown method");
        return IEMIC_EINVAL;
    }
    return fgmres(c, b, x, opt, info);
}
}  // namespace iemic
