#!/bin/bash
# A/B patches, one indexed file (verdict round 4, item 8): each variant is a function that
# edits a copy of i-emic_amd/ in the current directory; scripts/ab_build.sh name=ab:<variant>
# runs it in a temporary copy and builds i-emic_amd/lib/libiemic_amd_<name>.so, timed on one
# box by scripts/gpu_ab.sh + scripts/ab_probe.py (untraced with AB_TRACE=0).  A patch applies
# to the sources it was measured against (column "sources"); the adopted ones are in the tree,
# the others are the record of what was measured.
#
# | variant | what | outcome | sources |
# |---|---|---|---|
# | bts_t | load-policy flips (temporal / non-temporal) | the tree keeps the faster policy of each | round 4 |
# | coeffuse | final sums + coefficients in one workgroup | rejected (25 µs) | round 4 |
# | col512 | column kernels in 512-thread workgroups | no gain | round 4 |
# | cols_all | loads issued on land cells too | rejected (slower in every kernel) | round 4 |
# | cr_nodesc_probe | probe: Schur step vectors without the descriptor wait | no gain: pushing vectors would not pay | round 4 |
# | cr_rc8 | Schur apply steps in 8-row chunks | adopted (−1.3 ms per step) | round 4 |
# | cr_stage | Schur step vectors staged in one flat pass | adopted (solve 30.6 → 29.7 µs) | round 4 |
# | crpk_t | load-policy flips (temporal / non-temporal) | the tree keeps the faster policy of each | round 4 |
# | dcgs_lin | dot pass without the XCD dealing | rejected | round 4 |
# | dcgs_nt | non-temporal basis loads in the DCGS2 passes | adopted (dot 84.2 → 73.7 µs) | round 4 |
# | dot1_e2 | 2 / 8 elements per lane in the one-read dot pass | rejected (93.5 / 90.8 vs 85.4 µs) | round 4 |
# | dot1_e8 | 2 / 8 elements per lane in the one-read dot pass | rejected (93.5 / 90.8 vs 85.4 µs) | round 4 |
# | dyn2c | defect with 2 cells per lane / 8 waves | rejected | round 4 |
# | dyn8w | defect with 2 cells per lane / 8 waves | rejected | round 4 |
# | dyn_all | loads issued on land cells too | rejected (slower in every kernel) | round 4 |
# | dyn_noskip | defect reading the W row's T/S slots again | rejected (22.5 -> 24.7 us) | round 5 (f500835) |
# | dyn_nt | non-temporal defect / rcol loads, re-tested | rejected (+2 / +1 ms) | round 4 |
# | dyn_occ4 | defect capped at 4 waves per SIMD | rejected (slower) | round 5 (f500835) |
# | dyn_occ5 | defect capped at 5 waves per SIMD | rejected (slower) | round 5 (f500835) |
# | dyn_t | load-policy flips (temporal / non-temporal) | the tree keeps the faster policy of each | round 4 |
# | upd_fit | DCGS2 update pass on a grid fitted to the compressed basis | adopted (117.3 -> 117.1 ms) | round 6 (54c7f0e) |
# | rev:180a20a | the in-solve SpMV as a persistent kernel (k_spmv7p; its patches sp7c / sp7p4 there) | rejected: 33.3-34.1 vs 29.1 us per launch | round 6 (180a20a) |
# | dot1_e2 (re-test) | 2 elements per lane on the compressed basis (709 workgroups) | rejected (117.3 -> 118.7 ms) | round 6 (54c7f0e) |
# | gemvw_t | load-policy flips (temporal / non-temporal) | the tree keeps the faster policy of each | round 4 |
# | mg_unfused | coarse T/S levels by the unfused launches (k_mg_zl + k_mg_rc) | the fused k_mg_dn / k_mg_up adopted | round 5 (f500835) |
# | mg_wg64 | z-line / restriction launches in 64-thread workgroups | adopted (T/S 112 → 103 µs per apply) | round 4 |
# | ptil_all | loads issued on land cells too | rejected (slower in every kernel) | round 4 |
# | pw_all | loads issued on land cells too | rejected (slower in every kernel) | round 4 |
# | rcol_nt | non-temporal defect / rcol loads, re-tested | rejected (+2 / +1 ms) | round 4 |
# | rr_idonly | entry-kernel store variants | no gain | round 4 |
# | rr_vec | entry-kernel store variants | no gain | round 4 |
# | small64 | tail / coarsest GEMV in 64-thread workgroups | rejected | round 4 |
# | soa_probe | probe: unit-stride accesses in the dynamics kernels | led to the planar dynamics vectors (adopted, −10 ms) | round 4 |
# | spmv_t | load-policy flips (temporal / non-temporal) | the tree keeps the faster policy of each | round 4 |
# | upd_g2048 | update pass variants | rejected | round 4 |
# | upd_un8 | update pass variants | rejected | round 4 |
# | uvp_all | loads issued on land cells too | rejected (slower in every kernel) | round 4 |
# | vb_stage | explicit staging in the GEMVs | no gain | round 4 |
# | xh1 | x halos on the first 1 / 2 intermediate T/S levels only | rejected (285 / 276 vs 206 FGMRES steps at 4 × 2) | round 4 |
# | xh2 | x halos on the first 1 / 2 intermediate T/S levels only | rejected (285 / 276 vs 206 FGMRES steps at 4 × 2) | round 4 |
#
# usage: (cd <copy>/i-emic_amd && bash <repo>/scripts/ab_patches.sh <variant>)
set -e

ab_bts_t() {
# T/S right-hand side coefficients with the default (temporal) load policy
sed -i 's/? 0.0 : __builtin_nontemporal_load(val + (int64_t)(B + s) \* nloc + lc);/? 0.0 : val[(int64_t)(B + s) * nloc + lc];/' csrc/prec_gs.hip
}

ab_coeffuse() {
# one rank: the DCGS2 dot rows summed over the workgroup partials inside the coefficient
# kernel (one 1024-thread launch instead of k_mdot_final + k_dcgs_coef)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
anchor='/* DCGS2 update pass, one read of Q:'
new='''/* rows t < nrow of hb = sum over the nb partials (partial[t * nb + b]), one wave per row in
 * turn, then the coefficients as k_dcgs_coef (one rank: no sum over ranks in between) */
__global__ void __launch_bounds__(1024) k_dcgs_final_coef(const double* __restrict__ partial, int nb,
                                                          double* __restrict__ hb, int nv,
                                                          double* __restrict__ coef)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int nrow = 2 * nv + 3;
    for (int t = wv; t < nrow; t += nw) {
        double a = 0.0;
        for (int b = lane; b < nb; b += 64) a += partial[(int64_t)t * nb + b];
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) hb[t] = a;
    }
    __syncthreads();
    __shared__ double sm[2 * 16];
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
}

'''
s=s.replace(anchor,new+anchor,1)
old='''                hipLaunchKernelGGL(k_mdot_final, dim3(2 * nv + 3), dim3(256), 0, c->stream, c->d_part.p,
                                   nbx1, 2 * nv + 3, c->d_hbuf.p);
                if ((rc2 = allreduce_sum(c, c->d_hbuf.p, 2 * nv + 3))) return rc2;
                hipLaunchKernelGGL(k_dcgs_coef, dim3(1), dim3(256), 0, c->stream, c->d_hbuf.p, nv,
                                   c->d_hbuf.p + RED_ROWS);'''
new2='''                if (c->nranks <= 1) {
                    hipLaunchKernelGGL(k_dcgs_final_coef, dim3(1), dim3(1024), 0, c->stream, c->d_part.p, nbx1,
                                       c->d_hbuf.p, nv, c->d_hbuf.p + RED_ROWS);
                } else {
                    hipLaunchKernelGGL(k_mdot_final, dim3(2 * nv + 3), dim3(256), 0, c->stream, c->d_part.p,
                                       nbx1, 2 * nv + 3, c->d_hbuf.p);
                    if ((rc2 = allreduce_sum(c, c->d_hbuf.p, 2 * nv + 3))) return rc2;
                    hipLaunchKernelGGL(k_dcgs_coef, dim3(1), dim3(256), 0, c->stream, c->d_hbuf.p, nv,
                                       c->d_hbuf.p + RED_ROWS);
                }'''
assert old in s
s=s.replace(old,new2)
open(p,'w').write(s)
PY
}

ab_col512() {
# column kernels (ptil + rcol, p/w) in 512-thread workgroups: 32 columns x 16 levels, twice
# the workgroups (228 -> 456 at 2 degrees: every CU busy)
sed -i 's|^constexpr int col_ti() { return 1024 / LP; }|constexpr int col_ti() { return 512 / LP; }|' csrc/prec_gs.hip
sed -i 's|^    const int cti = 1024 / Pl;|    const int cti = 512 / Pl;|' csrc/prec_gs.hip
sed -i 's|^    const dim3 bct(1024u);|    const dim3 bct(512u);|' csrc/prec_gs.hip
grep -q "return 512 / LP" csrc/prec_gs.hip && grep -q "bct(512u)" csrc/prec_gs.hip && grep -q "cti = 512 / Pl" csrc/prec_gs.hip
}

ab_cols_all() {
ab_uvp_all && ab_pw_all && ab_ptil_all
}

ab_cr_nodesc_probe() {
# timing probe only (wrong values): the Schur step vectors staged from fixed offsets of b, so
# no vector load waits for the workgroup's descriptor (upper bound of pushing the vectors
# into consumer order)
python3 - <<'PY'
p='csrc/schur_cr.hip'
s=open(p).read()
old='''            int ref = refs[0];
#pragma unroll
            for (int q = 1; q < CR_MT; q++)
                if (qv[i] == q) ref = refs[q];
            v[i] = cv[i] >= 0 ? base[ref >> 28][(ref & 0x0fffffff) + cv[i]] : 0.0;'''
new='''            (void)refs;
            v[i] = cv[i] >= 0 ? b[(w % 64) * m + qv[i] * m + cv[i]] : 0.0;'''
assert old in s
s=s.replace(old,new)
s=s.replace('const int tot = nv * m;','const int tot = 6 * m;')
open(p,'w').write(s)
PY
}

ab_cr_rc8() {
# Schur apply steps in 8-row chunks (twice the workgroups of the 16-row default)
sed -i 's/^    int rcw = 16;$/    int rcw = 8;/' csrc/schur_cr.hip
grep -q "^    int rcw = 8;$" csrc/schur_cr.hip
}

ab_cr_stage() {
# Schur apply step: the nv vectors staged in one flat pass (every lane's loads issued together)
python3 - <<'PY'
p='csrc/schur_cr.hip'
s=open(p).read()
old='''    const CrWg& d = wgs[w];
    const int nv = d.nv;
    const double* base[4] = {b, x, bv, xv};
    for (int q = 0; q < nv; q++) {
        const int ref = d.vref[q];
        const double* src = base[ref >> 28] + (ref & 0x0fffffff);
        for (int c = t; c < m; c += 256) vs[q][c] = src[c];
    }
    __syncthreads();'''
new='''    const CrWg& d = wgs[w];
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
    __syncthreads();'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_crpk_t() {
# packed Schur operators with the default (temporal) load policy
sed -i 's/__builtin_nontemporal_load(Pw + ((int64_t)q \* m + c) \* RC + rr)/Pw[((int64_t)q * m + c) * RC + rr]/' csrc/schur_cr.hip
}

ab_dcgs_lin() {
# DCGS2 dot pass in the plain block order (group index fastest, no XCD dealing)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('    const int G = nq + 1, sb = blockIdx.x / (8 * G), rem = blockIdx.x % (8 * G);')
b=s.index('\n', s.index('const int by = rem / 8, bx = sb * 8 + rem % 8;'))
s=s[:a]+'    const int by = blockIdx.x % (nq + 1), bx = blockIdx.x / (nq + 1);'+s[b:]
open(p,'w').write(s)
PY
}

ab_dcgs_nt() {
# DCGS2 passes with non-temporal loads of the basis (streamed once per pass, 1 GB > the
# Infinity Cache)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
helper='''__device__ __forceinline__ double2 ldnt2(const double2* p)
{
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
'''
a=s.index('constexpr int DOT1_E')
s=s[:a]+helper+s[a:]
reps=[('qn[k] = reinterpret_cast<const double2*>(V)[ex[k]];','qn[k] = ldnt2(reinterpret_cast<const double2*>(V) + ex[k]);'),
      ('qn[k] = qv[ex[k]];','qn[k] = ldnt2(qv + ex[k]);'),
      ('q[k] = reinterpret_cast<const double2*>(V + (int64_t)(i + k) * ldv)[e];','q[k] = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)(i + k) * ldv) + e);'),
      ('const double2 q = reinterpret_cast<const double2*>(V + (int64_t)i * ldv)[e];','const double2 q = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)i * ldv) + e);')]
for o,n in reps:
    assert o in s, o
    s=s.replace(o,n)
open(p,'w').write(s)
PY
}

ab_dot1_e2() {
# DCGS2 one-read dot pass with 2 16-byte elements of u, w per lane
sed -i 's/^constexpr int DOT1_E = 4;/constexpr int DOT1_E = 2;/' csrc/krylov.hip
grep -q "DOT1_E = 2;" csrc/krylov.hip
}

ab_dot1_e8() {
# DCGS2 one-read dot pass with 8 16-byte elements of u, w per lane
sed -i 's/^constexpr int DOT1_E = 4;/constexpr int DOT1_E = 8;/' csrc/krylov.hip
grep -q "DOT1_E = 8;" csrc/krylov.hip
}

ab_dyn2c() {
# dynamics defect with two cells per lane (128-cell workgroups): twice the independent loads
# in flight per wave, half the waves
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('__global__ void __launch_bounds__(256) k_spmv_dyn(')
b=s.index('int spmv_dyn_defect(', a)
new='''__global__ void __launch_bounds__(256) k_spmv_dyn(SubLay X, const double* __restrict__ val,
                                                  const double* __restrict__ z,
                                                  const double* __restrict__ r,
                                                  const uint8_t* __restrict__ knP,
                                                  double* __restrict__ d, int64_t nloc, int nblk, int64_t ps)
{
    __shared__ double red[4][2][128];
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t lc0 = (int64_t)tile * 128;
    const int64_t e0 = (int64_t)HALO * X.l * X.nx;
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int64_t lc = lc0 + 64 * h + c;
        if (lc >= nloc) continue;
        const int il = (int)(lc % X.nx), k = (int)((lc / X.nx) % X.l), j = X.jb0 + (int)(lc / ((int64_t)X.nx * X.l));
        int nc[3][9];
        nb_cells(X, il, j, k, nc);
        const int64_t cell = e0 + lc;
        const int v0 = g == 0 ? 0 : g - 1;
        const bool on[2] = {!knP[cell + ps * v0], g > 0 && !knP[cell + ps * (v0 + 1)]};
        if (g == 0) dyn_partial<0, 16>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else if (g == 1) dyn_partial<16, 32>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else if (g == 2) dyn_partial<32, 48>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else dyn_partial<48, 64>(val, z, lc, nloc, nc, on, ps, acc[h]);
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
        red[g][0][64 * h + c] = acc[h][0];
        red[g][1][64 * h + c] = acc[h][1];
    }
    __syncthreads();
    const int R = threadIdx.x >> 6;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int cc = 64 * h + (threadIdx.x & 63);
        if (lc0 + cc >= nloc) break;
        const double sum = R == 0 ? red[0][0][cc] + red[1][0][cc]
                         : R == 1 ? red[1][1][cc] + red[2][0][cc]
                         : R == 2 ? red[2][1][cc] + red[3][0][cc]
                                  : red[3][1][cc];
        const int64_t cell = e0 + lc0 + cc, e = cell + ps * R;
        d[e] = knP[e] ? 0.0 : r[NUN * cell + R] - sum;
    }
}

'''
s=s[:a]+new+s[b:]
old="""    const int nblk = (int)((c->nloc + 63) / 64);
    const unsigned grid = 8u * (unsigned)((nblk + 7) / 8);
    hipLaunchKernelGGL(k_spmv_dyn,"""
new2="""    const int nblk = (int)((c->nloc + 127) / 128);
    const unsigned grid = 8u * (unsigned)((nblk + 7) / 8);
    hipLaunchKernelGGL(k_spmv_dyn,"""
assert old in s
s=s.replace(old,new2)
open(p,'w').write(s)
PY
}

ab_dyn8w() {
# dynamics defect with eight waves of 8 slots per 64 cells (512 threads): half the loads per
# lane, twice the waves
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('__global__ void __launch_bounds__(256) k_spmv_dyn(')
b=s.index('int spmv_dyn_defect(', a)
new='''__global__ void __launch_bounds__(512) k_spmv_dyn(SubLay X, const double* __restrict__ val,
                                                  const double* __restrict__ z,
                                                  const double* __restrict__ r,
                                                  const uint8_t* __restrict__ knP,
                                                  double* __restrict__ d, int64_t nloc, int nblk, int64_t ps)
{
    __shared__ double red[8][2][64];
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t lc0 = (int64_t)tile * 64, lc = lc0 + c;
    const bool act = lc < nloc;
    const int64_t e0 = (int64_t)HALO * X.l * X.nx;
    double acc[2] = {0.0, 0.0};
    if (act) {
        const int il = (int)(lc % X.nx), k = (int)((lc / X.nx) % X.l), j = X.jb0 + (int)(lc / ((int64_t)X.nx * X.l));
        int nc[3][9];
        nb_cells(X, il, j, k, nc);
        const int64_t cell = e0 + lc;
        /* rows of the groups: g0-2 {U} g3-4 {V} g5 {V, W} g6 {W, P} g7 {P} */
        const int v0 = g < 3 ? 0 : g < 5 ? 1 : g == 5 ? 1 : g == 6 ? 2 : 3;
        const bool on[2] = {!knP[cell + ps * v0], (g == 5 || g == 6) && !knP[cell + ps * (v0 + 1)]};
        switch (g) {
        case 0: dyn_partial<0, 8>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 1: dyn_partial<8, 16>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 2: dyn_partial<16, 24>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 3: dyn_partial<24, 32>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 4: dyn_partial<32, 40>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 5: dyn_partial<40, 48>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 6: dyn_partial<48, 56>(val, z, lc, nloc, nc, on, ps, acc); break;
        default: dyn_partial<56, 64>(val, z, lc, nloc, nc, on, ps, acc); break;
        }
    }
    red[g][0][c] = acc[0];
    red[g][1][c] = acc[1];
    __syncthreads();
    if (threadIdx.x >= 256) return;
    const int R = threadIdx.x >> 6, cc = threadIdx.x & 63;
    if (lc0 + cc >= nloc) return;
    const double sum = R == 0 ? (red[0][0][cc] + red[1][0][cc]) + red[2][0][cc]
                     : R == 1 ? (red[3][0][cc] + red[4][0][cc]) + red[5][0][cc]
                     : R == 2 ? red[5][1][cc] + red[6][0][cc]
                              : red[6][1][cc] + red[7][0][cc];
    const int64_t cell = e0 + lc0 + cc, e = cell + ps * R;
    d[e] = knP[e] ? 0.0 : r[NUN * cell + R] - sum;
}

'''
s=s[:a]+new+s[b:]
old="""    hipLaunchKernelGGL(k_spmv_dyn, dim3(grid), dim3(256),"""
assert old in s
s=s.replace(old,"""    hipLaunchKernelGGL(k_spmv_dyn, dim3(grid), dim3(512),""")
open(p,'w').write(s)
PY
}

ab_dyn_all() {
# dynamics defect: the coefficient loads issued for every row (identity rows' sums discarded)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
old='''        const int q = sp7_row(s) - sp7_row(S0);
        if (!on[q]) continue;
        const int cidx'''
new='''        const int q = sp7_row(s) - sp7_row(S0);
        (void)on;
        const int cidx'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_dyn_noskip() {
# A/B: the dynamics defect reading the W row's T/S slots again (z(T, S) = 0: same values)
sed -i '/if (sl.var == TT || sl.var == SS) continue;      \/\* z(T, S) = 0 in every pass \*\//d' csrc/krylov.hip
! grep -q "z(T, S) = 0 in every pass" csrc/krylov.hip
}

ab_dyn_nt() {
# dynamics defect coefficients loaded non-temporally (re-test with the Krylov basis streamed
# non-temporally)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
old='acc[q] += val[(int64_t)s * nloc + lc] * z[(int64_t)cidx + ps * sl.var];'
assert old in s
s=s.replace(old,'acc[q] += __builtin_nontemporal_load(val + (int64_t)s * nloc + lc) * z[(int64_t)cidx + ps * sl.var];')
open(p,'w').write(s)
PY
}

ab_dyn_occ4() {
# A/B: the dynamics defect capped at 4 waves per SIMD
sed -i 's/__global__ void __launch_bounds__(256) k_spmv_dyn(/__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) k_spmv_dyn(/' csrc/krylov.hip
grep -q "amdgpu_waves_per_eu(1, 4))) k_spmv_dyn" csrc/krylov.hip
}

ab_dyn_occ5() {
# A/B: the dynamics defect capped at 5 waves per SIMD (its round-4 occupancy)
sed -i 's/__global__ void __launch_bounds__(256) k_spmv_dyn(/__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 5))) k_spmv_dyn(/' csrc/krylov.hip
grep -q "amdgpu_waves_per_eu(1, 5))) k_spmv_dyn" csrc/krylov.hip
}

ab_dyn_t() {
# dynamics defect coefficients with the default (temporal) load policy
sed -i 's/acc\[q\] += __builtin_nontemporal_load(val + (int64_t)s \* nloc + lc) \* z/acc[q] += val[(int64_t)s * nloc + lc] * z/' csrc/krylov.hip
}

ab_gemvw_t() {
# coarse T/S inverse GEMV with the default (temporal) load policy
sed -i 's/a\[u\] = c < N ? __builtin_nontemporal_load(A + c) : 0.0;/a[u] = c < N ? A[c] : 0.0;/' csrc/prec_gs.hip
}

ab_mg_unfused() {
# A/B: the coarse T/S levels by the unfused launches (k_mg_zl + k_mg_rc) instead of k_mg_dn / k_mg_up
sed -i 's/if (q < 1 || q + 1 >= gs.mg_nlev/if (true || q < 1 || q + 1 >= gs.mg_nlev/' csrc/prec_gs.hip
grep -q "if (true || q < 1" csrc/prec_gs.hip
}

ab_mg_wg64() {
# z-line and restriction launches in 64-thread workgroups (4 columns each): a coarse level's
# few columns spread over 4x the CUs
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
s=s.replace('''#define MG_LAUNCH_P(P, KERNEL, GRID, ...)''','''#define MG_LAUNCH_P64(P, KERNEL, GRID, ...)                                                \\
    do {                                                                                   \\
        if ((P) == 16) hipLaunchKernelGGL(KERNEL<16>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \\
        else if ((P) == 32) hipLaunchKernelGGL(KERNEL<32>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \\
        else hipLaunchKernelGGL(KERNEL<64>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__);     \\
    } while (0)
#define MG_LAUNCH_P(P, KERNEL, GRID, ...)''')
old='''    const unsigned g = blocks_for(mg_columns_of(V, colour) * P);
    if (!g) return 0;'''
new='''    const unsigned g = (unsigned)((mg_columns_of(V, colour) * P + 63) / 64);
    if (!g) return 0;'''
assert old in s
s=s.replace(old,new)
s=s.replace("MG_LAUNCH_P(P, k_mg_zl, g,","MG_LAUNCH_P64(P, k_mg_zl, g,")
s=s.replace("MG_LAUNCH_P(P, k_mg_rc, blocks_for((int64_t)C.n * C.mb * P),","MG_LAUNCH_P64(P, k_mg_rc, (unsigned)(((int64_t)C.n * C.mb * P + 63) / 64),")
open(p,'w').write(s)
PY
grep -q "MG_LAUNCH_P64(P, k_mg_rc" csrc/prec_gs.hip
}

ab_ptil_all() {
# k_gs_ptil_rcol: corner and own-P loads issued on every cell (no branch on the P flag)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='''        if (pa) {
            /* the corner and own-P coefficients vanish on an inactive P row (land): not read */
#pragma unroll'''
new='''        {
#pragma unroll'''
assert old in s
s=s.replace(old,new)
old='''            if (k < l - 1 && !kw) {
                const double g0 = val[(int64_t)S_WP0 * ncell + (cell - L.own0)];
                const double g1 = val[(int64_t)S_WP1 * ncell + (cell - L.own0)];
                if (g0 != 0.0) {'''
new='''            if (k < l - 1) {
                const double g0 = val[(int64_t)S_WP0 * ncell + (cell - L.own0)];
                const double g1 = val[(int64_t)S_WP1 * ncell + (cell - L.own0)];
                if (pa && !kw && g0 != 0.0) {'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_pw_all() {
# k_gs_pw_t: the P-row loads issued on every cell (no branch on the P flag before them)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='''    if (pa) {
        /* an inactive P row (land) reads nothing: its (A, B) = (0, 0) */
        const double a = val[(int64_t)S_PW0 * ncell + (cell - L.own0)];
        const double b = val[(int64_t)S_PWM * ncell + (cell - L.own0)];
        const double rhs = rr[NUN * cell + PP] - duv_uv(val, known, z, i, j, k, cell - L.own0, L);
        pb = pbar[(int64_t)i * L.m + j];
        zp = z[NUN * cell + PP];
        if (wa && a != 0.0) {
            A = rhs / a;
            B = -b / a;
        }
    }'''
new='''    if (on) {
        const double a = val[(int64_t)S_PW0 * ncell + (cell - L.own0)];
        const double b = val[(int64_t)S_PWM * ncell + (cell - L.own0)];
        const double rhs = rr[NUN * cell + PP] - duv_uv(val, known, z, i, j, k, cell - L.own0, L);
        pb = pa ? pbar[(int64_t)i * L.m + j] : 0.0;
        zp = pa ? z[NUN * cell + PP] : 0.0;
        if (pa && wa && a != 0.0) {
            A = rhs / a;
            B = -b / a;
        }
    }'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_rcol_nt() {
# ptil + Schur right-hand side: the rcol coefficients loaded non-temporally
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
reps=[('for (int e = 0; e < 9; e++) a0 += R[e * es] * rr[PL(nc9[e], WW)];','for (int e = 0; e < 9; e++) a0 += __builtin_nontemporal_load(R + e * es) * rr[PL(nc9[e], WW)];'),
      ('a1 += R[(9 + q4) * es] * rr[PL(qc, UU)];','a1 += __builtin_nontemporal_load(R + (9 + q4) * es) * rr[PL(qc, UU)];'),
      ('a2 += R[(13 + q4) * es] * rr[PL(qc, VV)];','a2 += __builtin_nontemporal_load(R + (13 + q4) * es) * rr[PL(qc, VV)];'),
      ('a2 += R[17 * es] * rr[PL(cell, PP)];','a2 += __builtin_nontemporal_load(R + 17 * es) * rr[PL(cell, PP)];')]
for o,n in reps:
    assert o in s, o
    s=s.replace(o,n)
open(p,'w').write(s)
PY
}

ab_rr_idonly() {
# entry kernel: the output's identity rows only (the active rows are all written later: U/V/W/P
# by the last pass, T/S by the multigrid's final launches)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old="""        const double zv = kn[R] ? acc[R] : 0.0;
        z[row] = zv;
        zP[PL(cell, R)] = zv;"""
new="""        const double zv = kn[R] ? acc[R] : 0.0;
        if (kn[R] || rr) z[row] = zv;
        zP[PL(cell, R)] = zv;"""
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_rr_vec() {
# k_gs_rr with 16-byte loads and stores of the AoS cell records and the planar flags
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old="""    double acc[NUN];
    bool kn[NUN];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        const int64_t row = NUN * cell + R;
        acc[R] = r[row];
        kn[R] = known[row] != 0;
        const double zv = kn[R] ? acc[R] : 0.0;
        z[row] = zv;
        zP[PL(cell, R)] = zv;
    }"""
new="""    double acc[NUN];
    bool kn[NUN];
    {
        const double2* r2 = reinterpret_cast<const double2*>(r + NUN * cell);
        const double2 a0 = r2[0], a1 = r2[1], a2 = r2[2];
        acc[0] = a0.x; acc[1] = a0.y; acc[2] = a1.x; acc[3] = a1.y; acc[4] = a2.x; acc[5] = a2.y;
    }
    double zv[NUN];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        kn[R] = known[NUN * cell + R] != 0;
        zv[R] = kn[R] ? acc[R] : 0.0;
        zP[PL(cell, R)] = zv[R];
    }
    {
        double2* z2 = reinterpret_cast<double2*>(z + NUN * cell);
        z2[0] = make_double2(zv[0], zv[1]);
        z2[1] = make_double2(zv[2], zv[3]);
        z2[2] = make_double2(zv[4], zv[5]);
    }"""
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_small64() {
# the dense tail GEMV of the Schur solve and the coarsest T/S GEMV in 64-thread workgroups
# (one row each: 4x the workgroups)
python3 - <<'PY'
for p, kern in (('csrc/schur_cr.hip', 'k_cr_tail('), ('csrc/prec_gs.hip', 'k_gemv_w(')):
    s=open(p).read()
    a=s.index(kern); b=s.index('\n}\n', a)
    k=s[a:b]
    k=k.replace('r = blockIdx.x * 4 + (threadIdx.x >> 6);','r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);')
    k=k.replace('c += 256) vb[c] = b[c];','c += blockDim.x) vb[c] = b[c];')
    s=s[:a]+k+s[b:]
    if kern == 'k_cr_tail(':
        old='hipLaunchKernelGGL(k_cr_tail, dim3((cr.tM + 3) / 4), dim3(256),'
        assert old in s
        s=s.replace(old,'hipLaunchKernelGGL(k_cr_tail, dim3(cr.tM), dim3(64),')
    else:
        for NLv in ('16','32'):
            old=f'hipLaunchKernelGGL(k_gemv_w<{NLv}>, dim3((unsigned)((N + 3) / 4)), dim3(256),'
            assert old in s
            s=s.replace(old,f'hipLaunchKernelGGL(k_gemv_w<{NLv}>, dim3((unsigned)N), dim3(64),')
    open(p,'w').write(s)
PY
}

ab_soa_probe() {
# timing probe only (wrong values): the AoS accesses of the dynamics-pass kernels (ptil + rcol,
# U/V, p/w with duv_uv, the entry k_gs_rr) made stride-1, as a component-planar layout would
# read them (upper bound of a planar-layout rewrite); set-up kernels untouched
python3 - <<'PY'
import re
p='csrc/prec_gs.hip'
s=open(p).read()
for name in ['k_gs_ptil_rcol(', 'k_gs_uvp(', 'k_gs_pw_t(', 'double duv_uv(', 'k_gs_rr(']:
    a=s.rindex(name) if name == 'double duv_uv(' else s.index(name)
    a=s.index('{', a)
    depth=0; b=a
    while True:
        if s[b]=='{': depth+=1
        elif s[b]=='}':
            depth-=1
            if depth==0: break
        b+=1
    s=s[:a]+s[a:b].replace('NUN * ','1 * ')+s[b:]
open(p,'w').write(s)
PY
}

ab_spmv_t() {
# SpMV coefficients with the default (temporal) load policy
sed -i 's/v\[s - S0\] = !act ? 0.0 : __builtin_nontemporal_load(val + (int64_t)s \* nloc + lc);/v[s - S0] = !act ? 0.0 : val[(int64_t)s * nloc + lc];/' csrc/krylov.hip
}

ab_upd_g2048() {
# DCGS2 update pass on 2048 workgroups
sed -i 's/hipLaunchKernelGGL(k_dcgs_update, dim3(1024)/hipLaunchKernelGGL(k_dcgs_update, dim3(2048)/' csrc/krylov.hip
grep -q "k_dcgs_update, dim3(2048)" csrc/krylov.hip
}

ab_upd_un8() {
# DCGS2 update pass with eight basis vectors per step
sed -i 's/^    constexpr int UN = 4;/    constexpr int UN = 8;/' csrc/krylov.hip
grep -q "constexpr int UN = 8;" csrc/krylov.hip
}

ab_uvp_all() {
# k_gs_uvp: every cell issues its loads at once (no early return on land; stores predicated)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='    if (!ua && !va) return;                 /* land: none of the point\'s operands is read */\n'
assert old in s
s=s.replace(old,'')
open(p,'w').write(s)
PY
}

ab_vb_stage() {
# tail and coarsest GEMVs: the right-hand side staged with all of a lane's loads issued first
python3 - <<'PY'
for p, old, nmax in (('csrc/schur_cr.hip', '    for (int c = threadIdx.x; c < M; c += 256) vb[c] = b[c];', 'CR_TAIL_MAX'),
                     ('csrc/prec_gs.hip', '    for (int c = threadIdx.x; c < N; c += 256) vb[c] = b[c];', '64 * NL')):
    s=open(p).read()
    assert old in s, p
    lim = 'M' if 'M;' in old else 'N'
    new=f"""    {{
        constexpr int SV = ({nmax} + 255) / 256;
        double t_[SV];
#pragma unroll
        for (int u = 0; u < SV; u++) {{
            const int c = threadIdx.x + 256 * u;
            t_[u] = c < {lim} ? b[c] : 0.0;
        }}
#pragma unroll
        for (int u = 0; u < SV; u++) {{
            const int c = threadIdx.x + 256 * u;
            if (c < {lim}) vb[c] = t_[u];
        }}
    }}"""
    s=s.replace(old,new)
    open(p,'w').write(s)
PY
}

ab_upd_fit() {
# DCGS2 update pass on a grid fitted to the compressed basis (one 16-byte element per lane)
# instead of 1024 workgroups striding over it (1.4 elements per lane at 2 degrees)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
old="hipLaunchKernelGGL(k_dcgs_update, dim3(1024), dim3(256), 0, c->stream, Q, LQ, nv,"
new="hipLaunchKernelGGL(k_dcgs_update, dim3((unsigned)std::min<int64_t>(4096, (NQ / 2 + 255) / 256)), dim3(256), 0, c->stream, Q, LQ, nv,"
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
}

ab_xh1() {
# x halos on the first 1 intermediate T/S levels only
sed -i "s/^constexpr int MG_XHALO_LEVELS = 99;/constexpr int MG_XHALO_LEVELS = 1;/" csrc/prec_gs.hip
}

ab_xh2() {
# x halos on the first 2 intermediate T/S levels only
sed -i "s/^constexpr int MG_XHALO_LEVELS = 99;/constexpr int MG_XHALO_LEVELS = 2;/" csrc/prec_gs.hip
}

v=${1:?variant}
declare -F "ab_$v" >/dev/null || { echo "no A/B variant $v" >&2; exit 2; }
"ab_$v"
