/*
 * coupled.hip -- the I-EMIC atmosphere model and the coupled ocean + atmosphere block system
 * on the device (BASELINE config C4).
 *
 *   AtmosLocal / Atmosphere (src/atmosphere/AtmosLocal.C, Atmosphere.C)  -> iemic_atmos_*
 *     2-D energy-balance / moisture / albedo model, 3 unknowns per surface cell (T, q, A)
 *     plus the global precipitation anomaly P; one process (aux = 1, integral condition on q)
 *   CoupledModel (src/coupledmodel/CoupledModel.C) with CouplingBlock (CouplingBlock.H)
 *     -> iemic_coupled_*: synchronize (218-233), computeRHS / computeJacobian (236-271),
 *     applyMatrix (436-470), forward block Gauss-Seidel applyPrecon 'F' (544-585) and the
 *     FGMRES solve (274-432)
 *   Ocean::getBlock(atmos) (Ocean.C:1538-1667), Atmosphere::getBlock(ocean)
 *     (Atmosphere.C:502-613) -> the coupling kernels below (applied matrix-free)
 *
 * Data layout: the atmosphere vector in the reference order, row = 3*(j*n + i) + xx
 * (xx = T, q, A; FIND_ROW_ATMOS0, AtmosphereDefinitions.H:45-54), P last.  Its Jacobian
 * is an ELL with 7 slots per row (T: W S C N E + A + P; q: W S C N E + P; A: T A P) plus
 * the two dense rows (q integral, precipitation) applied as reductions.  The per-row
 * arithmetic keeps the reference's evaluation order (compiled without FMA contraction),
 * so the device values equal the CPU restatement oracle/atmos_oracle.py.
 *
 * Atmosphere preconditioner (replaces the Ifpack "Amesos" direct subdomain solve,
 * Atmosphere.C:1349-1366): P from its diagonal, A from its diagonal, then the T and the q
 * 2-D operators solved exactly by block cyclic reduction over longitudes (schur_cr.hip),
 * the q-integral row replaced by an identity row.  The coupled Krylov vectors are packed
 * [ocean owned rows | atmosphere]; one process (the coupled grid is small: 4 degrees).
 */
#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "common.h"
#include "stencil.h"

using namespace iemic;

namespace {
constexpr double PI_ = 3.14159265358979323846;
constexpr int AT = 0, AQ = 1, AA = 2, ANUN = 3, ASL = 7;
}

/* scalar parameters and coefficients (AtmosLocal::setParameters 106-171, setup 174-245) */
struct AtmPar {
    double comb, sunp, lonf, humf, latf, albf, tdif;
    double Ad, bmua, amua, Phv, nuq, eta, qdim, tdim, dqso, dqsi, Po0, Eo0, Ei0, Cs, lvscale;
    double a0, da, tauf, tauc, Ooa, Tm, Tr, Pa, epm, epr, epa, t0o, t0i;
    double total_area;
};

struct iemic_atmos {
    iemic_ctx* oc = nullptr;             /* the ocean context: device, stream, surface mask  */
    int refs = 1;                        /* the handle + coupled models built on it          */
    iemic_atmos_params prm{};
    int n = 0, m = 0, periodic = 0, dim = 0, rowint = 0, rowP = 0;
    AtmPar P{};
    double eta0 = 0, hdimq = 0, rhoo = 0, rhoa = 0, r0dim = 0, udim = 0;   /* for nuq */
    std::vector<int> surf;               /* (j, i): 1 land                                   */
    std::vector<double> tab;             /* per j (1..m): datc*cosdx2i, t4, t6, cosdx2i, q4, */
                                         /* q6, suna, suno (8 (m+1))                         */
    std::vector<double> pdist, pint;     /* n*m                                              */
    DevBuf<double> d_tab, d_pdist, d_pint, d_x, d_sst, d_F, d_val, d_red, d_tmp, d_y;
    DevBuf<int> d_surf, d_col;
    /* preconditioner: 9-point T and q operators, their cyclic reductions, work vectors */
    DevBuf<double> d_s9t, d_s9q, d_bt, d_bq, d_zt, d_zq;
    DevBuf<double> d_w, d_g, d_pred;          /* S_q^-1 (q-P column), P Schur partials + scalar   */
    DevBuf<int> d_colij;
    SchurCR crT, crQ;
    int jac_valid = 0, prec_valid = 0;
};

struct iemic_coupled {
    iemic_ctx* oc = nullptr;
    iemic_atmos* at = nullptr;
    int64_t NL = 0, NA = 0, NC = 0;      /* ocean owned rows, atmosphere rows, packed total  */
    DevBuf<double> xo, yo, ro, zo;       /* ocean ext-layout scratch                         */
    DevBuf<double> V, Z, w, r, tmpa, part, hb;
    DevBuf<double> hc;                   /* FGMRES: the step's CGS2 coefficients and norm    */
    DevBuf<double> tsurf;            /* n*m surface T of a packed vector (several ranks)  */
    int mk = 0;
    int synced = 0;
    double pars[18] = {};                /* CommPars of the last synchronisation            */
    double* h_red = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};  /* FGMRES: a step's coefficients in h_red         */
    ~iemic_coupled()
    {
        if (h_red) (void)hipHostFree(h_red);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

namespace iemic {
namespace {

/* ---- per-cell atmosphere rows (computeJacobian 585-746 + boundaries 1429-1479) ------- */
struct AtmGeo {
    int n, m, periodic, dim, rowint, rowP;
    const double* tab;
    const double* pdist;
    const int* surf;
};

HD double H_(double x, double eps) { return (1. / 2.) * (1.0 + libm_tanh(x / eps)); }

HD double atm_Tl(const AtmPar& P, const AtmGeo& G, double A, double Ta, int j1)
{
    const double suno = G.tab[7 * (G.m + 1) + j1];
    return Ta + P.comb * P.sunp * suno * ((1 - P.a0) - P.da * A) / P.Ooa;
}
HD double atm_aF(const AtmPar& P, const AtmGeo& G, double A, double Ta, double Pv, int i, int j1)
{
    const double dimP = 3600. * 24. * 365. * G.pdist[(j1 - 1) * G.n + i] * (P.Po0 + P.eta * P.qdim * Pv);
    const double tl = atm_Tl(P, G, A, Ta, j1);
    return H_(P.Tm - tl, P.epm) * H_(P.Tr - tl, P.epr) * H_(dimP - P.Pa, P.epa);
}

/* rows T, q, A of cell (i, j) (0-based i, j): values and columns in the reference CRS
 * order, 7 slots each (unused: column -1) */
HD void atm_cell(const AtmPar& P, const AtmGeo& G, const double* x, int i, int j, double v[3][ASL],
                 int col[3][ASL])
{
    const int n = G.n, m = G.m, j1 = j + 1, M1 = m + 1;
    const bool land = G.surf[j * n + i] != 0;
    const double* tb = G.tab;
    const double cx = tb[j1], t4 = tb[M1 + j1], t6 = tb[2 * M1 + j1];
    const double qx = tb[3 * M1 + j1], q4 = tb[4 * M1 + j1], q6 = tb[5 * M1 + j1];
    const double suna = tb[6 * M1 + j1], suno = tb[7 * M1 + j1];
    const double sT = P.tdif * P.Ad;
    const double tc = land ? 0.0 : 1.0;
    /* loc order 2 (W), 4 (S), 5 (C), 6 (N), 8 (E) */
    double a[5], q[5];
    {
        const double txx[5] = {cx, 0.0, -2 * cx, 0.0, cx};
        const double tyy[5] = {0.0, t4, -(t4 + t6), t6, 0.0};
        for (int s = 0; s < 5; s++) {
            double val = sT * txx[s] + sT * tyy[s];
            val = val + (-1.0) * (s == 2 ? tc : 0.0);
            val = val + (-P.bmua) * (s == 2 ? 1.0 : 0.0);
            a[s] = val;
        }
        const double qxx[5] = {qx, 0.0, -2 * qx, 0.0, qx};
        const double qyy[5] = {0.0, q4, -(q4 + q6), q6, 0.0};
        for (int s = 0; s < 5; s++) {
            double val = P.Phv * qxx[s] + P.Phv * qyy[s];
            val = val + (-P.nuq) * (s == 2 ? tc : 0.0);
            q[s] = val;
        }
    }
    double* bs[2] = {a, q};
    for (int b = 0; b < 2; b++) {
        double* z = bs[b];
        if (i == 0 && !G.periodic) { z[2] = z[2] + z[0]; z[0] = 0.0; }
        if (i == n - 1 && !G.periodic) { z[2] = z[2] + z[4]; z[4] = 0.0; }
        if (j1 == m) { z[2] = z[2] + z[3]; z[3] = 0.0; }
        if (j1 == 1) { z[2] = z[2] + z[1]; z[1] = 0.0; }
    }
    const double pd = G.pdist[j * n + i];
    const double tt_pp = P.comb * P.latf * P.lvscale * P.eta * P.qdim * pd;
    const double dTadA = -P.comb * P.sunp * suna * P.da;
    const double dTldA = -P.comb * P.sunp * suno * P.da / P.Ooa;
    const double tt_aa = land ? (dTldA + dTadA) : dTadA;
    const double qq_pp = -P.nuq * pd;
    const int rT = ANUN * (j * n + i);
    double dAdA, dAdP, dAdT;
    if (land) {
        const double A = x[rT + AA], Ta = x[rT + AT], Pv = x[G.rowP];
        const double df = 1e-6;
        const double f0 = atm_aF(P, G, A, Ta, Pv, i, j1);
        const double daA = (atm_aF(P, G, A + df, Ta, Pv, i, j1) - f0) / df;
        const double daP = (atm_aF(P, G, A, Ta, Pv + df, i, j1) - f0) / df;
        const double daT = (atm_aF(P, G, A, Ta + df, Pv, i, j1) - f0) / df;
        dAdA = (P.comb * P.albf * daA - 1) / P.tauf;
        dAdP = (P.comb * P.albf * daP) / P.tauf;
        dAdT = (P.comb * P.albf * daT) / P.tauf;
    } else {
        dAdA = -1 / P.tauc;
        dAdP = 0.0;
        dAdT = 0.0;
    }
    int iw = i - 1, ie = i + 1;
    if (G.periodic) {
        if (iw < 0) iw = n - 1;
        if (ie > n - 1) ie = 0;
    }
    const int cW = ANUN * (j * n + iw), cE = ANUN * (j * n + ie);
    const int cS = ANUN * ((j - 1) * n + i), cN = ANUN * ((j + 1) * n + i);
    for (int r = 0; r < 3; r++)
        for (int s = 0; s < ASL; s++) { v[r][s] = 0.0; col[r][s] = -1; }
    /* T row: W S C(T A P) N E */
    v[0][0] = a[0]; col[0][0] = a[0] != 0.0 ? cW + AT : -1;
    v[0][1] = a[1]; col[0][1] = a[1] != 0.0 ? cS + AT : -1;
    v[0][2] = a[2]; col[0][2] = rT + AT;
    v[0][3] = tt_aa; col[0][3] = rT + AA;
    v[0][4] = tt_pp; col[0][4] = G.rowP;
    v[0][5] = a[3]; col[0][5] = a[3] != 0.0 ? cN + AT : -1;
    v[0][6] = a[4]; col[0][6] = a[4] != 0.0 ? cE + AT : -1;
    /* q row: W S C(q P) N E */
    v[1][0] = q[0]; col[1][0] = q[0] != 0.0 ? cW + AQ : -1;
    v[1][1] = q[1]; col[1][1] = q[1] != 0.0 ? cS + AQ : -1;
    v[1][2] = q[2]; col[1][2] = rT + AQ;
    v[1][3] = qq_pp; col[1][3] = G.rowP;
    v[1][4] = q[3]; col[1][4] = q[3] != 0.0 ? cN + AQ : -1;
    v[1][5] = q[4]; col[1][5] = q[4] != 0.0 ? cE + AQ : -1;
    /* A row: T A P */
    v[2][0] = dAdT; col[2][0] = rT + AT;
    v[2][1] = dAdA; col[2][1] = rT + AA;
    v[2][2] = dAdP; col[2][2] = G.rowP;
}

/* AtmosLocal::forcing (871-984), parallel mode; no sea ice (Msi = sit = 0) */
HD void atm_forcing(const AtmPar& P, const AtmGeo& G, const double* x, const double* sst, int i, int j,
                    double f[3])
{
    const int n = G.n, j1 = j + 1, M1 = G.m + 1;
    const int sr = j * n + i, rT = ANUN * sr;
    const double suna = G.tab[6 * M1 + j1], suno = G.tab[7 * M1 + j1];
    const bool land = G.surf[sr] != 0;
    const double A = x[rT + AA], Ta = x[rT + AT];
    const double QSW = suna * (1 - P.a0);
    const double msi = 0.0, sit = 0.0;
    double v;
    if (land) {
        v = P.comb * P.sunp * suno * (1 - P.a0) / P.Ooa;
        v += P.comb * (P.sunp * QSW - P.lonf * P.amua);
    } else {
        const double Ts = sst[sr] + msi * (sit - sst[sr] + P.t0i - P.t0o);
        v = Ts + P.comb * (P.sunp * QSW - P.lonf * P.amua);
        v += P.comb * P.latf * P.lvscale * G.pdist[sr] * P.Po0;
    }
    f[0] = v;
    if (land) {
        v = 0.0;
    } else {
        const double Eo = (P.tdim / P.qdim) * P.dqso * sst[sr];
        const double Ei = (P.tdim / P.qdim) * P.dqsi * sit;
        v = P.nuq * (Eo + msi * (Ei - Eo + P.Cs));
    }
    f[1] = v;
    if (land)
        v = (P.comb * P.albf * atm_aF(P, G, A, Ta, x[G.rowP], i, j1) - A) / P.tauf;
    else
        v = (P.comb * P.albf * msi - A) / P.tauc;
    f[2] = v;
}

__global__ void k_atm_jac(AtmPar P, AtmGeo G, const double* __restrict__ x, double* __restrict__ val,
                          int* __restrict__ col)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    double v[3][ASL];
    int cl[3][ASL];
    atm_cell(P, G, x, c % G.n, c / G.n, v, cl);
    for (int r = 0; r < 3; r++) {
        const int row = ANUN * c + r;
        const bool dense = row == G.rowint;
        for (int s = 0; s < ASL; s++) {
            val[(size_t)row * ASL + s] = dense ? 0.0 : v[r][s];
            col[(size_t)row * ASL + s] = dense ? -1 : cl[r][s];
        }
    }
}

/* F of the local rows: sum over the non-zero entries in CRS order, then + forcing;
 * the albedo row is its forcing only (AtmosLocal::computeRHS 810-828) */
__global__ void k_atm_rhs(AtmPar P, AtmGeo G, const double* __restrict__ x, const double* __restrict__ sst,
                          double* __restrict__ F)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    const int i = c % G.n, j = c / G.n;
    double v[3][ASL];
    int cl[3][ASL];
    atm_cell(P, G, x, i, j, v, cl);
    double f[3];
    atm_forcing(P, G, x, sst, i, j, f);
    for (int r = 0; r < 3; r++) {
        double val = 0.0;
        if (r != AA) {
            double mv = 0.0;
            for (int s = 0; s < ASL; s++)
                if (cl[r][s] >= 0 && v[r][s] != 0.0) mv += v[r][s] * x[cl[r][s]];
            val += mv;
        }
        val += f[r];
        F[ANUN * c + r] = val;
    }
}

/* block partials of sum w_q x_q over the cells (w: n*m weights; x stride 3 from off) */
__global__ void __launch_bounds__(256) k_atm_wdot(const double* __restrict__ w, const double* __restrict__ x,
                                                  int stride, int off, int nm, double* __restrict__ part)
{
    __shared__ double sm[256];
    double s = 0.0;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nm; q += gridDim.x * blockDim.x)
        s += w[q] * x[(int64_t)stride * q + off];
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}
constexpr int AR_BLOCKS = 64;

/* F[rowint] = intc . x ;  F[P] = -x_P - q_int + sst_int (+ Msi Cs integral = 0)
 * (Atmosphere::computeRHS 320-391); part[0..AR) = intc.x, part[AR..2AR) = pint.sigma */
__global__ void k_atm_rhs_dense(AtmPar P, AtmGeo G, const double* __restrict__ x, const double* __restrict__ part,
                                double* __restrict__ F)
{
    if (threadIdx.x || blockIdx.x) return;
    double a = 0.0, b = 0.0;
    for (int q = 0; q < AR_BLOCKS; q++) a += part[q];
    for (int q = 0; q < AR_BLOCKS; q++) b += part[AR_BLOCKS + q];
    const double intcond = a;
    const double sst_int = b * (1.0 / P.total_area) * (P.tdim / P.qdim);
    const double q_int = intcond * 1.0 / P.total_area;
    const double mcs_int = 0.0 * P.Cs / P.total_area;
    F[G.rowint] = intcond;
    F[G.rowP] = -x[G.rowP] - q_int + sst_int + mcs_int;
}

/* sigma = dqso sst + Msi (dqsi sit - dqso sst) with Msi = sit = 0 (Atmosphere.C:352-363) */
__global__ void k_atm_sigma(AtmPar P, const double* __restrict__ sst, double* __restrict__ sig, int nm)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nm) return;
    const double tmp = P.dqsi * 0.0 + (-P.dqso) * sst[q];
    sig[q] = P.dqso * sst[q] + 1.0 * 0.0 * tmp;
}

/* y = J x on the local rows (ELL); the dense rows from the reduction */
__global__ void k_atm_spmv(const double* __restrict__ val, const int* __restrict__ col, const double* __restrict__ x,
                           double* __restrict__ y, int nrow)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrow) return;
    double s = 0.0;
    for (int k = 0; k < ASL; k++) {
        const int c = col[(size_t)r * ASL + k];
        if (c >= 0) s += val[(size_t)r * ASL + k] * x[c];
    }
    y[r] = s;
}
__global__ void k_atm_spmv_dense(AtmPar P, AtmGeo G, const double* __restrict__ x, const double* __restrict__ part,
                                 double* __restrict__ y)
{
    if (threadIdx.x || blockIdx.x) return;
    double a = 0.0;
    for (int q = 0; q < AR_BLOCKS; q++) a += part[q];
    y[G.rowint] = a;
    y[G.rowP] = (-1.0 / P.total_area) * a + (-1.0) * x[G.rowP];
}

/* preconditioner set-up: 9-point rows (c = i*m + j) of the T-T and q-q blocks; the
 * q-integral row becomes an identity row */
__global__ void k_atm_s9(AtmGeo G, const double* __restrict__ val, double* __restrict__ s9t, double* __restrict__ s9q)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    const int i = c % G.n, j = c / G.n, sc = i * G.m + j;
    double* t = s9t + (size_t)sc * 9;
    double* q = s9q + (size_t)sc * 9;
    for (int o = 0; o < 9; o++) t[o] = q[o] = 0.0;
    const double* vt = val + (size_t)(ANUN * c + AT) * ASL;
    const double* vq = val + (size_t)(ANUN * c + AQ) * ASL;
    /* offsets o = (dj+1)*3 + (di+1): W 3, S 1, C 4, N 7, E 5 */
    t[3] += vt[0]; t[1] += vt[1]; t[4] += vt[2]; t[7] += vt[5]; t[5] += vt[6];
    if (ANUN * c + AQ == G.rowint) {
        q[4] = 1.0;
    } else {
        q[3] += vq[0]; q[1] += vq[1]; q[4] += vq[2]; q[7] += vq[4]; q[5] += vq[5];
    }
}

/* The [q; P] block is solved exactly.  Its two global rows -- the q integral condition
 * (row k: intc . q = b_k) and the precipitation row (rr . q - P = b_P, rr = -(1/A) intc;
 * Atmosphere.C:1039-1067) -- are bordered onto S~, the q stencil operator with row k
 * replaced by the identity (without the integral row the [q; P] system is singular:
 * q = -Pdist t, P = t).  With d = intc - e_k, mu = d . q:
 *   S~ q = b - c P - e_k mu  ->  q = y - w P - g mu,  y = S~^-1 b, w = S~^-1 c, g = S~^-1 e_k
 *   [d.w   d.g + 1] [P ]   [d.y       ]
 *   [rr.w + 1  rr.g] [mu] = [rr.y - b_P]
 * (c: the q rows' P column -nuq Pdist).  w, g and the 2x2 inverse at set-up; per apply one
 * cyclic-reduction solve for y and one reduction.  Then A from its row (A_A z_A = r_A -
 * A_P P) and T from S_T with the A and P columns moved to the right-hand side. */
__global__ void k_atm_qcol(AtmGeo G, const double* __restrict__ val, const double* __restrict__ r,
                           double* __restrict__ cq, double* __restrict__ gk, double* __restrict__ bq)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    const int sc = (c % G.n) * G.m + c / G.n;
    const bool ri = ANUN * c + AQ == G.rowint;
    if (cq) cq[sc] = ri ? 0.0 : val[(size_t)(ANUN * c + AQ) * ASL + 3];
    if (gk) gk[sc] = ri ? 1.0 : 0.0;
    if (bq) bq[sc] = r[ANUN * c + AQ];
}
/* partials of sum_cells pint(cell) v(sc(cell)) */
__global__ void __launch_bounds__(256) k_atm_pdot_sc(AtmGeo G, const double* __restrict__ pint,
                                                     const double* __restrict__ v, double* __restrict__ part)
{
    __shared__ double sm[256];
    double s = 0.0;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < G.n * G.m; c += gridDim.x * blockDim.x)
        s += pint[c] * v[(c % G.n) * G.m + c / G.n];
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}
HD int atm_sk(const AtmGeo& G) { const int ck = (G.rowint - AQ) / ANUN; return (ck % G.n) * G.m + ck / G.n; }
/* pred[0..AR): I.w partials, [AR..2AR): I.g partials -> pred[2AR..2AR+4) = 2x2 inverse */
__global__ void k_atm_pschur(AtmPar P, AtmGeo G, const double* __restrict__ w, const double* __restrict__ g,
                             double* __restrict__ pred)
{
    if (threadIdx.x || blockIdx.x) return;
    double Iw = 0.0, Ig = 0.0;
    for (int q = 0; q < AR_BLOCKS; q++) Iw += pred[q];
    for (int q = 0; q < AR_BLOCKS; q++) Ig += pred[AR_BLOCKS + q];
    const int sk = atm_sk(G);
    const double rA = -1.0 / P.total_area;
    const double a11 = Iw - w[sk], a12 = (Ig - g[sk]) + 1.0;
    const double a21 = rA * Iw + 1.0, a22 = rA * Ig;
    const double det = a11 * a22 - a12 * a21;
    double* M = pred + 2 * AR_BLOCKS;
    M[0] = a22 / det; M[1] = -a12 / det; M[2] = -a21 / det; M[3] = a11 / det;
}
__global__ void k_atm_prec_a(AtmPar P, AtmGeo G, const double* __restrict__ val, const double* __restrict__ r,
                             const double* __restrict__ w, const double* __restrict__ g, const double* __restrict__ y,
                             const double* __restrict__ pred, double* __restrict__ z, double* __restrict__ bt)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    const int sc = (c % G.n) * G.m + c / G.n;
    double Iy = 0.0;
    for (int q = 0; q < AR_BLOCKS; q++) Iy += pred[2 * AR_BLOCKS + 4 + q];
    const double* M = pred + 2 * AR_BLOCKS;
    const double f1 = Iy - y[atm_sk(G)], f2 = (-1.0 / P.total_area) * Iy - r[G.rowP];
    const double zP = M[0] * f1 + M[1] * f2, mu = M[2] * f1 + M[3] * f2;
    z[ANUN * c + AQ] = y[sc] - w[sc] * zP - g[sc] * mu;
    const double* va = val + (size_t)(ANUN * c + AA) * ASL;
    const double zA = (r[ANUN * c + AA] - va[2] * zP) / va[1];
    z[ANUN * c + AA] = zA;
    const double* vt = val + (size_t)(ANUN * c + AT) * ASL;
    bt[sc] = r[ANUN * c + AT] - vt[3] * zA - vt[4] * zP;
    if (c == 0) z[G.rowP] = zP;
}
__global__ void k_atm_prec_b(AtmGeo G, const double* __restrict__ zt, const double* __restrict__ zq,
                             double* __restrict__ z)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= G.n * G.m) return;
    const int sc = (c % G.n) * G.m + c / G.n;
    z[ANUN * c + AT] = zt[sc];
    (void)zq;
}

/* ---- coupling (applied matrix-free) -------------------------------------------------- */
struct CplPar {
    int n, m, l;
    int ib0, jb0, nx, mb;  /* the ocean subdomain's owned columns / rows (Decomp2D)  */
    int64_t own0;          /* first owned ext cell of the ocean                    */
    double dTFQ;           /* nuq tdim/qdim dqso (1 - M)  (Atmosphere.C:547)        */
    double pfac;           /* (1/A)(tdim/qdim) dqso        (Atmosphere.C:596-597)   */
    double Ooa, aft, dqft; /* Ocean.C:1613-1627: Ooa, -comb sunp albed, lvsc eta qdim */
    int ct, cs;            /* coupled_T, coupled_S                                  */
    double nus;            /* Ocean.C:1639-1651: -dQFS = nus, -dPFS = nus Pd        */
    int64_t sint_row;      /* packed row of the ocean's integral condition, or -1   */
};

/* SST of the ocean state: T at (i, j, l-1) (Ocean::interfaceT -> Atmosphere::synchronize),
 * the subdomain's owned surface cells into the n*m surface (the other entries untouched:
 * on several ranks zeroed before and summed after) */
__global__ void k_sst(CplPar K, const double* __restrict__ xo_ext, double* __restrict__ sst)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= K.nx * K.mb) return;
    const int il = e % K.nx, jl = e / K.nx;
    const int64_t cell = ((int64_t)(jl + HALO) * K.l + (K.l - 1)) * K.nx + il;
    sst[(int64_t)(K.jb0 + jl) * K.n + K.ib0 + il] = xo_ext[NUN * cell + TT];
}
/* surface T of a packed ocean vector (owned rows) into the n*m surface, owned cells */
__global__ void k_surf_t(CplPar K, const double* __restrict__ xo_packed, double* __restrict__ out)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= K.nx * K.mb) return;
    const int il = e % K.nx, jl = e / K.nx;
    const int64_t lc = ((int64_t)jl * K.l + (K.l - 1)) * K.nx + il;
    out[(int64_t)(K.jb0 + jl) * K.n + K.ib0 + il] = xo_packed[NUN * lc + TT];
}
/* Atmosphere::interfaceT/Q/A/P (449-493, getP 1160-1225): the surface fields the ocean
 * needs; P dimensional, Pdist (Eo0 + eta qdim P) over water */
__global__ void k_atm_fields(AtmPar P, AtmGeo G, const double* __restrict__ xa, double* __restrict__ out, int nm)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nm) return;
    out[q] = xa[ANUN * q + AT];
    out[nm + q] = xa[ANUN * q + AQ];
    out[2 * nm + q] = xa[ANUN * q + AA];
    out[3 * nm + q] = G.surf[q] == 0 ? G.pdist[q] * (P.Eo0 + P.eta * P.qdim * xa[G.rowP]) : 0.0;
}

/* y_o(surface T rows) += C_oa x_a  (Ocean::getBlock(atmos): -dTFT, -dAFT, -dQFT; with
 * coupled_S the surface S rows: -dQFS, -dPFS) */
__global__ void k_cpl_oa(CplPar K, const int* __restrict__ surf, const double* __restrict__ suno,
                         const double* __restrict__ pdist, int rowP, const double* __restrict__ xa,
                         double* __restrict__ yo_packed)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= K.nx * K.mb) return;
    const int il = e % K.nx, jl = e / K.nx, j = K.jb0 + jl;
    const int q = j * K.n + K.ib0 + il;
    if (surf[q]) return;
    const int64_t lc = ((int64_t)jl * K.l + (K.l - 1)) * K.nx + il;   /* owned-local cell */
    const double S = suno[j + 1];
    const double dTFT = K.Ooa * (1.0 - 0.0);
    const double dAFT = K.aft * S * (1.0 - 0.0);
    const double dQFT = K.dqft * (1.0 - 0.0);
    if (K.ct) {
        double z = 0.0;
        z += -dTFT * xa[ANUN * q + AT];
        z += -dAFT * xa[ANUN * q + AA];
        z += -dQFT * xa[ANUN * q + AQ];
        yo_packed[NUN * lc + TT] += z;
    }
    if (K.cs && NUN * lc + SS != K.sint_row) {
        const double dQFS = -K.nus * (1.0 - 0.0);
        const double dPFS = -K.nus * pdist[q] * (1.0 - 0.0);
        double z = 0.0;
        z += -dQFS * xa[ANUN * q + AQ];
        z += -dPFS * xa[rowP];
        yo_packed[NUN * lc + SS] += z;
    }
}
/* surface T of cell q: from the gathered n*m surface (several ranks) or straight from the
 * packed ocean vector (one rank) */
__device__ __forceinline__ double surf_t(const CplPar& K, const double* __restrict__ tsurf,
                                         const double* __restrict__ xo_packed, int q)
{
    if (tsurf) return tsurf[q];
    const int i = q % K.n, j = q / K.n;
    return xo_packed[NUN * (((int64_t)j * K.l + (K.l - 1)) * K.n + i) + TT];
}
/* y_a += C_ao x_o on the T and q rows (Atmosphere::getBlock(ocean)) */
__global__ void k_cpl_ao(CplPar K, AtmGeo G, const double* __restrict__ tsurf, const double* __restrict__ xo_packed,
                         double* __restrict__ ya)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= K.n * K.m) return;
    if (G.surf[q]) return;
    const double t = surf_t(K, tsurf, xo_packed, q);
    if (ANUN * q + AT != G.rowint) ya[ANUN * q + AT] += (1.0 - 0.0) * t;
    if (ANUN * q + AQ != G.rowint) ya[ANUN * q + AQ] += K.dTFQ * t;
}
/* partials of sum_q intc_q T_o(q) (the precipitation row's SST dependence) */
__global__ void __launch_bounds__(256) k_cpl_pdot(CplPar K, const double* __restrict__ pint,
                                                  const double* __restrict__ tsurf,
                                                  const double* __restrict__ xo_packed, double* __restrict__ part)
{
    __shared__ double sm[256];
    double s = 0.0;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < K.n * K.m; q += gridDim.x * blockDim.x)
        s += pint[q] * surf_t(K, tsurf, xo_packed, q);
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}
__global__ void k_cpl_pfin(CplPar K, AtmGeo G, const double* __restrict__ part, double* __restrict__ ya, double sgn)
{
    if (threadIdx.x || blockIdx.x) return;
    double a = 0.0;
    for (int q = 0; q < AR_BLOCKS; q++) a += part[q];
    ya[G.rowP] += sgn * K.pfac * a;
}

/* ---- packed-vector Krylov kernels ------------------------------------------------------ */
constexpr int KB = 512;
/* part[v*KB + b] = partial of V_v . w (v < nv), part[nv*KB + b] = w . w */
__global__ void __launch_bounds__(256) k_cdots(const double* __restrict__ V, int64_t ld, int nv,
                                               const double* __restrict__ w, int64_t N, double* __restrict__ part)
{
    __shared__ double sm[256];
    const int v = blockIdx.y;
    const double* a = v < nv ? V + (int64_t)v * ld : w;
    double s = 0.0;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x)
        s += a[q] * w[q];
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(int64_t)v * KB + blockIdx.x] = sm[0];
}
__global__ void k_cfinal(const double* __restrict__ part, int nvec, double* __restrict__ out)
{
    __shared__ double sm[256];
    const int v = blockIdx.x;
    double s = 0.0;
    for (int q = threadIdx.x; q < KB; q += blockDim.x) s += part[(int64_t)v * KB + q];
    sm[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if (threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0 && v < nvec) out[v] = sm[0];
}
/* y = a*y + sum_v c_v X_v */
__global__ void k_cupdate(const double* __restrict__ X, int64_t ld, int nv, const double* __restrict__ c, double a,
                          double* __restrict__ y, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x) {
        double s = a * y[q];
        for (int v = 0; v < nv; v++) s += c[v] * X[(int64_t)v * ld + q];
        y[q] = s;
    }
}
/* y = a y + sum_i c_i X_i (i < nv <= 16) */
struct LinC {
    int nv;
    double a;
    double c[16];
    const double* X[16];
};
/* y may also be one of the X (IDR's U(:,k) update): no __restrict__ */
__global__ void __launch_bounds__(256) k_clincomb(LinC L, double* y, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x) {
        double acc = L.a == 0.0 ? 0.0 : L.a * y[q];
        for (int i = 0; i < L.nv; i++) acc += L.c[i] * L.X[i][q];
        y[q] = acc;
    }
}
/* two independent combinations in one pass (the paired IDR updates) */
__global__ void __launch_bounds__(256) k_clincomb2(LinC L1, double* y1, LinC L2, double* y2, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x) {
        double a1 = L1.a == 0.0 ? 0.0 : L1.a * y1[q];
        for (int i = 0; i < L1.nv; i++) a1 += L1.c[i] * L1.X[i][q];
        double a2 = L2.a == 0.0 ? 0.0 : L2.a * y2[q];
        for (int i = 0; i < L2.nv; i++) a2 += L2.c[i] * L2.X[i][q];
        y1[q] = a1;
        y2[q] = a2;
    }
}
/* IDR shadow space: uniform in [-1, 1] from splitmix64 over the packed row index */
__global__ void k_cidr_random(double* __restrict__ P, int64_t ld, int s, int64_t N)
{
    const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q0 >= N) return;
    for (int q = 0; q < s; q++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * ((uint64_t)q0 * 16 + (uint64_t)q + 1) + 20261017ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        P[(int64_t)q * ld + q0] = 2.0 * ((double)(z >> 11) * (1.0 / 9007199254740992.0)) - 1.0;
    }
}
__global__ void k_axpby_c(double a, const double* __restrict__ x, double b, const double* __restrict__ y,
                          double* __restrict__ out, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x)
        out[q] = a * x[q] + b * y[q];
}
__global__ void k_cscale(double s, const double* __restrict__ x, double* __restrict__ y, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x)
        y[q] = s * x[q];
}
/* y -= sum_v c_v X_v with the coefficients in device memory (CGS2 pass without a host trip) */
__global__ void k_cupdate_m(const double* __restrict__ X, int64_t ld, int nv, const double* __restrict__ c,
                            double* __restrict__ y, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x) {
        double s = y[q];
        for (int v = 0; v < nv; v++) s += -c[v] * X[(int64_t)v * ld + q];
        y[q] = s;
    }
}
/* y *= 1 / sqrt(nrm2) from the device-resident squared norm (unchanged when it is not > 0) */
__global__ void k_cscale_dev(const double* __restrict__ nrm2, double* __restrict__ y, int64_t N)
{
    const double n2 = *nrm2;
    if (!(n2 > 0.0)) return;
    const double s = 1.0 / sqrt(n2);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (int64_t)gridDim.x * blockDim.x)
        y[q] = s * y[q];
}

}  // namespace
}  // namespace iemic

/* ======================================================================================= */
namespace {

AtmGeo atm_geo(const iemic_atmos* a)
{
    return AtmGeo{a->n, a->m, a->periodic, a->dim, a->rowint, a->rowP, a->d_tab.p, a->d_pdist.p, a->d_surf.p};
}

void atm_set_nuq(iemic_atmos* a)
{
    AtmPar& P = a->P;
    P.nuq = P.comb * P.humf * (a->eta0 / a->hdimq) * (a->rhoo / a->rhoa) * (a->r0dim / a->udim);
}

unsigned blocks_for(int64_t N) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((N + 255) / 256, 4096)); }

int coupled_check(iemic_ctx* c)
{
    if (!c->cfg.coupled_t && !c->cfg.coupled_s) {
        set_error("coupled model: the ocean context needs coupled_t = 1 (or coupled_s = 1)");
        return IEMIC_EINVAL;
    }
    return 0;
}

}  // namespace

extern "C" int iemic_atmos_default_params(iemic_atmos_params* p)
{
    if (!p) return IEMIC_EINVAL;
    /* AtmosLocal::setParameters defaults (AtmosLocal.C:109-170) */
    *p = iemic_atmos_params{};
    p->rhoa = 1.25; p->rhoo = 1024; p->hdima = 8400.; p->hdimq = 1800.; p->cpa = 1000.;
    p->D0 = 3.1e+06; p->kappa = 1e+06; p->arad = 212.0; p->brad = 1.5; p->sun0 = 1360.;
    p->c0 = 0.43; p->ce = 1.3e-03; p->ch = 0.94 * 1.3e-03; p->uw = 8.5; p->t0a = 15.0; p->t0o = 15.0;
    p->t0i = -5.0; p->tdim = 1.0; p->q0 = 2e-3; p->qdim = 1e-3; p->lv = 2.5e06; p->udim = 0.1e+00;
    p->r0dim = 6.37e+06; p->a0 = 0.3; p->da = 0.5; p->tauf_days = 1.0; p->tauc_days = 1.0;
    p->Tm = 0.0; p->Tr = 1.0; p->Pa = 0.2; p->epm = 5.0; p->epr = 1.0; p->epa = 0.1;
    p->par[0] = 0.0; p->par[1] = 1.0; p->par[2] = 1.0; p->par[3] = 1.0; p->par[4] = 1.0;
    p->par[5] = 1.0; p->par[6] = 1.0;
    return 0;
}

extern "C" int iemic_atmos_create(iemic_atmos** out, iemic_ctx* oc, const iemic_atmos_params* prm)
{
    if (!out || !oc || !prm) return IEMIC_EINVAL;
    int rc = coupled_check(oc);
    if (rc) return rc;
    if (hipSetDevice(oc->device) != hipSuccess) return IEMIC_EDEVICE;
    iemic_atmos* a = new iemic_atmos();
    a->oc = oc;
    a->prm = *prm;
    const int n = oc->n, m = oc->m;
    a->n = n; a->m = m; a->periodic = oc->cfg.periodic;
    a->dim = ANUN * n * m + 1;
    a->rowP = a->dim - 1;
    a->rowint = ANUN * ((m - 1) * n + (n - 1)) + AQ;     /* Atmosphere.C:49-51 */
    /* surface mask: the ocean's effective mask at k = l (AtmosLocal::setSurfaceMask) */
    const host::Setup& su = oc->su;
    a->surf.assign((size_t)n * m, 0);
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++)
            a->surf[(size_t)j * n + i] = su.landm[((size_t)su.l * (m + 2) + (j + 1)) * (n + 2) + (i + 1)] != 0;
    /* parameters and coefficients (setParameters + setup) */
    AtmPar& P = a->P;
    const iemic_atmos_params& p = *prm;
    const double muoa = p.rhoa * p.ch * p.cpa * p.uw;
    P.amua = (p.arad + p.brad * p.t0a) / muoa;
    P.bmua = p.brad / muoa;
    P.Ad = p.rhoa * p.hdima * p.cpa * p.D0 / (muoa * p.r0dim * p.r0dim);
    const double As = p.sun0 * (1 - p.c0) / (4 * muoa);
    P.eta = (p.rhoa / p.rhoo) * p.ce * p.uw;
    a->eta0 = P.eta; a->hdimq = p.hdimq; a->rhoo = p.rhoo; a->rhoa = p.rhoa; a->r0dim = p.r0dim; a->udim = p.udim;
    P.Phv = p.kappa / (p.udim * p.r0dim);
    const double c1 = 3.8e-3, c2 = 21.87, c3 = 265.5, c4 = 17.67, c5 = 243.5;
    const double qso = c1 * std::exp(c4 * p.t0o / (p.t0o + c5));
    const double qsi = c1 * std::exp(c2 * p.t0i / (p.t0i + c3));
    P.Eo0 = P.eta * (qso - p.q0);
    P.Ei0 = P.eta * (qsi - p.q0);
    P.qdim = p.qdim; P.tdim = p.tdim;
    P.Cs = (P.Ei0 - P.Eo0) / P.eta / P.qdim;
    P.Po0 = P.Eo0;
    P.Tr = p.Tr - p.t0o;
    P.Tm = p.Tm - p.t0o;
    P.dqso = 5e-4;                                   /* AtmosLocal.C:233 */
    P.dqsi = (c1 * c2 * c3) / ((p.t0i + c3) * (p.t0i + c3));
    P.dqsi *= std::exp((c2 * p.t0i) / (p.t0i + c3));
    P.lvscale = p.rhoo * p.lv / muoa;
    P.a0 = p.a0; P.da = p.da;
    P.tauf = (p.tauf_days * 3600. * 24. * p.udim) / p.r0dim;
    P.tauc = (p.tauc_days * 3600. * 24. * p.udim) / p.r0dim;
    P.Pa = p.Pa; P.epm = p.epm; P.epr = p.epr; P.epa = p.epa; P.t0o = p.t0o; P.t0i = p.t0i;
    P.comb = p.par[0]; P.sunp = p.par[1]; P.lonf = p.par[2]; P.humf = p.par[3]; P.latf = p.par[4];
    P.albf = p.par[5]; P.tdif = p.par[6];
    P.Ooa = su.Ooa;                                  /* getdeps (AtmosLocal.C:249) */
    const double Os = su.Os;
    atm_set_nuq(a);
    /* grid and per-latitude tables (setup 341-371, discretize 1162-1232) */
    const double xmin = oc->cfg.xmin * PI_ / 180.0, xmax = oc->cfg.xmax * PI_ / 180.0;
    const double ymin = oc->cfg.ymin * PI_ / 180.0, ymax = oc->cfg.ymax * PI_ / 180.0;
    const double dx = (xmax - xmin) / n, dy = (ymax - ymin) / m;
    const int M1 = m + 1;
    std::vector<double> yc(M1), yv(M1), datv(M1);
    for (int j = 0; j < M1; j++) {
        yc[j] = ymin + (j - 0.5) * dy;
        yv[j] = ymin + j * dy;
        datv[j] = 0.9 + 1.5 * std::exp(-12 * yv[j] * yv[j] / PI_);
    }
    a->tab.assign((size_t)8 * M1, 0.0);
    const double dy2i = 1.0 / (dy * dy);   /* pow(v, 2) of the reference: v*v */
    for (int j = 1; j <= m; j++) {
        const double datc = 0.9 + 1.5 * std::exp(-12 * yc[j] * yc[j] / PI_);
        const double cdx = std::cos(yc[j]) * dx;
        const double cosdx2i = 1.0 / (cdx * cdx);
        const double cyc = std::cos(yc[j]);
        a->tab[j] = datc * cosdx2i;
        a->tab[M1 + j] = dy2i * datv[j - 1] * std::cos(yv[j - 1]) / cyc;
        a->tab[2 * M1 + j] = dy2i * datv[j] * std::cos(yv[j]) / cyc;
        a->tab[3 * M1 + j] = cosdx2i;
        a->tab[4 * M1 + j] = dy2i * std::cos(yv[j - 1]) / cyc;
        a->tab[5 * M1 + j] = dy2i * std::cos(yv[j]) / cyc;
        const double sy = std::sin(yc[j]);
        a->tab[6 * M1 + j] = As * (1 - .482 * (3 * (sy * sy) - 1.) / 2.);
        a->tab[7 * M1 + j] = Os * (1 - .482 * (3 * (sy * sy) - 1.) / 2.);
    }
    /* integral coefficients and the precipitation distribution (setupIntCoeff, setPdist) */
    a->pint.assign((size_t)n * m, 0.0);
    std::vector<double> pd((size_t)n * m, 0.0);
    double total = 0.0;
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++)
            if (!a->surf[(size_t)j * n + i]) a->pint[(size_t)j * n + i] = std::cos(yc[j + 1]) * dx * dy;
    for (double v : a->pint) total += std::fabs(v);
    P.total_area = total;
    for (int j = 1; j <= m; j++) {
        const double y = yc[j];
        const double s2 = std::sin(2.0 * y);
        const double v = 2 * std::exp(-((6 * y) * (6 * y))) + s2 * s2;
        for (int i = 0; i < n; i++)
            if (!a->surf[(size_t)(j - 1) * n + i]) pd[(size_t)(j - 1) * n + i] = v;
    }
    double ipd = 0.0;
    for (size_t q = 0; q < pd.size(); q++) ipd += a->pint[q] * pd[q];
    const double corr = 1 - ipd / total;
    a->pdist.assign((size_t)n * m, 0.0);
    for (size_t q = 0; q < pd.size(); q++)
        a->pdist[q] = corr * (std::fabs(a->pint[q]) > 1e-7 ? 1.0 : 0.0) + pd[q];
    /* device buffers */
    rc = 0;
    rc |= a->d_tab.alloc(a->tab.size());
    rc |= a->d_pdist.alloc((size_t)n * m);
    rc |= a->d_pint.alloc((size_t)n * m);
    rc |= a->d_surf.alloc((size_t)n * m);
    rc |= a->d_x.alloc(a->dim);
    rc |= a->d_sst.alloc((size_t)n * m);
    rc |= a->d_F.alloc(a->dim);
    rc |= a->d_y.alloc(a->dim);
    rc |= a->d_val.alloc((size_t)(a->dim - 1) * ASL);
    rc |= a->d_col.alloc((size_t)(a->dim - 1) * ASL);
    rc |= a->d_red.alloc(4 * AR_BLOCKS);
    rc |= a->d_tmp.alloc((size_t)3 * n * m + a->dim);
    rc |= a->d_s9t.alloc((size_t)9 * n * m);
    rc |= a->d_s9q.alloc((size_t)9 * n * m);
    rc |= a->d_bt.alloc((size_t)n * m);
    rc |= a->d_bq.alloc((size_t)n * m);
    rc |= a->d_zt.alloc((size_t)n * m);
    rc |= a->d_zq.alloc((size_t)n * m);
    rc |= a->d_colij.alloc((size_t)n * m);
    rc |= a->d_w.alloc((size_t)n * m);
    rc |= a->d_g.alloc((size_t)n * m);
    rc |= a->d_pred.alloc((size_t)3 * AR_BLOCKS + 8);
    if (rc) {
        delete a;
        set_error("iemic_atmos_create: out of device memory");
        return IEMIC_ENOMEM;
    }
    std::vector<int> colij((size_t)n * m);
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++) colij[(size_t)j * n + i] = i * m + j;
    rc = h2d(oc, a->d_tab.p, a->tab.data(), sizeof(double) * a->tab.size());
    if (!rc) rc = h2d(oc, a->d_pdist.p, a->pdist.data(), sizeof(double) * n * m);
    if (!rc) rc = h2d(oc, a->d_pint.p, a->pint.data(), sizeof(double) * n * m);
    if (!rc) rc = h2d(oc, a->d_surf.p, a->surf.data(), sizeof(int) * n * m);
    if (!rc) rc = h2d(oc, a->d_colij.p, colij.data(), sizeof(int) * n * m);
    if (!rc) rc = cr_init(oc, a->crT, n, m, a->periodic);
    if (!rc) rc = cr_init(oc, a->crQ, n, m, a->periodic);
    if (rc) {
        delete a;
        return rc;
    }
    (void)hipMemsetAsync(a->d_x.p, 0, sizeof(double) * a->dim, oc->stream);
    (void)hipMemsetAsync(a->d_sst.p, 0, sizeof(double) * n * m, oc->stream);
    (void)hipStreamSynchronize(oc->stream);
    oc->refs++;
    *out = a;
    return 0;
}

/* the atmosphere lives on while a coupled model built on it exists; its last reference
 * releases the ocean context's */
static void atmos_release(iemic_atmos* a)
{
    if (!a || --a->refs > 0) return;
    iemic_ctx* oc = a->oc;
    (void)hipSetDevice(oc->device);
    (void)hipStreamSynchronize(oc->stream);
    delete a;
    ctx_release(oc);
}

extern "C" void iemic_atmos_destroy(iemic_atmos* a) { atmos_release(a); }

extern "C" int iemic_atmos_dim(const iemic_atmos* a) { return a ? a->dim : -1; }

/* AtmosLocal::setPar (1654-1677): 0 Combined, 1 Solar, 2 Longwave, 3 Humidity,
 * 4 Latent Heat, 5 Albedo Forcing, 6 T Eddy Diffusivity */
extern "C" int iemic_atmos_set_par(iemic_atmos* a, int idx, double v)
{
    if (!a || idx < 0 || idx > 6) return IEMIC_EINVAL;
    double* slot[7] = {&a->P.comb, &a->P.sunp, &a->P.lonf, &a->P.humf, &a->P.latf, &a->P.albf, &a->P.tdif};
    *slot[idx] = v;
    atm_set_nuq(a);
    a->jac_valid = a->prec_valid = 0;
    return 0;
}

extern "C" int iemic_atmos_set_state(iemic_atmos* a, const double* x)
{
    if (!a || !x) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    a->jac_valid = 0;
    return h2d(a->oc, a->d_x.p, x, sizeof(double) * a->dim);
}
extern "C" int iemic_atmos_get_state(iemic_atmos* a, double* x)
{
    if (!a || !x) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    return d2h(a->oc, x, a->d_x.p, sizeof(double) * a->dim);
}
/* Atmosphere::setOceanTemperature (796-814): n*m surface vector */
extern "C" int iemic_atmos_set_sst(iemic_atmos* a, const double* sst)
{
    if (!a || !sst) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    return h2d(a->oc, a->d_sst.p, sst, sizeof(double) * a->n * a->m);
}

namespace {
int atm_rhs_dev(iemic_atmos* a)
{
    hipStream_t s = a->oc->stream;
    const AtmGeo G = atm_geo(a);
    const int nm = a->n * a->m;
    hipLaunchKernelGGL(k_atm_rhs, dim3((nm + 127) / 128), dim3(128), 0, s, a->P, G, (const double*)a->d_x.p,
                       (const double*)a->d_sst.p, a->d_F.p);
    double* sig = a->d_tmp.p;
    hipLaunchKernelGGL(k_atm_sigma, dim3((nm + 255) / 256), dim3(256), 0, s, a->P, (const double*)a->d_sst.p, sig, nm);
    /* intc . x over the q unknowns: intc_q = pint at the q rows (integralCoeff, nun = 3) */
    hipLaunchKernelGGL(k_atm_wdot, dim3(AR_BLOCKS), dim3(256), 0, s, (const double*)a->d_pint.p,
                       (const double*)a->d_x.p, ANUN, AQ, nm, a->d_red.p);
    hipLaunchKernelGGL(k_atm_wdot, dim3(AR_BLOCKS), dim3(256), 0, s, (const double*)a->d_pint.p, (const double*)sig,
                       1, 0, nm, a->d_red.p + AR_BLOCKS);
    hipLaunchKernelGGL(k_atm_rhs_dense, dim3(1), dim3(64), 0, s, a->P, G, (const double*)a->d_x.p,
                       (const double*)a->d_red.p, a->d_F.p);
    HIP_OK(hipGetLastError());
    return 0;
}
int atm_jac_dev(iemic_atmos* a)
{
    const int nm = a->n * a->m;
    hipLaunchKernelGGL(k_atm_jac, dim3((nm + 127) / 128), dim3(128), 0, a->oc->stream, a->P, atm_geo(a),
                       (const double*)a->d_x.p, a->d_val.p, a->d_col.p);
    HIP_OK(hipGetLastError());
    a->jac_valid = 1;
    a->prec_valid = 0;
    return 0;
}
/* y = J_a x (device vectors of length dim) */
int atm_spmv_dev(iemic_atmos* a, const double* x, double* y)
{
    hipStream_t s = a->oc->stream;
    const int nm = a->n * a->m, nrow = a->dim - 1;
    hipLaunchKernelGGL(k_atm_spmv, dim3((nrow + 255) / 256), dim3(256), 0, s, (const double*)a->d_val.p,
                       (const int*)a->d_col.p, x, y, nrow);
    hipLaunchKernelGGL(k_atm_wdot, dim3(AR_BLOCKS), dim3(256), 0, s, (const double*)a->d_pint.p, x, ANUN, AQ, nm,
                       a->d_red.p + 2 * AR_BLOCKS);
    hipLaunchKernelGGL(k_atm_spmv_dense, dim3(1), dim3(64), 0, s, a->P, atm_geo(a), x,
                       (const double*)a->d_red.p + 2 * AR_BLOCKS, y);
    HIP_OK(hipGetLastError());
    return 0;
}
int atm_prec_compute(iemic_atmos* a)
{
    const int nm = a->n * a->m;
    hipStream_t s = a->oc->stream;
    hipLaunchKernelGGL(k_atm_s9, dim3((nm + 255) / 256), dim3(256), 0, s, atm_geo(a), (const double*)a->d_val.p,
                       a->d_s9t.p, a->d_s9q.p);
    int rc = cr_factor(a->oc, a->crT, a->d_s9t.p, a->d_colij.p);
    if (!rc) rc = cr_factor(a->oc, a->crQ, a->d_s9q.p, a->d_colij.p);
    if (!rc) rc = cr_check(a->oc, a->crT);
    if (!rc) rc = cr_check(a->oc, a->crQ);
    if (rc) return rc;
    /* the bordered [q; P] block: w = S~^-1 c, g = S~^-1 e_k and the 2x2 inverse */
    const AtmGeo G = atm_geo(a);
    hipLaunchKernelGGL(k_atm_qcol, dim3((nm + 255) / 256), dim3(256), 0, s, G, (const double*)a->d_val.p,
                       (const double*)nullptr, a->d_bq.p, a->d_bt.p, (double*)nullptr);
    if ((rc = cr_solve(a->oc, a->crQ, a->d_bq.p, a->d_w.p, s))) return rc;
    if ((rc = cr_solve(a->oc, a->crQ, a->d_bt.p, a->d_g.p, s))) return rc;
    hipLaunchKernelGGL(k_atm_pdot_sc, dim3(AR_BLOCKS), dim3(256), 0, s, G, (const double*)a->d_pint.p,
                       (const double*)a->d_w.p, a->d_pred.p);
    hipLaunchKernelGGL(k_atm_pdot_sc, dim3(AR_BLOCKS), dim3(256), 0, s, G, (const double*)a->d_pint.p,
                       (const double*)a->d_g.p, a->d_pred.p + AR_BLOCKS);
    hipLaunchKernelGGL(k_atm_pschur, dim3(1), dim3(64), 0, s, a->P, G, (const double*)a->d_w.p,
                       (const double*)a->d_g.p, a->d_pred.p);
    HIP_OK(hipGetLastError());
    a->prec_valid = 1;
    return 0;
}
int atm_prec_apply(iemic_atmos* a, const double* r, double* z)
{
    const int nm = a->n * a->m;
    hipStream_t s = a->oc->stream;
    const AtmGeo G = atm_geo(a);
    const unsigned gb = (nm + 255) / 256;
    hipLaunchKernelGGL(k_atm_qcol, dim3(gb), dim3(256), 0, s, G, (const double*)a->d_val.p, r, (double*)nullptr,
                       (double*)nullptr, a->d_bq.p);
    int rc = cr_solve(a->oc, a->crQ, a->d_bq.p, a->d_zq.p, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_atm_pdot_sc, dim3(AR_BLOCKS), dim3(256), 0, s, G, (const double*)a->d_pint.p,
                       (const double*)a->d_zq.p, a->d_pred.p + 2 * AR_BLOCKS + 4);
    hipLaunchKernelGGL(k_atm_prec_a, dim3(gb), dim3(256), 0, s, a->P, G, (const double*)a->d_val.p, r,
                       (const double*)a->d_w.p, (const double*)a->d_g.p, (const double*)a->d_zq.p,
                       (const double*)a->d_pred.p, z, a->d_bt.p);
    if ((rc = cr_solve(a->oc, a->crT, a->d_bt.p, a->d_zt.p, s))) return rc;
    hipLaunchKernelGGL(k_atm_prec_b, dim3(gb), dim3(256), 0, s, G, (const double*)a->d_zt.p,
                       (const double*)a->d_zq.p, z);
    HIP_OK(hipGetLastError());
    return 0;
}
}  // namespace

/* Atmosphere::computeRHS (266-393); F may be null (kept on the device) */
extern "C" int iemic_atmos_rhs(iemic_atmos* a, double* F)
{
    if (!a) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    int rc = atm_rhs_dev(a);
    if (rc) return rc;
    if (F) return d2h(a->oc, F, a->d_F.p, sizeof(double) * a->dim);
    DEV_SYNC(a->oc);
    return 0;
}
/* Atmosphere::computeJacobian (911-1126) */
extern "C" int iemic_atmos_jacobian(iemic_atmos* a)
{
    if (!a) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    int rc = atm_jac_dev(a);
    if (rc) return rc;
    DEV_SYNC(a->oc);
    return 0;
}
/* the local rows as ELL (dim-1 rows x 7: values, columns, -1 unused); the dense q-integral
 * and precipitation rows are defined by iemic_atmos_integral_coeff */
extern "C" int iemic_atmos_export_ell(iemic_atmos* a, double* val, int* col)
{
    if (!a || !val || !col) return IEMIC_EINVAL;
    if (!a->jac_valid) return IEMIC_ESTATE;
    const size_t ne = (size_t)(a->dim - 1) * ASL;
    int rc = d2h(a->oc, val, a->d_val.p, sizeof(double) * ne);
    if (!rc) rc = d2h(a->oc, col, a->d_col.p, sizeof(int) * ne);
    return rc;
}
/* pint (n*m, the q-integral weights cos(y) dx dy of ocean cells), total area, rowint, rowP */
extern "C" int iemic_atmos_integral_coeff(iemic_atmos* a, double* pint, double* total_area, int* rowint,
                                          int* rowP)
{
    if (!a) return IEMIC_EINVAL;
    if (pint) std::copy(a->pint.begin(), a->pint.end(), pint);
    if (total_area) *total_area = a->P.total_area;
    if (rowint) *rowint = a->rowint;
    if (rowP) *rowP = a->rowP;
    return 0;
}
/* AtmosLocal::getCommPars (537-557) */
extern "C" int iemic_atmos_commpars(iemic_atmos* a, double* out18)
{
    if (!a || !out18) return IEMIC_EINVAL;
    const AtmPar& P = a->P;
    const double v[18] = {P.tdim, P.qdim, P.nuq, P.eta, P.dqso, P.dqsi, P.nuq * P.tdim / P.qdim * P.dqso,
                          P.Eo0, P.Ei0, P.Cs, P.t0o, P.t0i, P.a0, P.da, P.tauf, P.tauc, P.comb, P.albf};
    for (int i = 0; i < 18; i++) out18[i] = v[i];
    return 0;
}
/* Atmosphere::getPdist, n*m */
extern "C" int iemic_atmos_pdist(iemic_atmos* a, double* out)
{
    if (!a || !out) return IEMIC_EINVAL;
    std::copy(a->pdist.begin(), a->pdist.end(), out);
    return 0;
}
extern "C" int iemic_atmos_spmv(iemic_atmos* a, const double* x, double* y)
{
    if (!a || !x || !y) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    if (!a->jac_valid) return IEMIC_ESTATE;
    double* dx = a->d_tmp.p;                      /* dim <= tmp size */
    int rc = h2d(a->oc, dx, x, sizeof(double) * a->dim);
    if (!rc) rc = atm_spmv_dev(a, dx, a->d_y.p);
    if (!rc) rc = d2h(a->oc, y, a->d_y.p, sizeof(double) * a->dim);
    return rc;
}
extern "C" int iemic_atmos_prec_apply(iemic_atmos* a, const double* r, double* z)
{
    if (!a || !r || !z) return IEMIC_EINVAL;
    if (hipSetDevice(a->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    if (!a->jac_valid) return IEMIC_ESTATE;
    int rc = a->prec_valid ? 0 : atm_prec_compute(a);
    if (rc) return rc;
    DevBuf<double> dr, dz;
    if (dr.alloc(a->dim) || dz.alloc(a->dim)) return IEMIC_ENOMEM;
    rc = h2d(a->oc, dr.p, r, sizeof(double) * a->dim);
    if (!rc) rc = atm_prec_apply(a, dr.p, dz.p);
    if (!rc) rc = d2h(a->oc, z, dz.p, sizeof(double) * a->dim);
    return rc;
}

/* =========================== coupled model ============================================ */
namespace {
CplPar cpl_par(const iemic_coupled* cm)
{
    const iemic_ctx* oc = cm->oc;
    const iemic_atmos* a = cm->at;
    const host::Setup& su = oc->su;
    CplPar K{};
    K.n = oc->n; K.m = oc->m; K.l = oc->l;
    K.ib0 = oc->ib0; K.jb0 = oc->jb0; K.nx = oc->nx; K.mb = oc->jb1 - oc->jb0;
    K.own0 = oc->own0;
    const AtmPar& P = a->P;
    K.dTFQ = P.nuq * P.tdim / P.qdim * P.dqso * (1.0 - 0.0);
    K.pfac = (1.0 / P.total_area) * (P.tdim / P.qdim) * P.dqso * (1.0 - 0.0);
    K.Ooa = su.Ooa;
    K.aft = -su.par[P_COMB] * su.par[P_SUNP] * P.da;
    K.dqft = su.lvsc * su.eta_a * su.qdim_a;
    K.ct = oc->cfg.coupled_t;
    K.cs = oc->cfg.coupled_s;
    K.nus = su.nus;
    K.sint_row = oc->rowintcon >= 0 ? oc->rowintcon - NUN * oc->own0 : -1;
    return K;
}

/* CoupledModel::synchronize (218-233): ocean <- atmosphere fields + CommPars
 * (Ocean::synchronize(atmos)), atmosphere <- SST (Atmosphere::synchronize(ocean)) */
int cpl_sync(iemic_coupled* cm)
{
    iemic_ctx* oc = cm->oc;
    iemic_atmos* a = cm->at;
    const int nm = a->n * a->m;
    hipStream_t s = oc->stream;
    hipLaunchKernelGGL(k_atm_fields, dim3((nm + 255) / 256), dim3(256), 0, s, a->P, atm_geo(a), (const double*)a->d_x.p,
                       oc->d_atm.p, nm);
    double pars[18];
    iemic_atmos_commpars(a, pars);
    /* the ocean Jacobian depends on the CommPars only through lin's latent-heat term */
    if (!cm->synced || !std::equal(pars, pars + 18, cm->pars)) oc->jac_valid = 0;
    std::copy(pars, pars + 18, cm->pars);
    cm->synced = 1;
    oc->su.set_atmos(pars);
    int rc = compute_forcing(oc);
    if (rc) return rc;
    /* the atmosphere (replicated on every rank) sees the whole surface: each rank writes its
     * owned cells, the sum over the ranks fills the rest */
    if (oc->nranks > 1) HIP_OK(hipMemsetAsync(a->d_sst.p, 0, sizeof(double) * nm, s));
    hipLaunchKernelGGL(k_sst, dim3((nm + 255) / 256), dim3(256), 0, s, cpl_par(cm), (const double*)oc->d_x.p,
                       a->d_sst.p);
    HIP_OK(hipGetLastError());
    if (oc->nranks > 1 && (rc = allreduce_sum(oc, a->d_sst.p, nm))) return rc;
    return 0;
}

/* the surface T of a packed ocean vector for the atmosphere rows: null on one rank (the
 * coupling kernels read the vector), else the n*m surface summed over the ranks */
int cpl_surf(iemic_coupled* cm, const double* xo_packed, const double** tsurf)
{
    iemic_ctx* oc = cm->oc;
    *tsurf = nullptr;
    if (oc->nranks <= 1) return 0;
    const int nm = oc->n * oc->m;
    hipStream_t s = oc->stream;
    double* t = cm->tsurf.p;
    HIP_OK(hipMemsetAsync(t, 0, sizeof(double) * nm, s));
    hipLaunchKernelGGL(k_surf_t, dim3((nm + 255) / 256), dim3(256), 0, s, cpl_par(cm), xo_packed, t);
    HIP_OK(hipGetLastError());
    int rc = allreduce_sum(oc, t, nm);
    if (rc) return rc;
    *tsurf = t;
    return 0;
}

/* y = [J_o C_oa; C_ao J_a] x on packed vectors [ocean owned rows | atmosphere] */
int cpl_apply(iemic_coupled* cm, const double* x, double* y)
{
    iemic_ctx* oc = cm->oc;
    iemic_atmos* a = cm->at;
    hipStream_t s = oc->stream;
    const int64_t o = NUN * oc->own0, NL = cm->NL;
    const int nm = a->n * a->m;
    const CplPar K = cpl_par(cm);
    HIP_OK(hipMemcpyAsync(cm->xo.p + o, x, sizeof(double) * NL, hipMemcpyDeviceToDevice, s));
    int rc = spmv(oc, cm->xo.p, cm->yo.p, s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(y, cm->yo.p + o, sizeof(double) * NL, hipMemcpyDeviceToDevice, s));
    if ((rc = atm_spmv_dev(a, x + NL, y + NL))) return rc;
    hipLaunchKernelGGL(k_cpl_oa, dim3((nm + 255) / 256), dim3(256), 0, s, K, (const int*)a->d_surf.p,
                       (const double*)(oc->d_tab.p + 9 * (oc->m + 2) + 2 * (oc->l + 2)), (const double*)a->d_pdist.p,
                       a->rowP, x + NL, y);
    const double* ts = nullptr;
    if ((rc = cpl_surf(cm, x, &ts))) return rc;
    hipLaunchKernelGGL(k_cpl_ao, dim3((nm + 255) / 256), dim3(256), 0, s, K, atm_geo(a), ts, x, y + NL);
    hipLaunchKernelGGL(k_cpl_pdot, dim3(AR_BLOCKS), dim3(256), 0, s, K, (const double*)a->d_pint.p, ts, x,
                       a->d_red.p + 3 * AR_BLOCKS);
    hipLaunchKernelGGL(k_cpl_pfin, dim3(1), dim3(64), 0, s, K, atm_geo(a), (const double*)a->d_red.p + 3 * AR_BLOCKS,
                       y + NL, 1.0);
    HIP_OK(hipGetLastError());
    return 0;
}

/* forward block Gauss-Seidel (CoupledModel.C:544-585, 'F'): z_o = M_o^-1 r_o;
 * z_a = M_a^-1 (r_a - C_ao z_o) */
int cpl_prec(iemic_coupled* cm, const double* r, double* z, int use_prec)
{
    iemic_ctx* oc = cm->oc;
    iemic_atmos* a = cm->at;
    hipStream_t s = oc->stream;
    const int64_t o = NUN * oc->own0, NL = cm->NL, NA = cm->NA;
    const int nm = a->n * a->m;
    if (!use_prec) {
        HIP_OK(hipMemcpyAsync(z, r, sizeof(double) * (NL + NA), hipMemcpyDeviceToDevice, s));
        return 0;
    }
    HIP_OK(hipMemcpyAsync(cm->ro.p + o, r, sizeof(double) * NL, hipMemcpyDeviceToDevice, s));
    int rc = prec_apply(oc, cm->ro.p, cm->zo.p);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(z, cm->zo.p + o, sizeof(double) * NL, hipMemcpyDeviceToDevice, s));
    /* b_a = r_a - C_ao z_o */
    double* b = cm->tmpa.p;
    HIP_OK(hipMemsetAsync(b, 0, sizeof(double) * NA, s));
    const CplPar K = cpl_par(cm);
    const double* ts = nullptr;
    if ((rc = cpl_surf(cm, z, &ts))) return rc;
    hipLaunchKernelGGL(k_cpl_ao, dim3((nm + 255) / 256), dim3(256), 0, s, K, atm_geo(a), ts, (const double*)z, b);
    hipLaunchKernelGGL(k_cpl_pdot, dim3(AR_BLOCKS), dim3(256), 0, s, K, (const double*)a->d_pint.p, ts,
                       (const double*)z, a->d_red.p + 3 * AR_BLOCKS);
    hipLaunchKernelGGL(k_cpl_pfin, dim3(1), dim3(64), 0, s, K, atm_geo(a), (const double*)a->d_red.p + 3 * AR_BLOCKS,
                       b, 1.0);
    hipLaunchKernelGGL(k_axpby_c, dim3(blocks_for(NA)), dim3(256), 0, s, 1.0, r + NL, -1.0, (const double*)b, b, NA);
    if ((rc = atm_prec_apply(a, b, z + NL))) return rc;
    HIP_OK(hipGetLastError());
    return 0;
}
}  // namespace

extern "C" int iemic_coupled_create(iemic_coupled** out, iemic_ctx* oc, iemic_atmos* a)
{
    if (!out || !oc || !a || a->oc != oc) return IEMIC_EINVAL;
    int rc = coupled_check(oc);
    if (rc) return rc;
    if (hipSetDevice(oc->device) != hipSuccess) return IEMIC_EDEVICE;
    iemic_coupled* cm = new iemic_coupled();
    cm->oc = oc;
    cm->at = a;
    cm->NL = oc->nlrows;
    cm->NA = a->dim;
    cm->NC = cm->NL + cm->NA;
    const int64_t NE = oc->nerows;
    rc = 0;
    rc |= cm->xo.alloc(NE);
    rc |= cm->yo.alloc(NE);
    rc |= cm->ro.alloc(NE);
    rc |= cm->zo.alloc(NE);
    rc |= cm->tmpa.alloc(cm->NA);
    rc |= cm->tsurf.alloc((size_t)oc->n * oc->m);
    rc |= cm->w.alloc(cm->NC);
    rc |= cm->r.alloc(cm->NC);
    rc |= cm->part.alloc((size_t)KB * (MAX_KRYLOV + 2));
    rc |= cm->hb.alloc((size_t)2 * MAX_KRYLOV + 8);
    rc |= cm->hc.alloc((size_t)2 * (2 * MAX_KRYLOV + 8));
    for (hipEvent_t& e : cm->ev)
        if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = 1;
    if (!rc && hipHostMalloc(&cm->h_red, sizeof(double) * 2 * (2 * MAX_KRYLOV + 8)) != hipSuccess) rc = 1;
    if (rc) {
        delete cm;
        set_error("iemic_coupled_create: out of device memory");
        return IEMIC_ENOMEM;
    }
    for (DevBuf<double>* b : {&cm->xo, &cm->yo, &cm->ro, &cm->zo})
        (void)hipMemsetAsync(b->p, 0, sizeof(double) * b->n, oc->stream);
    (void)hipStreamSynchronize(oc->stream);
    oc->refs++;
    a->refs++;
    *out = cm;
    return 0;
}

extern "C" void iemic_coupled_destroy(iemic_coupled* cm)
{
    if (!cm) return;
    iemic_ctx* oc = cm->oc;
    iemic_atmos* a = cm->at;
    (void)hipSetDevice(oc->device);
    (void)hipStreamSynchronize(oc->stream);
    delete cm;
    atmos_release(a);
    ctx_release(oc);
}

extern "C" int iemic_coupled_synchronize(iemic_coupled* cm)
{
    if (!cm) return IEMIC_EINVAL;
    if (hipSetDevice(cm->oc->device) != hipSuccess) return IEMIC_EDEVICE;
    int rc = cpl_sync(cm);
    if (rc) return rc;
    DEV_SYNC(cm->oc);
    return 0;
}

/* CoupledModel::computeRHS (260-271): synchronize, then each model's F (device copies
 * stay in the contexts; host copies if pointers are given: ocean in reference order) */
extern "C" int iemic_coupled_rhs(iemic_coupled* cm, double* F_ocean, double* F_atmos)
{
    if (!cm) return IEMIC_EINVAL;
    int rc = iemic_coupled_synchronize(cm);
    if (!rc) rc = iemic_rhs(cm->oc, F_ocean);
    if (!rc) rc = iemic_atmos_rhs(cm->at, F_atmos);
    return rc;
}

/* CoupledModel::computeJacobian (236-257): synchronize, each model's Jacobian; the
 * coupling blocks are applied matrix-free from the synchronized parameters */
extern "C" int iemic_coupled_jacobian(iemic_coupled* cm)
{
    if (!cm) return IEMIC_EINVAL;
    int rc = iemic_coupled_synchronize(cm);
    if (!rc) rc = iemic_jacobian(cm->oc);
    if (!rc) rc = iemic_atmos_jacobian(cm->at);
    return rc;
}

/* CoupledModel::applyMatrix (436-470) on host vectors [ocean (reference order) | atmosphere] */
extern "C" int iemic_coupled_spmv(iemic_coupled* cm, const double* x, double* y)
{
    if (!cm || !x || !y) return IEMIC_EINVAL;
    iemic_ctx* oc = cm->oc;
    if (hipSetDevice(oc->device) != hipSuccess) return IEMIC_EDEVICE;
    if (!oc->jac_valid || !cm->at->jac_valid) {
        set_error("iemic_coupled_spmv: no Jacobian assembled");
        return IEMIC_ESTATE;
    }
    const int64_t NL = cm->NL, NA = cm->NA, o = NUN * oc->own0;
    std::vector<double> ext((size_t)oc->nerows, 0.0), packed((size_t)(NL + NA));
    oc->su.ref_to_ext(x, ext.data());
    std::copy(ext.begin() + o, ext.begin() + o + NL, packed.begin());
    std::copy(x + oc->nrows, x + oc->nrows + NA, packed.begin() + NL);
    DevBuf<double> dx, dy;
    if (dx.alloc(NL + NA) || dy.alloc(NL + NA)) return IEMIC_ENOMEM;
    int rc = h2d(oc, dx.p, packed.data(), sizeof(double) * (NL + NA));
    if (!rc) rc = cpl_apply(cm, dx.p, dy.p);
    if (!rc) rc = d2h(oc, packed.data(), dy.p, sizeof(double) * (NL + NA));
    if (rc) return rc;
    std::copy(packed.begin(), packed.begin() + NL, ext.begin() + o);
    oc->su.ext_to_ref(ext.data(), y);
    std::copy(packed.begin() + NL, packed.end(), y + oc->nrows);
    return 0;
}

namespace {
/* dots of packed vectors: the ocean's owned rows on every rank, the (replicated) atmosphere
 * on rank 0 only, summed over the ranks -- the same values on every rank */
double cdot_host(iemic_coupled* cm, const double* V, int64_t ld, int nv, const double* w, double* out)
{
    hipStream_t s = cm->oc->stream;
    const int64_t N = cm->oc->rank == 0 ? cm->NC : cm->NL;
    hipLaunchKernelGGL(k_cdots, dim3(KB, nv + 1), dim3(256), 0, s, V, ld, nv, w, N, cm->part.p);
    hipLaunchKernelGGL(k_cfinal, dim3(nv + 1), dim3(256), 0, s, (const double*)cm->part.p, nv + 1, cm->hb.p);
    if (cm->oc->nranks > 1 && allreduce_sum(cm->oc, cm->hb.p, nv + 1)) {
        for (int i = 0; i <= nv; i++) out[i] = std::nan("");
        return out[nv];
    }
    (void)hipMemcpyAsync(cm->h_red, cm->hb.p, sizeof(double) * (nv + 1), hipMemcpyDeviceToHost, s);
    if (dev_wait(cm->oc, nullptr, "coupled dots")) {
        for (int i = 0; i <= nv; i++) out[i] = std::nan("");
        return out[nv];
    }
    for (int i = 0; i <= nv; i++) out[i] = cm->h_red[i];
    return out[nv];
}
}  // namespace

namespace {
/* cdot_host's reduction left on the device: out[0..nv] (summed over the ranks) */
int cdot_dev(iemic_coupled* cm, const double* V, int64_t ld, int nv, const double* w, double* out)
{
    hipStream_t s = cm->oc->stream;
    const int64_t N = cm->oc->rank == 0 ? cm->NC : cm->NL;
    hipLaunchKernelGGL(k_cdots, dim3(KB, nv + 1), dim3(256), 0, s, V, ld, nv, w, N, cm->part.p);
    hipLaunchKernelGGL(k_cfinal, dim3(nv + 1), dim3(256), 0, s, (const double*)cm->part.p, nv + 1, out);
    if (cm->oc->nranks > 1) return allreduce_sum(cm->oc, out, nv + 1);
    return 0;
}

LinC make_linc(double a, const std::vector<double>& cs, const std::vector<const double*>& xs)
{
    LinC L{};
    L.a = a;
    for (size_t q = 0; q < cs.size() && q < 16; q++) {
        L.c[L.nv] = cs[q];
        L.X[L.nv] = xs[q];
        L.nv++;
    }
    return L;
}
void clin(iemic_coupled* cm, double a, double* y, const std::vector<double>& cs, const std::vector<const double*>& xs)
{
    hipLaunchKernelGGL(k_clincomb, dim3(blocks_for(cm->NC)), dim3(256), 0, cm->oc->stream, make_linc(a, cs, xs), y,
                       cm->NC);
}
void clin2(iemic_coupled* cm, double a1, double* y1, const std::vector<double>& c1, const std::vector<const double*>& x1,
           double a2, double* y2, const std::vector<double>& c2, const std::vector<const double*>& x2)
{
    hipLaunchKernelGGL(k_clincomb2, dim3(blocks_for(cm->NC)), dim3(256), 0, cm->oc->stream, make_linc(a1, c1, x1), y1,
                       make_linc(a2, c2, x2), y2, cm->NC);
}

/* IDR(s) on the packed coupled vector (IDRSolver.H:109-340: the same restatement as the
 * ocean's krylov.hip idrs -- bi-orthogonalisation against the shadow space P, omega with
 * the angle safeguard, optional residual replacement), right preconditioned by the block
 * Gauss-Seidel preconditioner.  b, x: device packed vectors; x starts at 0. */
int coupled_idrs(iemic_coupled* cm, const double* b, double* x, const iemic_krylov* opt, double normb,
                 iemic_solve_info& inf)
{
    hipStream_t st = cm->oc->stream;
    const int s = std::max(1, std::min(opt->idr_s > 0 ? opt->idr_s : 4, 8));
    const double angle = opt->idr_angle > 0.0 ? opt->idr_angle : 0.7;
    const double mp = 1e-13;
    const int maxit = std::max(1, opt->krylov_dim * (opt->max_restarts + 1));
    const int64_t NC = cm->NC;
    const int need = 3 * s + 3;
    if (cm->mk < need) {
        if (cm->V.alloc((size_t)(need + 1) * NC) || cm->Z.alloc((size_t)need * NC)) {
            set_error("coupled IDR(s): out of device memory");
            return IEMIC_ENOMEM;
        }
        cm->mk = need;
    }
    double* P = cm->V.p;
    double* U = P + (int64_t)s * NC;
    double* G = U + (int64_t)s * NC;
    double* t = G + (int64_t)s * NC;
    double* r = t + NC;
    double* v = r + NC;
    auto Ui = [&](int i) { return U + (int64_t)i * NC; };
    auto Gi = [&](int i) { return G + (int64_t)i * NC; };
    auto Pi = [&](int i) { return P + (int64_t)i * NC; };
    std::vector<double> tmp(s + 2);
    int rc = 0;
    hipLaunchKernelGGL(k_cidr_random, dim3((unsigned)((NC + 255) / 256)), dim3(256), 0, st, P, NC, s, NC);
    for (int j = 0; j < s; j++) {
        if (j > 0) {
            cdot_host(cm, P, NC, j, Pi(j), tmp.data());
            std::vector<double> cs;
            std::vector<const double*> xs;
            for (int k = 0; k < j; k++) { cs.push_back(-tmp[k]); xs.push_back(Pi(k)); }
            clin(cm, 1.0, Pi(j), cs, xs);
        }
        const double nn = std::sqrt(std::max(0.0, cdot_host(cm, nullptr, 0, 0, Pi(j), tmp.data())));
        hipLaunchKernelGGL(k_cscale, dim3(blocks_for(NC)), dim3(256), 0, st, 1.0 / nn, (const double*)Pi(j), Pi(j), NC);
    }
    HIP_OK(hipMemcpyAsync(r, b, sizeof(double) * NC, hipMemcpyDeviceToDevice, st));
    const double tolb = opt->tol * normb;
    double normr = normb;
    std::vector<double> f(s + 1, 0.0), gamma(s, 0.0), d(s + 2, 0.0);
    std::vector<std::vector<double>> M(s, std::vector<double>(s, 0.0));
    double om = 1.0;
    int jj = 0, iter = 0;
    bool trueres = false;
    auto prec = [&](const double* in, double* out) { return cpl_prec(cm, in, out, opt->prec > 0); };
    while (normr > tolb && iter < maxit) {
        cdot_host(cm, P, NC, s, r, f.data());                         /* f = P' r */
        for (int k = 0; k < s; k++) {
            if (jj > 0) {
                std::vector<double> cs{1.0};
                std::vector<const double*> xs{r};
                for (int i = k; i < s; i++) {
                    double gi = f[i];
                    for (int j = k; j < i; j++) gi -= M[i][j] * gamma[j];
                    gamma[i] = gi / M[i][i];
                    cs.push_back(-gamma[i]);
                    xs.push_back(Gi(i));
                }
                clin(cm, 0.0, v, cs, xs);                                    /* v = r - G gamma */
                if ((rc = prec(v, t))) return rc;
                cs.assign(1, om);
                xs.assign(1, t);
                for (int i = k; i < s; i++) { cs.push_back(gamma[i]); xs.push_back(Ui(i)); }
                clin(cm, 0.0, Ui(k), cs, xs);
            } else {
                if ((rc = prec(r, Ui(k)))) return rc;
            }
            if ((rc = cpl_apply(cm, Ui(k), Gi(k)))) return rc;
            cdot_host(cm, P, NC, s, Gi(k), d.data());
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
                clin2(cm, 1.0, Gi(k), cs, xg, 1.0, Ui(k), cs, xu);
            }
            if (!std::isfinite(M[k][k]) || M[k][k] == 0.0) {
                set_error("coupled IDR(s): breakdown");
                return IEMIC_ERANGE;
            }
            const double beta = f[k] / M[k][k];
            clin2(cm, 1.0, r, {-beta}, {Gi(k)}, 1.0, x, {beta}, {Ui(k)});
            normr = std::sqrt(std::max(0.0, cdot_host(cm, nullptr, 0, 0, r, tmp.data())));
            if (!std::isfinite(normr)) {
                set_error("coupled IDR(s): non-finite residual");
                return IEMIC_ERANGE;
            }
            if (opt->idr_replace && normr > tolb / mp) trueres = true;
            for (int i = k + 1; i < s; i++) f[i] -= beta * M[i][k];
            iter++;
            if (normr < tolb || iter >= maxit) break;
        }
        if (normr < tolb || iter >= maxit) break;
        jj++;
        if ((rc = prec(r, v))) return rc;
        if ((rc = cpl_apply(cm, v, t))) return rc;
        double tt_tr[2];
        cdot_host(cm, r, NC, 1, t, tmp.data());                      /* r.t, t.t */
        tt_tr[0] = tmp[1];
        tt_tr[1] = tmp[0];
        const double nt = std::sqrt(std::max(0.0, tt_tr[0])), ts = tt_tr[1];
        if (!(nt > 0.0) || !std::isfinite(ts)) {
            set_error("coupled IDR(s): breakdown in omega");
            return IEMIC_ERANGE;
        }
        const double rho = std::fabs(ts / (nt * normr));
        om = ts / (nt * nt);
        if (rho < angle) om = om * angle / rho;
        clin2(cm, 1.0, r, {-om}, {t}, 1.0, x, {om}, {v});
        normr = std::sqrt(std::max(0.0, cdot_host(cm, nullptr, 0, 0, r, tmp.data())));
        if (opt->idr_replace && normr > tolb / mp) trueres = true;
        if (trueres && normr < normb) {
            if ((rc = cpl_apply(cm, x, r))) return rc;
            hipLaunchKernelGGL(k_axpby_c, dim3(blocks_for(NC)), dim3(256), 0, st, 1.0, b, -1.0, (const double*)r, r, NC);
            normr = std::sqrt(std::max(0.0, cdot_host(cm, nullptr, 0, 0, r, tmp.data())));
            trueres = false;
            inf.reorth++;
        }
        iter++;
    }
    inf.iters = iter;
    inf.implicit_rel_res = normr / normb;
    return 0;
}
}  // namespace

/* CoupledModel::solve -> FGMRESSolve (353-432): right-preconditioned FGMRES(m) with
 * restarts on the packed coupled vector, classical Gram-Schmidt with one
 * re-orthogonalisation pass, x0 = 0, explicit residual at the end.  b, x: host vectors
 * [ocean (reference order) | atmosphere].  Jacobian and preconditioner must be current
 * (iemic_coupled_jacobian); opt->prec > 0 selects the block Gauss-Seidel preconditioner
 * with the ocean's block preconditioner (computed here) inside. */
extern "C" int iemic_coupled_solve(iemic_coupled* cm, const double* b_host, double* x_host,
                                   const iemic_krylov* opt, iemic_solve_info* info)
{
    if (!cm || !b_host || !x_host || !opt) return IEMIC_EINVAL;
    iemic_ctx* oc = cm->oc;
    iemic_atmos* a = cm->at;
    if (hipSetDevice(oc->device) != hipSuccess) return IEMIC_EDEVICE;
    if (!oc->jac_valid || !a->jac_valid) {
        set_error("iemic_coupled_solve: no Jacobian assembled");
        return IEMIC_ESTATE;
    }
    StreamGuard guard{oc};
    auto T0 = std::chrono::steady_clock::now();
    hipStream_t s = oc->stream;
    const int m = std::max(1, std::min(opt->krylov_dim, MAX_KRYLOV - 1));
    const int64_t NL = cm->NL, NA = cm->NA, NC = cm->NC, o = NUN * oc->own0;
    int rc = 0;
    if (opt->prec > 0) {
        if ((rc = prec_compute(oc, opt))) return rc;
        if ((rc = atm_prec_compute(a))) return rc;
    }
    if (cm->mk < m) {
        if (cm->V.alloc((size_t)(m + 1) * NC) || cm->Z.alloc((size_t)m * NC)) {
            set_error("iemic_coupled_solve: out of device memory for the Krylov basis");
            return IEMIC_ENOMEM;
        }
        cm->mk = m;
    }
    /* b, x to packed device vectors */
    std::vector<double> ext((size_t)oc->nerows, 0.0), packed((size_t)NC);
    oc->su.ref_to_ext(b_host, ext.data());
    std::copy(ext.begin() + o, ext.begin() + o + NL, packed.begin());
    std::copy(b_host + oc->nrows, b_host + oc->nrows + NA, packed.begin() + NL);
    DevBuf<double> db, dxv;
    if (db.alloc(NC) || dxv.alloc(NC)) return IEMIC_ENOMEM;
    if ((rc = h2d(oc, db.p, packed.data(), sizeof(double) * NC))) return rc;
    HIP_OK(hipMemsetAsync(dxv.p, 0, sizeof(double) * NC, s));
    double* V = cm->V.p;
    double* Z = cm->Z.p;
    double* w = cm->w.p;
    double* r = cm->r.p;
    const unsigned G = blocks_for(NC);
    std::vector<double> H((size_t)(m + 1) * m, 0.0), cs(m), sn(m), g(m + 1), h(m + 2), h2(m + 2), y(m);
    std::vector<double> tmp(m + 2);
    iemic_solve_info inf{};
    double bb = cdot_host(cm, nullptr, 0, 0, db.p, tmp.data());
    const double bnorm = std::sqrt(std::max(bb, 0.0));
    if (!(bnorm > 0)) {
        inf.converged = 1;
        if (info) *info = inf;
        std::fill(x_host, x_host + oc->nrows + NA, 0.0);
        return 0;
    }
    double beta = bnorm, res = 1.0;
    int it = 0;
    if (opt->method == 1) {
        if ((rc = coupled_idrs(cm, db.p, dxv.p, opt, bnorm, inf))) return rc;
        it = inf.iters;
        res = inf.implicit_rel_res;
        if ((rc = cpl_apply(cm, dxv.p, w))) return rc;
        hipLaunchKernelGGL(k_axpby_c, dim3(G), dim3(256), 0, s, 1.0, (const double*)db.p, -1.0, (const double*)w, r, NC);
        beta = std::sqrt(std::max(cdot_host(cm, nullptr, 0, 0, r, tmp.data()), 0.0));
    } else {
    HIP_OK(hipMemcpyAsync(r, db.p, sizeof(double) * NC, hipMemcpyDeviceToDevice, s));
    for (int cycle = 0; cycle <= opt->max_restarts; cycle++) {
        hipLaunchKernelGGL(k_cscale, dim3(G), dim3(256), 0, s, 1.0 / beta, (const double*)r, V, NC);
        std::fill(g.begin(), g.end(), 0.0);
        g[0] = beta;
        /* step jj enqueued: preconditioner, operator, CGS2 with the coefficients on the
         * device, the new vector scaled on the device, its coefficients copied into half
         * jj & 1 of the pinned h_red; the host enqueues step jj + 1 before it reads step jj
         * (the work of a step after the last one of a cycle is discarded) */
        const size_t HH = 2 * MAX_KRYLOV + 8;
        auto enqueue = [&](int jj) -> int {
            double* vj = V + (int64_t)jj * NC;
            double* zj = Z + (int64_t)jj * NC;
            double* vn = V + (int64_t)(jj + 1) * NC;
            int rc2;
            if ((rc2 = cpl_prec(cm, vj, zj, opt->prec > 0))) return rc2;
            if ((rc2 = cpl_apply(cm, zj, vn))) return rc2;
            double* hc0 = cm->hc.p + (size_t)(jj & 1) * HH;
            double* hc1 = hc0 + (jj + 1);
            double* hcn = hc0 + 2 * (jj + 1);
            for (int pass = 0; pass < 2; pass++) {
                double* hv = pass ? hc1 : hc0;
                if ((rc2 = cdot_dev(cm, V, NC, jj + 1, vn, hv))) return rc2;
                hipLaunchKernelGGL(k_cupdate_m, dim3(G), dim3(256), 0, s, (const double*)V, NC, jj + 1,
                                   (const double*)hv, vn, NC);
            }
            if ((rc2 = cdot_dev(cm, nullptr, 0, 0, vn, hcn))) return rc2;
            hipLaunchKernelGGL(k_cscale_dev, dim3(G), dim3(256), 0, s, (const double*)hcn, vn, NC);
            HIP_OK(hipMemcpyAsync(cm->h_red + (size_t)(jj & 1) * HH, hc0, sizeof(double) * (2 * (jj + 1) + 1),
                                  hipMemcpyDeviceToHost, s));
            HIP_OK(hipEventRecord(cm->ev[jj & 1], s));
            return 0;
        };
        int j = 0;
        if ((rc = enqueue(0))) return rc;
        for (; j < m; j++) {
            if (j + 1 < m && (rc = enqueue(j + 1))) return rc;
            DEV_WAIT_EVENT(cm->oc, cm->ev[j & 1]);
            const double* hr = cm->h_red + (size_t)(j & 1) * HH;
            for (int i = 0; i <= j; i++) h[i] = hr[i] + hr[j + 1 + i];
            const double hn2 = hr[2 * (j + 1)];
            if (!std::isfinite(hn2)) {
                (void)dev_wait(cm->oc, nullptr, "coupled fgmres");
                set_error("coupled FGMRES: non-finite value in the Krylov basis");
                return IEMIC_ERANGE;
            }
            const double hn = std::sqrt(std::max(hn2, 0.0));
            for (int i = 0; i <= j; i++) H[(size_t)i * m + j] = h[i];
            H[(size_t)(j + 1) * m + j] = hn;
            for (int i = 0; i < j; i++) {
                const double x0 = H[(size_t)i * m + j], x1 = H[(size_t)(i + 1) * m + j];
                H[(size_t)i * m + j] = cs[i] * x0 + sn[i] * x1;
                H[(size_t)(i + 1) * m + j] = -sn[i] * x0 + cs[i] * x1;
            }
            const double x0 = H[(size_t)j * m + j], x1 = H[(size_t)(j + 1) * m + j];
            const double d = std::sqrt(x0 * x0 + x1 * x1);
            cs[j] = d > 0 ? x0 / d : 1.0;
            sn[j] = d > 0 ? x1 / d : 0.0;
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
        for (int i = j - 1; i >= 0; i--) {
            double t = g[i];
            for (int q = i + 1; q < j; q++) t -= H[(size_t)i * m + q] * y[q];
            y[i] = t / H[(size_t)i * m + i];
        }
        if (j > 0) {
            (void)hipMemcpyAsync(cm->hb.p + MAX_KRYLOV + 4, y.data(), sizeof(double) * j, hipMemcpyHostToDevice, s);
            hipLaunchKernelGGL(k_cupdate, dim3(G), dim3(256), 0, s, (const double*)Z, NC, j,
                               (const double*)(cm->hb.p + MAX_KRYLOV + 4), 1.0, dxv.p, NC);
        }
        /* r = b - A x */
        if ((rc = cpl_apply(cm, dxv.p, w))) return rc;
        hipLaunchKernelGGL(k_axpby_c, dim3(G), dim3(256), 0, s, 1.0, (const double*)db.p, -1.0, (const double*)w, r, NC);
        beta = std::sqrt(std::max(cdot_host(cm, nullptr, 0, 0, r, tmp.data()), 0.0));
        if (res <= opt->tol || cycle == opt->max_restarts) break;
    }
    }
    inf.iters = it;
    inf.implicit_rel_res = res;
    inf.explicit_rel_res = beta / bnorm;
    inf.converged = res <= opt->tol && inf.explicit_rel_res <= 10.0 * opt->tol;
    inf.t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
    if ((rc = d2h(oc, packed.data(), dxv.p, sizeof(double) * NC))) return rc;
    std::fill(ext.begin(), ext.end(), 0.0);
    std::copy(packed.begin(), packed.begin() + NL, ext.begin() + o);
    oc->su.ext_to_ref(ext.data(), x_host);
    std::copy(packed.begin() + NL, packed.end(), x_host + oc->nrows);
    if (info) *info = inf;
    return 0;
}
