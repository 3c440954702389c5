#include <cmath>
/*
 * stencil_emul.cpp -- TEST HARNESS: runs the device library's per-row assembly code
 * (i-emic_amd/csrc/stencil.h, host_setup.h) on the CPU, loop for loop like the kernels
 * k_jacobian / k_rhs / k_diagB / k_qint / k_forcing, over one Decomp2D subdomain (or a
 * latitude band) in the library's internal (ext) layout, so the restated arithmetic and
 * the decomposition -- partition, neighbours and halo-exchange plans of decomp.h -- can be
 * checked bit-for-bit against the oracle without a GPU.  Never linked into the product.
 */
#include <cstring>
#include <vector>

#include "../../i-emic_amd/csrc/host_setup.h"
#include "../../i-emic_amd/csrc/decomp.h"

using namespace iemic;

struct Emul {
    host::Setup su;
    Sub sub;
    std::vector<double> frc, qcor, val;
    std::vector<double> atm;      /* coupled: tatm | qatm | albe (n*m each) */
    const double* atm_p() const { return atm.empty() ? nullptr : atm.data(); }
};

template <int R>
static void jac_rows(const Geo& g, const double* x, int64_t nloc, int64_t rowintcon, double* val)
{
    constexpr int B = RowInfo<R>::B, NS = RowInfo<R>::NS;
    for (int64_t lc = 0; lc < nloc; lc++) {
        int i, j, k;
        owned_cell(g, lc, i, j, k);
        double A[NS];
        bool fz;
        assemble_row<R, true>(g, x, i, j, k, A, fz);
        const bool dense = (NUN * (own0(g) + lc) + R) == rowintcon;
        for (int s = 0; s < NS; s++) val[(int64_t)(B + s) * nloc + lc] = dense ? 0.0 : A[s];
    }
}
template <int R>
static void rhs_rows(const Geo& g, const double* x, const double* frc, int64_t nloc, double* F)
{
    for (int64_t lc = 0; lc < nloc; lc++) {
        int i, j, k;
        owned_cell(g, lc, i, j, k);
        const int64_t cell = own0(g) + lc;
        F[NUN * cell + R] = rhs_row_value<R>(g, x, frc, i, j, k, cell);
    }
}

extern "C" {

/* the device mixing's tanh (stencil.h), for the bitwise check against the host libm */
void emul_tanh(const double* x, double* y, long n)
{
    for (long q = 0; q < n; q++) y[q] = iemic::libm_tanh(x[q]);
}

void* emul_create_band(const iemic_grid* grid, const int* landm, int jb0, int jb1)
{
    Emul* e = new Emul();
    const int s0[2] = {0, jb0}, s1[2] = {grid->n, jb1 < 0 ? grid->m : jb1};
    e->su.init(*grid, landm, s0, s1, 0);
    e->su.vmix_init();
    e->atm.assign((size_t)4 * e->su.n * e->su.m, 0.0);
    return e;
}
/* the subdomain of rank `rank` of the library's decomposition (npx = 0: Decomp2D rule);
 * null when the library would refuse it */
void* emul_create_sub(const iemic_grid* grid, const int* landm, int rank, int nranks, int npx)
{
    Sub d;
    if (sub_init(d, grid->n, grid->m, grid->l, grid->periodic, rank, nranks, npx)) return nullptr;
    Emul* e = new Emul();
    e->sub = d;
    const int s0[2] = {d.ib0, d.jb0}, s1[2] = {d.ib1, d.jb1};
    e->su.init(*grid, landm, s0, s1, d.npx > 1 ? 1 : 0);
    e->su.vmix_init();
    e->atm.assign((size_t)4 * e->su.n * e->su.m, 0.0);
    return e;
}
/* subdomain facts: ib0 ib1 jb0 jb1 npx npy nb[4] */
void emul_sub_info(void* h, int* out10)
{
    const Sub& d = ((Emul*)h)->sub;
    const int v[10] = {d.ib0, d.ib1, d.jb0, d.jb1, d.npx, d.npy, d.nb[0], d.nb[1], d.nb[2], d.nb[3]};
    for (int q = 0; q < 10; q++) out10[q] = v[q];
}
/* the library's exchange plan (decomp.h plan_ext): phase 0 (x) or 1 (y); up to cap
 * messages as (send, peer, off, nblk, len, stride); returns the message count */
int emul_plan(void* h, int width, int depth, int phase, int64_t* out, int cap)
{
    std::vector<MsgD> x, y;
    plan_ext(((Emul*)h)->sub, width, depth, x, y);
    const std::vector<MsgD>& v = phase == 0 ? x : y;
    for (size_t q = 0; q < v.size() && (int)q < cap; q++) {
        const int64_t r[6] = {v[q].send, v[q].peer, v[q].s.off, v[q].s.nblk, v[q].s.len, v[q].s.stride};
        for (int t = 0; t < 6; t++) out[6 * q + t] = r[t];
    }
    return (int)v.size();
}
int emul_decomp2d(int n, int m, int P, int* npx, int* npy)
{
    decomp2d(n, m, P, *npx, *npy);
    return 0;
}
/* iemic_set_atmosphere (capi.hip) on the CPU */
void emul_set_atmosphere(void* h, const double* t, const double* q, const double* a, const double* p,
                         const double* pars)
{
    Emul* e = (Emul*)h;
    const size_t nm = (size_t)e->su.n * e->su.m;
    for (size_t r = 0; r < nm; r++) {
        e->atm[r] = t[r];
        e->atm[nm + r] = q[r];
        e->atm[2 * nm + r] = a[r];
        e->atm[3 * nm + r] = p ? p[r] : 0.0;
    }
    e->su.set_atmos(pars);
}
void emul_get_deps(void* h, double* out7)
{
    const host::Setup& su = ((Emul*)h)->su;
    const double v[7] = {su.Ooa, su.Os, su.nus, su.eta_a, su.lvsc, su.qdim_a,
                         su.par[P_COMB] * su.par[P_SALT] * su.qsnd};
    for (int i = 0; i < 7; i++) out7[i] = v[i];
}
void* emul_create(const iemic_grid* grid, const int* landm) { return emul_create_band(grid, landm, 0, -1); }
void emul_destroy(void* h) { delete (Emul*)h; }
void emul_set_par(void* h, int idx, double v) { ((Emul*)h)->su.par[idx] = v; }
double emul_get_par(void* h, int idx) { return ((Emul*)h)->su.par[idx]; }
/* ext length (rows) of the band */
int64_t emul_ext_rows(void* h) { return NUN * ((Emul*)h)->su.next; }

static void forcing(Emul* e)
{
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data(), e->atm_p());
    std::vector<double> ft = su.forcing_tables();
    e->qcor.assign(8, 0.0);
    forcing_qint(g, ft.data(), e->qcor.data(), su.cfg.tres == 0, su.cfg.sres == 0);
    e->frc.assign((size_t)NUN * su.next, 0.0);
    for (int64_t lc = 0; lc < su.nloc; lc++) {
        int i, j, k;
        owned_cell(g, lc, i, j, k);
        forcing_cell(g, ft.data(), e->qcor.data(), i, j, k, &e->frc[NUN * (own0(g) + lc)]);
    }
}

/* vmix_control for Mixing = 2 (as assembly.hip mix_control, one band) */
static void mix_control(Emul* e, const double* x)
{
    host::Setup& su = e->su;
    if (su.cfg.vmix != 2 || su.vmix_fix) return;
    double st = 0.0, ss = 0.0;
    for (int64_t lc = 0; lc < su.nloc; lc++) {
        const int64_t r = NUN * ((int64_t)HALO * su.l * su.nx + lc);
        st += x[r + TT] * x[r + TT];
        ss += x[r + SS] * x[r + SS];
    }
    su.vmix_t = std::sqrt(st) > 1.0e-12;
    su.vmix_s = std::sqrt(ss) > 1.0e-12;
    if (!su.vmix_t) su.vmix_s = 0;
    su.vmix_fix = 1;
}

/* x: ext-layout state (owned + halo rows); fills the band's slot values and B (ext) */
void emul_jacobian_ext(void* h, const double* x, double* B)
{
    Emul* e = (Emul*)h;
    mix_control(e, x);
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data(), e->atm_p());
    const int64_t nloc = su.nloc;
    e->val.assign((size_t)NSLOT * nloc, 0.0);
    double* val = e->val.data();
    jac_rows<UU>(g, x, nloc, su.rowintcon, val);
    jac_rows<VV>(g, x, nloc, su.rowintcon, val);
    jac_rows<WW>(g, x, nloc, su.rowintcon, val);
    jac_rows<PP>(g, x, nloc, su.rowintcon, val);
    jac_rows<TT>(g, x, nloc, su.rowintcon, val);
    jac_rows<SS>(g, x, nloc, su.rowintcon, val);
    if (B)
        for (int64_t lc = 0; lc < nloc; lc++) {
            int i, j, k;
            owned_cell(g, lc, i, j, k);
            double b[NUN];
            diagB_cell(g, i, j, k, b);
            const int64_t cell = own0(g) + lc;
            for (int v = 0; v < NUN; v++) B[NUN * cell + v] = (NUN * cell + v == su.rowintcon) ? 0.0 : b[v];
        }
}

/* F (ext) of the band; the intcond entry is the band's partial dot (callers sum bands) */
void emul_rhs_ext(void* h, const double* x, double* F, double* intcond_partial)
{
    Emul* e = (Emul*)h;
    mix_control(e, x);
    forcing(e);
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data(), e->atm_p());
    const int64_t nloc = su.nloc;
    rhs_rows<UU>(g, x, e->frc.data(), nloc, F);
    rhs_rows<VV>(g, x, e->frc.data(), nloc, F);
    rhs_rows<WW>(g, x, e->frc.data(), nloc, F);
    rhs_rows<PP>(g, x, e->frc.data(), nloc, F);
    rhs_rows<TT>(g, x, e->frc.data(), nloc, F);
    rhs_rows<SS>(g, x, e->frc.data(), nloc, F);
    double s = 0.0;
    if (su.rowintcon_ref >= 0) {
        std::vector<double> ic = su.intcond_coeff();
        for (size_t r = 0; r < ic.size(); r++) s += ic[r] * x[r];
        if (su.rowintcon >= 0) F[su.rowintcon] = su.cfg.int_sign * (s - 0.0);
    }
    if (intcond_partial) *intcond_partial = s;
}

/* Epetra-shaped CSR (reference numbering) of the band's rows from the last jacobian */
int64_t emul_to_csr(void* h, int64_t* rowptr, int* col, double* val)
{
    Emul* e = (Emul*)h;
    return e->su.to_csr(e->val.data(), rowptr, col, val);
}

/* reference-ordered global vector <-> ext (owned rows; halo rows untouched) */
void emul_ref_to_ext(void* h, const double* ref, double* ext) { ((Emul*)h)->su.ref_to_ext(ref, ext); }
void emul_ext_to_ref(void* h, const double* ext, double* ref) { ((Emul*)h)->su.ext_to_ref(ext, ref); }
}
