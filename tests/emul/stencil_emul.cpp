#include <cmath>
/*
 * stencil_emul.cpp -- TEST HARNESS: runs the device library's per-row assembly code
 * (i-emic_amd/csrc/stencil.h, host_setup.h) on the CPU, loop for loop like the kernels
 * k_jacobian / k_rhs / k_diagB / k_qint / k_forcing, over one latitude band [jb0, jb1) in
 * the library's internal (ext) layout, so the restated arithmetic and the band
 * decomposition can be checked bit-for-bit against the oracle without a GPU.  Never
 * linked into the product.
 */
#include <cstring>
#include <vector>

#include "../../i-emic_amd/csrc/host_setup.h"

using namespace iemic;

struct Emul {
    host::Setup su;
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
    e->su.init(*grid, landm, jb0, jb1);
    e->su.vmix_init();
    e->atm.assign((size_t)4 * e->su.n * e->su.m, 0.0);
    return e;
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
        const int64_t r = NUN * ((int64_t)HALO * su.l * su.n + lc);
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
