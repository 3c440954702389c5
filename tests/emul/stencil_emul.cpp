/*
 * stencil_emul.cpp -- TEST HARNESS: runs the device library's per-row assembly code
 * (i-emic_amd/csrc/stencil.h, host_setup.h) on the CPU, loop for loop like the kernels
 * k_jacobian / k_rhs / k_diagB / k_qint / k_forcing, so the restated arithmetic can be
 * checked bit-for-bit against the oracle without a GPU.  Never linked into the product.
 */
#include <cstring>
#include <vector>

#include "../../i-emic_amd/csrc/host_setup.h"

using namespace iemic;

struct Emul {
    host::Setup su;
    std::vector<double> frc, qcor;
};

template <int R>
static void jac_rows(const Geo& g, const double* x, int64_t ncell, int64_t rowintcon, double* val)
{
    constexpr int B = RowInfo<R>::B, NS = RowInfo<R>::NS;
    for (int64_t cell = 0; cell < ncell; cell++) {
        int i = (int)(cell % g.n) + 1, j = (int)((cell / g.n) % g.m) + 1, k = (int)(cell / ((int64_t)g.n * g.m)) + 1;
        double A[NS];
        bool fz;
        assemble_row<R, true>(g, x, i, j, k, A, fz);
        const bool dense = (NUN * cell + R) == rowintcon;
        for (int s = 0; s < NS; s++) val[(int64_t)(B + s) * ncell + cell] = dense ? 0.0 : A[s];
    }
}
template <int R>
static void rhs_rows(const Geo& g, const double* x, const double* frc, int64_t ncell, double* F)
{
    for (int64_t cell = 0; cell < ncell; cell++) {
        int i = (int)(cell % g.n) + 1, j = (int)((cell / g.n) % g.m) + 1, k = (int)(cell / ((int64_t)g.n * g.m)) + 1;
        F[NUN * cell + R] = rhs_row_value<R>(g, x, frc, i, j, k, cell);
    }
}

extern "C" {

void* emul_create(const iemic_grid* grid, const int* landm)
{
    Emul* e = new Emul();
    e->su.init(*grid, landm);
    return e;
}
void emul_destroy(void* h) { delete (Emul*)h; }
void emul_set_par(void* h, int idx, double v) { ((Emul*)h)->su.par[idx] = v; }
double emul_get_par(void* h, int idx) { return ((Emul*)h)->su.par[idx]; }

static void forcing(Emul* e)
{
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data());
    std::vector<double> ft = su.forcing_tables();
    e->qcor.assign(8, 0.0);
    forcing_qint(g, ft.data(), e->qcor.data(), su.cfg.tres == 0, su.cfg.sres == 0);
    int64_t ncell = (int64_t)su.n * su.m * su.l;
    e->frc.assign(NUN * ncell, 0.0);
    for (int64_t cell = 0; cell < ncell; cell++) {
        int i = (int)(cell % g.n) + 1, j = (int)((cell / g.n) % g.m) + 1, k = (int)(cell / ((int64_t)g.n * g.m)) + 1;
        forcing_cell(g, ft.data(), e->qcor.data(), i, j, k, &e->frc[NUN * cell]);
    }
}

void emul_jacobian(void* h, const double* x, double* val, double* B)
{
    Emul* e = (Emul*)h;
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data());
    int64_t ncell = (int64_t)su.n * su.m * su.l;
    jac_rows<UU>(g, x, ncell, su.rowintcon, val);
    jac_rows<VV>(g, x, ncell, su.rowintcon, val);
    jac_rows<WW>(g, x, ncell, su.rowintcon, val);
    jac_rows<PP>(g, x, ncell, su.rowintcon, val);
    jac_rows<TT>(g, x, ncell, su.rowintcon, val);
    jac_rows<SS>(g, x, ncell, su.rowintcon, val);
    for (int64_t cell = 0; cell < ncell; cell++) {
        int i = (int)(cell % g.n) + 1, j = (int)((cell / g.n) % g.m) + 1, k = (int)(cell / ((int64_t)g.n * g.m)) + 1;
        double b[NUN];
        diagB_cell(g, i, j, k, b);
        for (int v = 0; v < NUN; v++) B[NUN * cell + v] = (NUN * cell + v == su.rowintcon) ? 0.0 : b[v];
    }
}

void emul_rhs(void* h, const double* x, double* F)
{
    Emul* e = (Emul*)h;
    forcing(e);
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data());
    int64_t ncell = (int64_t)su.n * su.m * su.l;
    rhs_rows<UU>(g, x, e->frc.data(), ncell, F);
    rhs_rows<VV>(g, x, e->frc.data(), ncell, F);
    rhs_rows<WW>(g, x, e->frc.data(), ncell, F);
    rhs_rows<PP>(g, x, e->frc.data(), ncell, F);
    rhs_rows<TT>(g, x, e->frc.data(), ncell, F);
    rhs_rows<SS>(g, x, e->frc.data(), ncell, F);
    if (su.rowintcon >= 0) {
        std::vector<double> ic = su.intcond_coeff();
        double s = 0.0;
        for (size_t r = 0; r < ic.size(); r++) s += ic[r] * x[r];
        F[su.rowintcon] = su.cfg.int_sign * (s - 0.0);
    }
}

/* Epetra-shaped CSR of emulated slot values (same routine as iemic_export_csr) */
int64_t emul_to_csr(void* h, const double* v, int64_t* rowptr, int* col, double* val)
{
    Emul* e = (Emul*)h;
    std::vector<double> ic = e->su.intcond_coeff();
    return e->su.to_csr(v, ic.data(), rowptr, col, val);
}

/* slot -> column map helper for CSR conversion in tests */
int64_t emul_slot_col(void* h, int s, int64_t cell)
{
    Emul* e = (Emul*)h;
    const host::Setup& su = e->su;
    Geo g = su.geo(su.landm.data(), su.tab.data());
    int i = (int)(cell % g.n) + 1, j = (int)((cell / g.n) % g.m) + 1, k = (int)(cell / ((int64_t)g.n * g.m)) + 1;
    return slot_col(g, s, i, j, k);
}
}
