/*
 * thcm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C + OpenMP) of the reference's hot path for one Newton step
 * of the THCM ocean model.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product (i-emic_amd/) never does.
 *
 * Parity of this restatement is pinned against the reference's own Fortran compiled
 * in place (oracle/ref -> oracle/_ref/libthcm_ref.so) and against committed golden
 * fixtures generated from it (tests/golden/).
 */
#ifndef THCM_ORACLE_H
#define THCM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n, m, l;                       /* grid (global == local, serial)            */
    double xmin_deg, xmax_deg, ymin_deg, ymax_deg;
    int periodic;
    double hdim, qz;
    int tres, sres;                    /* restoring flags (THCM.C:232-233)          */
    int ite, its, iza;                 /* idealized forcing flags (must be 1,1,2)   */
    int forcing_type, ih, vmix, coriolis_on;
    double alphaT, alphaS;
    int int_sign;                      /* "Salinity Integral Sign" (THCM.C:235)     */
    int nic, mic;                      /* integral row coordinates (-1 = default)   */
    int rho_mixing;                    /* "Rho mixing" (mix_imp.f vmix_fun)         */
    int coupled_t, coupled_s;          /* "Coupled Temperature/Salinity" (THCM.C:232) */
} orc_cfg;

typedef struct orc orc_t;

/* landm: (n+2)(m+2)(l+2) ints in THCM layout (i fastest), as passed to init_
 * (usrc.F90:29); spert: n*m (get_spert, global.F90:590-611).  */
orc_t* orc_create(const orc_cfg* cfg, const int* landm, const double* spert);
/* Ocean::synchronize(atmos) (Ocean.C:1443-1472): atmosphere T, q, albedo, P on the n*m
 * surface (i fastest) -> THCM::setAtmosphereT/Q/A/P (inserts.F90) and the 18 CommPars ->
 * set_atmos_parameters (usrc.F90:237-293), then forcing */
void orc_set_atmos(orc_t* o, const double* t, const double* q, const double* a, const double* p,
                   const double* pars18);
/* getdeps (usrc.F90:201-219): Ooa, Os, nus, eta, lvsc, qdim, pQSnd */
void orc_get_deps(const orc_t* o, double* out7);
void orc_destroy(orc_t* o);
void orc_set_par(orc_t* o, int idx, double v);
double orc_get_par(const orc_t* o, int idx);
int orc_nrows(const orc_t* o);
int orc_rowintcon(const orc_t* o);
const int* orc_landm(const orc_t* o);

/* Fortran-style thresholded CSR of matrix() (1-based, fillcolA order).  Returns nnz;
 * pass NULL arrays to query the size. */
int64_t orc_fortran_matrix(orc_t* o, const double* x, int* beg, int* jco, double* co,
                           double* coB);
/* Fortran rhs B (usrc.F90:506-586), before the C++ sign flip. */
void orc_fortran_rhs(orc_t* o, const double* x, double* B);

/* Epetra-side view (THCM.C): maximal graph (rows sorted by column, 0-based) */
int64_t orc_graph_nnz(const orc_t* o);
void orc_graph(const orc_t* o, int64_t* rowptr, int* col);
/* Jacobian values in graph order + diag(B) (THCM.C:1074-1173) */
void orc_jacobian(orc_t* o, const double* x, double* val, double* diagB);
/* F(x) as Ocean::computeRHS returns it (THCM.C:993-1033) */
void orc_rhs(orc_t* o, const double* x, double* F);
/* intcond coefficient vector (THCM.C:2549-2577), length nrows */
void orc_intcond_coeff(const orc_t* o, double* coeff);

/* ---- CPU linear algebra used by the CPU baseline ---------------------------------- */
void orc_csr_spmv(int nrows, const int64_t* rowptr, const int* col, const double* val,
                  const double* x, double* y);

#ifdef __cplusplus
}
#endif
#endif
