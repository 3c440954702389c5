/*
 * thcm_ref_driver.c -- TEST INFRASTRUCTURE (oracle), never shipped, never measured.
 *
 * A serial C driver around the *reference's own* THCM Fortran assembly
 * (/root/reference/src/ocean/\*.F90, compiled in place by oracle/ref/Makefile into
 * oracle/_ref/libthcm_ref.so).  It replays the serial part of the THCM constructor
 * (src/ocean/THCM.C:178-798) and exposes the Fortran entry points the reference's
 * C++ bridge calls (src/ocean/THCM.C:47-174):
 *
 *   m_global::initialize     THCM.C:334-341   (global.F90:65-160)
 *   m_global::get_landm      THCM.C:391       (global.F90:306-329 -> topo.F90 topofit)
 *   m_global::get_spert      THCM.C:541       (global.F90:590-611)
 *   init_                    THCM.C:583-589   (usrc.F90:6-139)
 *   m_mat get_array_sizes / set_pointers  THCM.C:633-650 (mat.F90:56-102)
 *   setparcs_ / getparcs_    THCM.C:1877,1924 (usrc.F90:163-198)
 *   matrix_                  THCM.C:1058      (usrc.F90:432-504)
 *   rhs_                     THCM.C:993       (usrc.F90:506-586)
 *   m_thcm_utils::intcond_scaling THCM.C:2560 (thcm_utils.F90:285-312)
 *
 * plus the C callbacks the Fortran needs from the C++ side:
 *   thcm_forcing_integral_   serial restatement of THCM.C:2704-2737
 *   thcm_throw_error_        THCM.C:2741-2744 (aborts)
 *   timer_start_/timer_stop_ no-ops (GlobalDefinitions timers)
 *   dgetrf_/dgetri_/dgecon_  only referenced by m_scaling (never called here): abort
 *
 * Every Fortran call runs on a helper thread with a 2 GiB stack because THCM keeps
 * large automatic arrays (e.g. lin's ucsi(np,n,m,l)) on the stack (SURVEY.md §8c:
 * "run with ulimit -s unlimited").
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ---- Fortran symbols (flang mangling) ---------------------------------------- */
extern void _QMm_globalPinitialize(int*, int*, int*, double*, double*, double*, double*,
                                   double*, double*, int*, int*, int*, int*, int*, int*,
                                   int*, int*, int*, int*, int*, int*, int*,
                                   const char*, const char*, const char*, const char*,
                                   const char*);
extern void _QMm_globalPget_landm(int*);
extern void _QMm_globalPget_spert(double*);
extern void init_(int*, int*, int*, int*, double*, double*, double*, double*, double*,
                  double*, int*, int*, int*, int*, int*, int*, int*, double*, double*,
                  double*, double*, double*);
extern void _QMm_matPget_array_sizes(int*, int*);
extern void _QMm_matPset_pointers(int*, int*, int*, int*, double*, double*, int*, int*,
                                  double*);
extern void setparcs_(int*, double*);
extern void getparcs_(int*, double*);
extern void matrix_(double*);
extern void rhs_(double*, double*);
extern void _QMm_thcm_utilsPintcond_scaling(double*, int*, int*);
extern void _QMm_thcm_utilsPget_landm(int*);

/* ---- configuration (mirrors the THCM ParameterList entries used in THCM.C:189-265) */
typedef struct {
    int n, m, l;
    double xmin_deg, xmax_deg, ymin_deg, ymax_deg;
    int periodic;
    double hdim, qz;
    int itopo, flat, rd_mask;
    int tres, sres, iza, ite, its, rd_spertm;
    int coupled_T, coupled_S, forcing_type;
    int ih, vmix, tap, rho_mixing, coriolis_on;
    double alphaT, alphaS;
    char maskfile[256];
    char spertfile[256];
} thcmref_cfg;

static int g_n, g_m, g_l, g_ready;
static int *g_beg, *g_jco, *g_begF, *g_jcoF;
static double *g_co, *g_coB, *g_coF;
static int g_nrows, g_cap;

/* ---- C callbacks required by the Fortran -------------------------------------- */
void timer_start_(const char* s, long len) { (void)s; (void)len; }
void timer_stop_(const char* s, long len) { (void)s; (void)len; }
void thcm_throw_error_(const char* msg, long len)
{
    fprintf(stderr, "thcm_ref: Fortran error: %.*s\n", (int)len, msg);
    abort();
}
void dgetrf_(void) { fprintf(stderr, "thcm_ref: dgetrf_ stub called\n"); abort(); }
void dgetri_(void) { fprintf(stderr, "thcm_ref: dgetri_ stub called\n"); abort(); }
void dgecon_(void) { fprintf(stderr, "thcm_ref: dgecon_ stub called\n"); abort(); }

/* The C++ callback the Fortran forcing calls (THCM.C:2704-2737, serial case): the mean of
 * qfun2 over the wet surface cells, weighted by cos(latitude).  Accumulated latitude by
 * latitude, west to east, product before sum, as the reference does, so the sums are bitwise
 * the reference's.  y: y(1:m); landm: landm(0:n+1, 0:m+1, 0:l+1), the surface is level l. */
void thcm_forcing_integral_(double* qfun2, double* y, int* landm, double* fsint)
{
    const int nx = g_n, ny = g_m, top = g_l;
    double area = 0.0, flux = 0.0;
    for (int jj = 1; jj <= ny; jj++) {
        const double w = cos(y[jj - 1]);
        const int* wetrow = landm + ((size_t)top * (ny + 2) + jj) * (nx + 2);
        const double* frow = qfun2 + (size_t)(jj - 1) * nx;
        for (int ii = 1; ii <= nx; ii++) {
            const double wet = (double)(1 - wetrow[ii]);
            flux = frow[ii - 1] * w * wet + flux;
            area = w * wet + area;
        }
    }
    *fsint = flux / area;
}

/* ---- run a closure on a big-stack thread -------------------------------------- */
typedef void (*job_fn)(void*);
struct job { job_fn fn; void* arg; };
static void* job_tramp(void* p) { struct job* j = (struct job*)p; j->fn(j->arg); return NULL; }
static void run_big_stack(job_fn fn, void* arg)
{
    pthread_attr_t attr;
    pthread_t th;
    struct job j = {fn, arg};
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, (size_t)2 << 30);
    if (pthread_create(&th, &attr, job_tramp, &j) != 0) {
        fprintf(stderr, "thcm_ref: pthread_create failed\n");
        abort();
    }
    pthread_join(th, NULL);
    pthread_attr_destroy(&attr);
}

/* ---- init ---------------------------------------------------------------------- */
struct init_args { const thcmref_cfg* c; const int* landm_in; int rc; };

static void do_init(void* p)
{
    struct init_args* a = (struct init_args*)p;
    const thcmref_cfg* c = a->c;
    const double PI_ = 3.14159265358979323846;
    int n = c->n, m = c->m, l = c->l;
    double xmin = c->xmin_deg * PI_ / 180.0, xmax = c->xmax_deg * PI_ / 180.0;
    double ymin = c->ymin_deg * PI_ / 180.0, ymax = c->ymax_deg * PI_ / 180.0;
    double hdim = c->hdim, qz = c->qz, alphaT = c->alphaT, alphaS = c->alphaS;
    int periodic = c->periodic, itopo = c->itopo, flat = c->flat, rd_mask = c->rd_mask;
    int tres = c->tres, sres = c->sres, iza = c->iza, ite = c->ite, its = c->its;
    int rd_spertm = c->rd_spertm, cT = c->coupled_T, cS = c->coupled_S;
    int ftype = c->forcing_type, ih = c->ih, vmix = c->vmix, tap = c->tap;
    int rho = c->rho_mixing, cor = c->coriolis_on;
    g_n = n; g_m = m; g_l = l;

    /* THCM.C:334-341 */
    _QMm_globalPinitialize(&n, &m, &l, &xmin, &xmax, &ymin, &ymax, &hdim, &qz, &periodic,
                           &itopo, &flat, &rd_mask, &tres, &sres, &iza, &ite, &its,
                           &rd_spertm, &cT, &cS, &ftype, c->maskfile, c->spertfile,
                           "wind/trtau.dat", "levitus/new/t00an1", "levitus/new/s00an1");
    size_t nl = (size_t)(n + 2) * (m + 2) * (l + 2);
    int* landm = (int*)malloc(nl * sizeof(int));
    if (a->landm_in) {
        memcpy(landm, a->landm_in, nl * sizeof(int));
    } else {
        _QMm_globalPget_landm(landm); /* THCM.C:391 */
    }
    size_t nm = (size_t)n * m;
    double* taux = (double*)calloc(nm, sizeof(double));
    double* tauy = (double*)calloc(nm, sizeof(double));
    double* tatm = (double*)calloc(nm, sizeof(double));
    double* emip = (double*)calloc(nm, sizeof(double));
    double* spert = (double*)calloc(nm, sizeof(double));
    /* iza==2, ite==1, its==1 (idealized) give zero fields (global.F90:432-563); so does
     * coupled_T = 1 (get_temforcing puts tatm = 0, global.F90:472-510) */
    if (iza != 2 || ite != 1 || its != 1 || cT < 0 || cT > 1 || cS < 0 || cS > 1) {
        fprintf(stderr, "thcm_ref: only idealized ocean-only forcing is supported\n");
        a->rc = -1;
        return;
    }
    _QMm_globalPget_spert(spert); /* THCM.C:541 */
    int nmlglob = n * m * l;
    /* THCM.C:583-589 */
    init_(&n, &m, &l, &nmlglob, &xmin, &xmax, &ymin, &ymax, &alphaT, &alphaS, &ih, &vmix,
          &tap, &rho, &cor, &periodic, landm, taux, tauy, tatm, emip, spert);
    /* THCM.C:631-650 */
    _QMm_matPget_array_sizes(&g_nrows, &g_cap);
    g_beg = (int*)calloc(g_nrows + 1, sizeof(int));
    g_jco = (int*)calloc(g_cap, sizeof(int));
    g_co = (double*)calloc(g_cap, sizeof(double));
    g_coB = (double*)calloc(g_nrows, sizeof(double));
    g_begF = (int*)calloc(g_nrows + 1, sizeof(int));
    g_jcoF = (int*)calloc(g_nrows, sizeof(int));
    g_coF = (double*)calloc(g_nrows, sizeof(double));
    _QMm_matPset_pointers(&g_nrows, &g_cap, g_beg, g_jco, g_co, g_coB, g_begF, g_jcoF, g_coF);
    free(landm); free(taux); free(tauy); free(tatm); free(emip); free(spert);
    g_ready = 1;
    a->rc = 0;
}

int thcmref_init(const thcmref_cfg* cfg, const int* landm_in)
{
    if (g_ready) {
        fprintf(stderr, "thcm_ref: already initialised (THCM is a singleton)\n");
        return -1;
    }
    struct init_args a = {cfg, landm_in, -1};
    run_big_stack(do_init, &a);
    return a.rc;
}

/* ---- parameters ----------------------------------------------------------------- */
struct par_args { int idx; double v; };
static void do_setpar(void* p) { struct par_args* a = (struct par_args*)p; setparcs_(&a->idx, &a->v); }
static void do_getpar(void* p) { struct par_args* a = (struct par_args*)p; getparcs_(&a->idx, &a->v); }

void thcmref_set_par(int idx, double v) { struct par_args a = {idx, v}; run_big_stack(do_setpar, &a); }
double thcmref_get_par(int idx) { struct par_args a = {idx, 0.0}; run_big_stack(do_getpar, &a); return a.v; }

void thcmref_sizes(int* nrows, int* cap) { *nrows = g_nrows; *cap = g_cap; }

/* ---- matrix / rhs --------------------------------------------------------------- */
struct mat_args { double* x; };
static void do_matrix(void* p) { matrix_(((struct mat_args*)p)->x); }

/* Returns the Fortran CSR (1-based, as filled by fillcolA) and coB. */
int thcmref_matrix(const double* x, int* beg, int* jco, double* co, double* coB)
{
    if (!g_ready) return -1;
    double* xc = (double*)malloc(sizeof(double) * g_nrows);
    memcpy(xc, x, sizeof(double) * g_nrows);
    struct mat_args a = {xc};
    run_big_stack(do_matrix, &a);
    free(xc);
    int nnz = g_beg[g_nrows] - 1;
    memcpy(beg, g_beg, sizeof(int) * (g_nrows + 1));
    memcpy(jco, g_jco, sizeof(int) * nnz);
    memcpy(co, g_co, sizeof(double) * nnz);
    memcpy(coB, g_coB, sizeof(double) * g_nrows);
    return nnz;
}

struct rhs_args { double* x; double* B; };
static void do_rhs(void* p) { struct rhs_args* a = (struct rhs_args*)p; rhs_(a->x, a->B); }

/* Fortran rhs B (before the C++ sign flip of THCM.C:1003). */
int thcmref_rhs(const double* x, double* B)
{
    if (!g_ready) return -1;
    double* xc = (double*)malloc(sizeof(double) * g_nrows);
    memcpy(xc, x, sizeof(double) * g_nrows);
    struct rhs_args a = {xc, B};
    run_big_stack(do_rhs, &a);
    free(xc);
    return 0;
}

struct int_args { int* out; double* val; int* len; };
static void do_landm(void* p) { _QMm_thcm_utilsPget_landm(((struct int_args*)p)->out); }
static void do_intcond(void* p)
{
    struct int_args* a = (struct int_args*)p;
    _QMm_thcm_utilsPintcond_scaling(a->val, a->out, a->len);
}

/* local (post-init) landm(0:n+1,0:m+1,0:l+1) */
void thcmref_landm(int* out) { struct int_args a = {out, NULL, NULL}; run_big_stack(do_landm, &a); }

/* intcond_scaling: val/ind (1-based rows) of the S-integral, returns length */
int thcmref_intcond(double* val, int* ind)
{
    int len = 0;
    struct int_args a = {ind, val, &len};
    run_big_stack(do_intcond, &a);
    return len;
}

/* ---- coupled atmosphere (Ocean::synchronize(atmos), Ocean.C:1443-1472) ------------
 * THCM::setAtmosphereT/Q/A/P -> m_inserts insert_atmosphere_{t,q,a,p} (inserts.F90:12-100),
 * then set_atmos_parameters (usrc.F90:237-293: qdim, nuq, eta, dqso, eo0, albe0, albed,
 * nus, lvsc; calls forcing and lin).  pars = AtmosLocal::CommPars (18 doubles, in order). */
extern void _QMm_insertsPinsert_atmosphere_t(double*);
extern void _QMm_insertsPinsert_atmosphere_q(double*);
extern void _QMm_insertsPinsert_atmosphere_a(double*);
extern void _QMm_insertsPinsert_atmosphere_p(double*);
extern void set_atmos_parameters_(double*);
extern void getdeps_(double*, double*, double*, double*, double*, double*, double*);

struct atm_args { double *t, *q, *a, *p, *pars; };
static void do_set_atmos(void* p)
{
    struct atm_args* a = (struct atm_args*)p;
    _QMm_insertsPinsert_atmosphere_t(a->t);
    _QMm_insertsPinsert_atmosphere_q(a->q);
    _QMm_insertsPinsert_atmosphere_a(a->a);
    _QMm_insertsPinsert_atmosphere_p(a->p);
    set_atmos_parameters_(a->pars);
}
void thcmref_set_atmos(double* t, double* q, double* a, double* p, double* pars)
{
    struct atm_args x = {t, q, a, p, pars};
    run_big_stack(do_set_atmos, &x);
}

struct deps_args { double* out; };
static void do_getdeps(void* p)
{
    double* o = ((struct deps_args*)p)->out;
    getdeps_(o, o + 1, o + 2, o + 3, o + 4, o + 5, o + 6);
}
/* getdeps (usrc.F90:201-219): Ooa, Os, nus, eta, lvsc, qdim, pQSnd */
void thcmref_getdeps(double* out7)
{
    struct deps_args x = {out7};
    run_big_stack(do_getdeps, &x);
}
