/*
 * iemic.h -- C ABI of the MI355X-native Newton-Krylov core for the THCM ocean model.
 *
 * Drop-in boundary.  The reference splits this path across three seams;
 * this ABI replaces the two lower ones and is what the Ocean-shaped C++ host
 * (i-emic_amd/csrc/ocean.hpp) and the Python mirror (i-emic_amd/iemic/) bind:
 *
 *   THCM Fortran ABI (assembly)      src/ocean/THCM.C:47-174, usrc.F90:6-586
 *     init_ / setparcs_ / matrix_ / rhs_ / fillcolb_        -> iemic_create / iemic_set_par /
 *                                                              iemic_jacobian / iemic_rhs
 *   Epetra_CrsMatrix storage + Apply  THCM.C:739-751, Ocean.C:1352-1357
 *                                                           -> iemic_spmv / iemic_export_csr
 *   mrilucpp_* factor/apply           src/mrilucpp/Ifpack_MRILU.cpp:22-39,
 *                                     mrilucpp.F90:120-553   -> iemic_prec_compute / iemic_prec_apply
 *   Belos BlockGmresSolMgr (FGMRES)   Ocean.C:961-1137        -> iemic_solve
 *
 * Conventions
 *  - Return codes: 0 on success, negative errno-style values on failure; the ABI never
 *    throws and never falls back to the CPU: without a usable gfx950 device every
 *    compute entry point returns IEMIC_ENODEV.
 *  - Vectors are fp64 in the reference's global row order
 *    row = 6*((k*m + j)*n + i) + var, var in {u,v,w,p,T,S} (FIND_ROW2, THCMdefs.H:21).
 *  - Pointers are host pointers unless the function name ends in _dev (device pointers
 *    into memory the caller allocated on the context's device, e.g. torch tensors).
 *  - A context is single-host-thread and not re-entrant, like the reference THCM
 *    singleton; independent contexts may coexist (one per GPU / rank).
 */
#ifndef IEMIC_H
#define IEMIC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IEMIC_ENODEV  (-19)
#define IEMIC_EINVAL  (-22)
#define IEMIC_ENOMEM  (-12)
#define IEMIC_EDEVICE (-5)
#define IEMIC_ESTATE  (-71)
#define IEMIC_ERANGE  (-34)   /* non-finite value in the operator / preconditioner output */
#define IEMIC_ENOCONV (1)     /* warning: the step was applied but its linear solve did not
                                 reach the tolerance (iemic_newton_step)                   */

/* Version of this header's structs and entry points.  Bumped whenever a struct changes
 * size or meaning (5: iemic_solve_info gained `safeguard` in round 4, the device vector
 * algebra of round 5); a caller built against another header must refuse to run:
 *   if (iemic_abi_version() != IEMIC_ABI_VERSION) abort(); */
#define IEMIC_ABI_VERSION 6
int iemic_abi_version(void);

typedef struct iemic_ctx iemic_ctx;

/* THCM ParameterList subset used by the hot path (THCM.C:189-265; defaults 2748-2813). */
typedef struct {
    int n, m, l;                 /* "Global Grid-Size n/m/l"                         */
    double xmin, xmax, ymin, ymax;/* "Global Bound ..." in degrees                   */
    int periodic;                /* "Periodic"                                       */
    double hdim, qz;             /* "Depth hdim", "Grid Stretching qz"               */
    int tres, sres;              /* "Restoring Temperature/Salinity Profile"         */
    int forcing_type;            /* "Forcing Type"                                   */
    int ih;                      /* "Inhomogeneous Mixing"                           */
    int vmix;                    /* "Mixing" (vmix_GLB): 0, 1 or 2, default vmix_par   */
    int coriolis_on;             /* "Coriolis Force"                                 */
    double alpha_t, alpha_s;     /* "Linear EOS: alpha T/S"                          */
    int int_sign;                /* "Salinity Integral Sign"                         */
    int int_i, int_j;            /* "Integral row coordinate i/j" (-1: default)      */
    int analyze_jacobian;        /* Ocean "Analyze Jacobian" mask fix (Ocean.C:505)  */
    int max_mask_fixes;          /* Ocean "Max mask fixes" (default 5)               */
    int device;                  /* HIP device ordinal                               */
    int rho_mixing;              /* "Rho mixing" (vmix_fun: mix T and S as density)  */
    int coupled_t;               /* "Coupled Temperature" (THCM.C:232): surface heat    */
                                 /* flux from an atmosphere (iemic_set_atmosphere)      */
    int coupled_s;               /* "Coupled Salinity": E - P salinity flux (same)      */
} iemic_grid;

/* Krylov settings (Ocean.C:961-1020, getDefaultInitParameters 2232-2237). */
typedef struct {
    double tol;                  /* "FGMRES tolerance" (relative to ||b||, x0 = 0)   */
    int krylov_dim;              /* "FGMRES iterations" = restart length             */
    int max_restarts;            /* "FGMRES restarts"                                */
    int prec;                    /* 0: none, 1: cell block-Jacobi, 2: block Gauss-Seidel */
    int ts_sweeps;               /* symmetric red-black sweeps on the T/S block      */
    int orth;                    /* 0: DCGS2 (default), 1: DGKS (Belos' default)     */
    int dyn_iters;               /* block GS: defect-correction passes on the U/V/W/P */
                                 /* block (<= 1: one pass, the plain block GS)        */
    int method;                  /* 0: FGMRES (Belos, Ocean.C:961-1137), 1: IDR(s)    */
                                 /* (IDRSolver.H:109-340, right preconditioned)       */
    int ts_mg;                   /* block GS: T/S solve by this many aggregation-      */
                                 /* multigrid V-cycles (0: ts_sweeps plain sweeps)    */
    int mg_sweeps;               /* symmetric red-black sweeps before/after the coarse */
                                 /* correction on every multigrid level               */
    double dyn_omega;            /* block GS: step of the defect-correction passes    */
                                 /* (z_D += omega M_D^-1 d; 0 means 1)                */
    int dyn_mr;                  /* 1: minimal-residual step per pass instead         */
    int idr_s;                   /* "IDR s" (default 4)                               */
    double idr_angle;            /* "IDR angle" (omega safeguard, default 0.7)         */
    int idr_replace;             /* "IDR replace residuals" (default 0)               */
    int ts_at;                   /* block GS: form the T/S right-hand side after this  */
                                 /* many dynamics passes (0: after the last); earlier, */
                                 /* the T/S multigrid runs on a second stream beside   */
                                 /* the remaining passes (one rank)                    */
    int schur_passes;            /* block GS: this many of the dynamics passes solve   */
                                 /* the 2-D Schur system exactly, the first k - 1 and  */
                                 /* the last (k = 1: the first); the others take       */
                                 /* pbar = 0 (0 or >= dyn_iters: every pass)           */
} iemic_krylov;

typedef struct {
    int iters;                   /* total Arnoldi steps                              */
    int converged;
    double implicit_rel_res;     /* Givens estimate / ||b||                          */
    double explicit_rel_res;     /* ||b - J x|| / ||b||  (Ocean.C:1140-1150)         */
    double t_prec_ms, t_spmv_ms, t_orth_ms, t_total_ms;
    int reorth;                  /* DGKS second passes taken                         */
    int n_spmv;                  /* SpMV launches inside the Arnoldi loop (t_spmv_ms) */
    int safeguard;               /* stagnation safeguards taken: a restart cycle that cut */
                                 /* the true residual less than 4x switched the block GS  */
                                 /* correction passes to minimal-residual steps for the  */
                                 /* rest of the solve (Continuation.H:724-741's role)     */
} iemic_solve_info;

/* Domain decomposition over several GPUs (one process and one context per GPU, RCCL over
 * xGMI): the TRIOS Decomp2D split (TRIOS_Domain.C:81-195).  nranks =
 * npx * npy; rank r = py * npx + px owns columns [px*n/npx + min(px, n%npx) ...) and rows
 * likewise (the reference's remainder rule: the first ranks take one more), all levels.
 * npx = 0 picks the reference's factorisation (iemic_decomp2d); npx = 1 gives latitude
 * bands.  `id` is an RCCL unique id from iemic_comm_unique_id on rank 0, broadcast by the
 * caller (e.g. torch.distributed).  Vectors passed to the host-pointer entry points are
 * full reference-ordered global vectors of which each rank reads / writes its owned rows. */
typedef struct {
    int rank, nranks;
    unsigned char id[128];
    int npx;                     /* x parts (0: Decomp2D rule, 1: latitude bands)    */
} iemic_dist;
/* TRIOS::Domain::Decomp2D's factorisation nranks = npx * npy (TRIOS_Domain.C:88-109:
 * npy = the largest t1 <= nranks dividing it that minimises |m/t1 - n/(nranks/t1)|, ties
 * to the smaller t1) */
int iemic_decomp2d(int n, int m, int nranks, int* npx, int* npy);
/* Host transport (no RCCL): the caller's point-to-point and all-reduce over host memory,
 * e.g. torch.distributed gloo.  Per exchange batch the library calls send for every
 * outgoing message in order (it may return before delivery), then recv for every incoming
 * one in order (blocking), then wait; the k-th message sent from a to b is the k-th b
 * receives from a.  Return 0 on success. */
typedef struct {
    void* user;
    int (*send)(void* user, int peer, const double* buf, int64_t count);
    int (*recv)(void* user, int peer, double* buf, int64_t count);
    int (*wait)(void* user);
    int (*allreduce_sum)(void* user, double* buf, int64_t count);
} iemic_transport;

/* ---- lifecycle ---------------------------------------------------------------------- */
/* landm: (n+2)(m+2)(l+2) ints, i fastest, the global mask m_global::get_landm returns
 * (THCM.C:391).  The context applies init_'s border handling (usrc.F90:83-107), builds
 * grid metrics, stpnt parameters, forcing and the maximal graph, and (if requested)
 * runs the Ocean mask-fix cycle (Ocean.C:496-569, analyzeJacobian1). */
int  iemic_create(iemic_ctx** ctx, const iemic_grid* grid, const int* landm);
int  iemic_create_dist(iemic_ctx** ctx, const iemic_grid* grid, const int* landm,
                       const iemic_dist* dist);
int  iemic_comm_unique_id(unsigned char* id128);
/* the subdomain of a rank through a host transport (one process per rank, any device,
 * e.g. several processes on one GPU, where RCCL refuses duplicate devices) */
int  iemic_create_transport(iemic_ctx** ctx, const iemic_grid* grid, const int* landm, int rank,
                            int nranks, int npx, const iemic_transport* tp);
/* Test facility: the subdomains of one problem as contexts of one process (one host thread
 * each, all on `grid->device`), collectives host-staged through `group`.  Used to check
 * the decomposition on a single GPU.  iemic_create_local: latitude bands (npx = 1). */
void* iemic_local_group_new(int nranks);
void  iemic_local_group_free(void* group);
int   iemic_create_local(iemic_ctx** ctx, const iemic_grid* grid, const int* landm,
                         void* group, int rank, int nranks);
int   iemic_create_local_2d(iemic_ctx** ctx, const iemic_grid* grid, const int* landm,
                            void* group, int rank, int nranks, int npx);
/* releases the handle; the context itself is freed once no atmosphere or coupled model
 * built on it remains (each holds a reference, dropped by its own destroy) */
void iemic_destroy(iemic_ctx* ctx);
int  iemic_device_count(void);
const char* iemic_last_error(void);

/* ---- diagnostics of the state (host side, as the reference computes them) --------- */
/* THCM::getIntCondCoeff (THCM.C:2549-2577): integral-condition coefficients, global row
 * order (each rank fills its own rows) */
int iemic_get_intcond_coeff(iemic_ctx* ctx, double* coeff);
/* Ocean::getPsiM (Ocean.C:872-886, OceanGrid::recomputePsiM OceanGrid.C:270-346,
 * compute_psim thcm_utils.F90:95-118): extrema of the meridional overturning streamfunction
 * in Sv; psim (optional) = PsiM(j, k) at [(m+1) k + j], j = 0..m, k = 0..l */
int iemic_psim(iemic_ctx* ctx, double* psim_min, double* psim_max, double* psim);
/* Ocean::integralChecks (Ocean.C:1841-1848, THCM.C:2042-2118, integrals.F90:17-89): volume
 * integrals of the salt advection / diffusion operators of the state */
int iemic_integral_checks(iemic_ctx* ctx, double* salt_advection, double* salt_diffusion);

/* ---- parameters (setparcs_/getparcs_, usrc.F90:163-198; index 1..30 = par2int) --- */
int  iemic_set_par(iemic_ctx* ctx, int idx, double value);
/* THCM::setIntCondCorrection (THCM.C:2020-2038, called by Ocean at Ocean.C:144-148 for a
 * loaded SRES = 0 state): intCorrection = intcond coefficients . x, subtracted from the
 * integral-condition entry of F from then on.  x: global state in reference order, or NULL
 * for the current state.  No-op (correction 0) when SRES != 0. */
int  iemic_set_intcond_correction(iemic_ctx* ctx, const double* x);
int  iemic_get_intcond_correction(iemic_ctx* ctx, double* corr);
int  iemic_get_par(iemic_ctx* ctx, int idx, double* value);

/* ---- coupled atmosphere (grid.coupled_t = 1) ---------- */
/* Ocean::synchronize(atmos), Ocean.C:1443-1472: atmosphere T, q, albedo and dimensional
 * P on the n*m surface ((j, i), i fastest) and the 18 AtmosLocal::CommPars
 * (AtmosLocal.H:40-60) -> THCM::setAtmosphereT/Q/A/P + set_atmos_parameters_
 * (usrc.F90:237-293).  Refreshes the forcing; the next iemic_jacobian uses the new
 * latent-heat coefficient.  p (patm) enters with coupled_s = 1. */
int  iemic_set_atmosphere(iemic_ctx* ctx, const double* t, const double* q, const double* a,
                          const double* p, const double* commpars);
/* getdeps_ (usrc.F90:201-219, called by AtmosLocal::setup and Ocean::getBlock):
 * out7 = Ooa, Os, nus, eta, lvsc, qdim, pQSnd */
int  iemic_get_deps(iemic_ctx* ctx, double* out7);
/* THCM::getSunO (THCM.C:1517-1527): suno(j) broadcast on the n*m surface */
int  iemic_get_suno(iemic_ctx* ctx, double* out_nm);

/* ---- atmosphere (src/atmosphere: AtmosLocal.C, Atmosphere.C; one process, aux = 1) ---- */
typedef struct iemic_atmos iemic_atmos;
/* AtmosLocal::setParameters (AtmosLocal.C:106-171): the XML names in order */
typedef struct {
    double rhoa, rhoo, hdima, hdimq, cpa, D0, kappa, arad, brad, sun0, c0, ce, ch, uw;
    double t0a, t0o, t0i, tdim, q0, qdim, lv, udim, r0dim, a0, da;
    double tauf_days, tauc_days, Tm, Tr, Pa, epm, epr, epa;
    double par[7];   /* Combined, Solar, Longwave, Humidity, Latent Heat, Albedo Forcing,
                        T Eddy Diffusivity (AtmosLocal allParameters_, 154-170) */
} iemic_atmos_params;
int  iemic_atmos_default_params(iemic_atmos_params* p);
/* the atmosphere on the ocean context's grid, device and stream; its surface mask is the
 * ocean's top layer (AtmosLocal::setSurfaceMask 1722-1756), Ooa/Os from getdeps.  The
 * ocean context must have coupled_t = 1 (or coupled_s = 1).  On several ranks (Decomp2D
 * subdomains, CoupledModel.C:274-343) the atmosphere is replicated on every rank: its
 * host vectors are whole, the SST and the coupling rows' surface T are summed over the
 * ranks, and the coupled solver's dots count it once; ocean vectors are global
 * reference-ordered vectors of which each rank reads / writes its owned rows. */
int  iemic_atmos_create(iemic_atmos** a, iemic_ctx* ocean, const iemic_atmos_params* p);
void iemic_atmos_destroy(iemic_atmos* a);                       /* refcounted like the ocean */
int  iemic_atmos_dim(const iemic_atmos* a);                    /* 3 n m + 1               */
int  iemic_atmos_set_par(iemic_atmos* a, int idx, double v);   /* AtmosLocal::setPar      */
int  iemic_atmos_set_state(iemic_atmos* a, const double* x);
int  iemic_atmos_get_state(iemic_atmos* a, double* x);
int  iemic_atmos_set_sst(iemic_atmos* a, const double* sst);   /* setOceanTemperature     */
int  iemic_atmos_rhs(iemic_atmos* a, double* F);               /* Atmosphere::computeRHS  */
int  iemic_atmos_jacobian(iemic_atmos* a);                     /* ::computeJacobian       */
int  iemic_atmos_spmv(iemic_atmos* a, const double* x, double* y);   /* ::applyMatrix     */
int  iemic_atmos_prec_apply(iemic_atmos* a, const double* r, double* z); /* ::applyPrecon */
int  iemic_atmos_export_ell(iemic_atmos* a, double* val, int* col);  /* (dim-1) x 7      */
int  iemic_atmos_integral_coeff(iemic_atmos* a, double* pint, double* total_area, int* rowint,
                                int* rowP);
int  iemic_atmos_commpars(iemic_atmos* a, double* out18);      /* getCommPars             */
int  iemic_atmos_pdist(iemic_atmos* a, double* out_nm);        /* getPdist                */

/* ---- coupled ocean + atmosphere (src/coupledmodel/CoupledModel.C) -------------------- */
typedef struct iemic_coupled iemic_coupled;
int  iemic_coupled_create(iemic_coupled** cm, iemic_ctx* ocean, iemic_atmos* atmos);
void iemic_coupled_destroy(iemic_coupled* cm);
int  iemic_coupled_synchronize(iemic_coupled* cm);             /* synchronize 218-233      */
int  iemic_coupled_rhs(iemic_coupled* cm, double* F_ocean, double* F_atmos); /* 260-271    */
int  iemic_coupled_jacobian(iemic_coupled* cm);                /* computeJacobian 236-257  */
/* applyMatrix (436-470): x, y = [ocean (reference order) | atmosphere] */
int  iemic_coupled_spmv(iemic_coupled* cm, const double* x, double* y);
/* FGMRESSolve (366-432) with the forward block Gauss-Seidel preconditioner 'F'
 * (applyPrecon 544-585) */
int  iemic_coupled_solve(iemic_coupled* cm, const double* b, double* x, const iemic_krylov* opt,
                         iemic_solve_info* info);

/* ---- geometry queries ------------------------------------------------------------ */
int     iemic_nrows(const iemic_ctx* ctx);
int64_t iemic_graph_nnz(const iemic_ctx* ctx);       /* Epetra maximal-graph nnz       */
int     iemic_rowintcon(const iemic_ctx* ctx);       /* -1 when SRES != 0              */
int     iemic_landm(const iemic_ctx* ctx, int* out); /* effective (fixed) local mask   */
/* internal vector layout of the _dev entry points: out[0] ext length (rows), out[1] first
 * owned row, out[2] owned rows, out[3..4] owned rows [jb0, jb1), out[5] rank, out[6]
 * nranks, out[7..8] owned columns [ib0, ib1), out[9..10] process grid npx, npy, out[11]
 * x-halo width.  Internally the owned cells are ordered (j, k, i), i fastest, one
 * contiguous slab between 2 halo rows each side; the x halo (npx > 1) follows them. */
int     iemic_layout(const iemic_ctx* ctx, int64_t* out);
/* cells of this rank with a non-identity row (the rest are land: all six rows identity),
 * from the last preconditioner set-up (iemic_prec_compute / iemic_newton_step; 0 before):
 * FGMRES keeps its Arnoldi basis and the in-solve SpMV its output on these cells only */
int     iemic_active_cells(const iemic_ctx* ctx, int64_t* nact);
/* communication counters since the previous call (then reset): out[0] exchange batches
 * (one per phase of a halo exchange), out[1] messages sent, out[2] bytes sent, out[3]
 * all-reduces */
int     iemic_comm_stats(iemic_ctx* ctx, int64_t* out4);
/* the ranks the communicator itself reports (RCCL: ncclCommCount; one rank: 1) and the
 * transport: 0 none, 1 RCCL, 2 in-process group, 3 host transport (reports its nranks).
 * The reference queries Epetra_Comm::NumProc (e.g. THCM.C:404, 1717). */
int     iemic_comm_size(const iemic_ctx* ctx, int* size, int* transport);
/* Fail-fast bound (seconds) for every host wait of this context over RCCL (the stream or
 * event polled together with ncclCommGetAsyncError; on an error or timeout the communicator
 * is aborted and the call returns IEMIC_EDEVICE naming the wait, and for the first all-reduce
 * and halo batch the batch and peers) and for every barrier of the in-process group.  The
 * default, also for the collectives inside iemic_create_*, is the environment variable
 * IEMIC_COMM_TIMEOUT when set, else 300 s.  Exchange plans are checked to pair up across the
 * ranks when a context is created (a mismatch fails iemic_create_* with IEMIC_EINVAL). */
int     iemic_set_comm_timeout(iemic_ctx* ctx, double seconds);
/* Epetra_Comm::SumAll (e.g. Ocean::getColumnIntegral's column sums, Ocean.C:1851-1895):
 * buf (host, count doubles) summed over the context's ranks in place; collective */
int     iemic_allreduce_sum(iemic_ctx* ctx, double* buf, int64_t count);

/* ---- state ------------------------------------------------------------------------ */
int iemic_set_state(iemic_ctx* ctx, const double* x);     /* host -> device state     */
int iemic_get_state(iemic_ctx* ctx, double* x);
/* device -> device state copy on the library stream (x_dev: N doubles in HBM, reference
 * order, the global vector) */
int iemic_set_state_dev(iemic_ctx* ctx, const double* x_dev);

/* ---- assembly (THCM::evaluate, THCM.C:949-1192) --------------------------------- */
int iemic_jacobian(iemic_ctx* ctx);                 /* J(state) + diag(B) on device */
int iemic_rhs(iemic_ctx* ctx, double* F);           /* F(state); F may be NULL      */
int iemic_diag_b(iemic_ctx* ctx, double* B);
/* Epetra-identical CSR of J: rows sorted by column, 0-based, explicit zeros kept. */
int iemic_export_csr(iemic_ctx* ctx, int64_t* rowptr, int* col, double* val);

/* ---- operators (Epetra_Operator Apply / ApplyInverse) --------------------------- */
int iemic_spmv(iemic_ctx* ctx, const double* x, double* y);          /* y = J x     */
/* x, y: device vectors in the internal layout (iemic_layout); x's halo rows are updated */
int iemic_spmv_dev(iemic_ctx* ctx, double* x, double* y, void* stream);
int iemic_prec_compute(iemic_ctx* ctx, const iemic_krylov* opt);    /* factor once */
int iemic_prec_apply(iemic_ctx* ctx, const double* r, double* z);

/* ---- linear solve J x = b (Ocean::solve) ---------------------------------------- */
int iemic_solve(iemic_ctx* ctx, const double* b, double* x, const iemic_krylov* opt,
                iemic_solve_info* info);
/* device-resident variant: b, x are device vectors in the internal layout (iemic_layout) */
int iemic_solve_dev(iemic_ctx* ctx, const double* b, double* x, const iemic_krylov* opt,
                    iemic_solve_info* info);

/* ---- device vectors (Continuation.H's vector algebra, Utils::dot / norm / update on the
 * solve map, Continuation.H:389-813) ---------------------------------------------------
 * Vectors in the internal layout (iemic_layout: ext length, owned rows significant) on the
 * context's device, so a continuation driver keeps state, tangent, dF/dpar and the
 * corrector's solutions in HBM.  dot and norm_inf are summed / maximised over the
 * context's ranks (collective: every rank calls them in the same order). */
int iemic_vec_alloc(iemic_ctx* ctx, double** v);                 /* zeroed                 */
int iemic_vec_free(iemic_ctx* ctx, double* v);
/* z = a x + b y + c z on the owned rows (y may be NULL; c = 0 does not read z) */
int iemic_vec_update(iemic_ctx* ctx, double a, const double* x, double b, const double* y, double c,
                     double* z);
int iemic_vec_dot(iemic_ctx* ctx, const double* x, const double* y, double* out);
int iemic_vec_norm_inf(iemic_ctx* ctx, const double* x, double* out);
/* host global vector in reference order <-> device vector (owned rows) */
int iemic_vec_from_ref(iemic_ctx* ctx, const double* ref, double* v);
int iemic_vec_to_ref(iemic_ctx* ctx, const double* v, double* ref);
/* set = 0: v = state; set = 1: state = v (Model::getState / setState on the device) */
int iemic_state_vec(iemic_ctx* ctx, double* v, int set);
/* F(state) into the device vector F (Ocean::computeRHS without the host copy) */
int iemic_rhs_vec(iemic_ctx* ctx, double* F);

/* ---- one Newton step on the resident state (transient/Newton.H:92-99 form) -----
 * F(x); J(x); precond compute; solve J dx = -F; x += dx; F(x).  Returns ||F|| before /
 * after and the solve info.  Everything stays on the device. */
typedef struct {
    double norm_f0, norm_f1;
    iemic_solve_info solve;
    double t_jac_ms, t_rhs_ms, t_prec_ms, t_solve_ms, t_total_ms;
} iemic_newton_info;
int iemic_newton_step(iemic_ctx* ctx, const iemic_krylov* opt, iemic_newton_info* info);

/* ---- profiling helpers (bench): time n launches of the SpMV kernel with HIP events
 * on the stream it runs on; returns mean kernel milliseconds. */
int iemic_time_spmv(iemic_ctx* ctx, int nrep, double* ms_per_launch);
/* measurement helper (no reference counterpart): nrep back-to-back preconditioner applies
 * (iemic_prec_compute first) on the device, GPU ms per apply (events) and host ms per apply
 * spent enqueueing */
int iemic_time_prec(iemic_ctx* ctx, int nrep, double* ms_per_apply, double* host_ms_per_apply);
/* GPU microseconds per launch group of the block GS apply's parts, nrep each on zero data:
 * us4 = one Schur solve, one T/S block solve (right-hand side + V-cycle), one dynamics pass
 * (column kernels + Schur solve), one dynamics defect (diagnostics; block GS computed) */
int iemic_time_prec_parts(iemic_ctx* ctx, int nrep, double* us4);
/* Same, with the Infinity Cache flushed before every launch (a streaming read of
 * flush_bytes of flush_dev on the library stream, outside the timed span): the cold rate. */
int iemic_time_spmv_cold(iemic_ctx* ctx, int nrep, void* flush_dev, int64_t flush_bytes,
                         double* ms_per_launch);

/* ---- block ILU(0) factor handles: the MRILU seam (Ifpack_MRILU.cpp:22-39,
 * mrilucpp.F90:120-553), re-designed: a rank-local 0-based CSR (int64 row pointers) is
 * copied to the device as bs x bs blocks (bs = 6: the THCM cell block) and factorised by
 * block ILU(0) with level scheduling.  create ~ mrilucpp_create(id, n, nnz, beg, jco, co),
 * compute ~ mrilucpp_compute (once per handle: the matrix is consumed), apply ~
 * mrilucpp_apply(id, n, rhs, sol) (rhs, sol distinct), destroy ~ mrilucpp_destroy. */
typedef struct iemic_ilu iemic_ilu;
int  iemic_ilu_create(iemic_ilu** h, int device, int n, int64_t nnz, const int64_t* rowptr,
                      const int* col, const double* val, int blocksize);
int  iemic_ilu_compute(iemic_ilu* h);
int  iemic_ilu_apply(iemic_ilu* h, const double* rhs, double* sol);          /* host vectors   */
int  iemic_ilu_apply_dev(iemic_ilu* h, const double* rhs, double* sol);      /* device vectors */
/* levels of the two triangular solves and the pivot columns completed by a unit pivot */
int  iemic_ilu_stats(const iemic_ilu* h, int* lower_levels, int* upper_levels, int* perturbed);
void iemic_ilu_destroy(iemic_ilu* h);

#ifdef __cplusplus
}
#endif
#endif /* IEMIC_H */
