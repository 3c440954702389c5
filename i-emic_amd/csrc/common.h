/*
 * common.h -- device context shared by the assembly, Krylov and preconditioner units.
 */
#ifndef IEMIC_COMMON_H
#define IEMIC_COMMON_H

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/iemic.h"
#include "stencil.h"
#include "host_setup.h"
#include "decomp.h"

namespace iemic {

void set_error(const std::string& s);

#define HIP_OK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::iemic::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));     \
            return IEMIC_EDEVICE;                                                      \
        }                                                                              \
    } while (0)

template <typename T> struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int alloc(size_t count)
    {
        free();
        n = count;
        if (count == 0) return 0;
        if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) {
            p = nullptr;
            n = 0;
            return IEMIC_ENOMEM;
        }
        return 0;
    }
    void free()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept
    {
        if (this != &o) {
            free();
            p = o.p; n = o.n;
            o.p = nullptr; o.n = 0;
        }
        return *this;
    }
    ~DevBuf() { free(); }
};

/* Block cyclic reduction of the 2-D Schur complement (schur_cr.hip).  m x m blocks,
 * column-major; level l has N[l] blocks (N[nlev] = 1). */
struct CrGemm {                      /* C = C0 + C0b + s1 A1 B1 + s2 A2 B2                 */
    double* C;
    const double *C0, *C0b, *A1, *B1, *A2, *B2;
    double s1, s2;
};
/* one output block of a (composite) cyclic-reduction apply step: y = sum_t s_t A_t v_t
 * (A_t null: identity); vectors and output addressed as (base, offset) with base 0 the
 * solve's right-hand side b, 1 its solution x, 2 / 3 the internal level vectors bv / xv */
constexpr int CR_MT = 8;
struct CrOut {
    int yb, nt;
    int64_t yo;
    double s[CR_MT];
    const double* A[CR_MT];
    int vb[CR_MT];
    int64_t vo[CR_MT];
};
/* C = sum_k s_k A_k B_k (B_k null: s_k A_k; A_k null: s_k I), a composite operator */
struct CrComp {
    double* C;
    int nt;
    const double* A[4];
    const double* B[4];
    double s[4];
};
/* Packed apply step.  The matrix terms of every (output block, row chunk of rc rows) --
 * one workgroup -- are copied at set-up, scaled, into one contiguous run of the step's
 * buffer P: term-major, then column, then the chunk's rc rows, so a wave reads 512
 * contiguous bytes per load and no two workgroups share a cache line.  The workgroups are
 * sorted by their number of matrix terms into at most CR_NCLS classes, whose bounds travel
 * as kernel arguments: a workgroup finds its run in P without a memory load and issues its
 * matrix loads at once; only the vector references (CrWg) come from memory. */
constexpr int CR_NCLS = 8;
struct CrCls {
    int ncls;
    int w0[CR_NCLS + 1];             /* first workgroup of each class (w0[ncls] = nwg)     */
    int nA[CR_NCLS];                 /* matrix terms per workgroup of the class            */
    int64_t p0[CR_NCLS];             /* first double of the class in P                     */
};
struct CrWg {                        /* vectors of one workgroup                           */
    int yref, r0;                    /* output (base << 28 | offset), first row            */
    int nv, hasid;                   /* vector terms; the last is the identity (scale 1)   */
    int vref[CR_MT];                 /* (base << 28 | offset)                              */
};
struct CrPack {                      /* set-up copy: P[dst + c rc + rr] = s A[r0 + rr, c]  */
    const double* A;
    double s;
    int64_t dst;
    int r0;
};
struct CrStep {                      /* one apply launch                                  */
    int nwg = 0, rc = 16;            /* workgroups, rows per chunk                        */
    CrCls cls{};
    DevBuf<CrWg> wg;
    DevBuf<double> P;
    DevBuf<CrPack> jobs;
    int njobs = 0;
};
struct SchurCR {
    int n = 0, m = 0, periodic = 0, nlev = 0;
    std::vector<CrStep> down, up;    /* apply steps above the tail: one or two levels each */
    DevBuf<double> cmat;             /* composite operators                              */
    DevBuf<CrComp> cdesc;            /* their products (set-up)                          */
    int ncomp = 0;
    std::vector<int> N, per, merge;  /* blocks, periodic coupling, periodic pair merged   */
    std::vector<size_t> dlr_off;     /* level l: D, L, R blocks (3 N[l])                  */
    std::vector<size_t> ap_off;      /* level l: XL, XR (evens), Dinv, YL, YR (odds);      */
                                     /* level nlev: the last block's inverse              */
    std::vector<size_t> v_off;       /* level vectors b_l, x_l (l >= 1)                   */
    std::vector<int> g_off, g_cnt;   /* GEMM descriptor ranges: 3 per level               */
    int lt = 0, tM = 0;              /* dense tail: levels >= lt as one explicit inverse  */
    std::vector<size_t> tb_off;      /* tail set-up: batched level vectors, tM columns    */
    DevBuf<double> dlr, ap, bv, xv;
    DevBuf<double> tinv, tb, tx;     /* tail inverse (row-major tM x tM), set-up batches  */
    DevBuf<CrGemm> gd;
    DevBuf<int> info;
};
/* tail_max: the dense tail starts at the first level of at most tail_max unknowns (0: the
 * apply's default, 1024; n m: the whole problem, whose inverse cr.tinv is then built) */
int cr_init(iemic_ctx* c, SchurCR& cr, int n, int m, int periodic, int tail_max = 0);
int cr_factor(iemic_ctx* c, SchurCR& cr, const double* S9, const int* col_of_ij);
int cr_factor_blocks(iemic_ctx* c, SchurCR& cr);
int cr_check(iemic_ctx* c, SchurCR& cr);
int cr_solve(iemic_ctx* c, const SchurCR& cr, const double* b, double* x, hipStream_t s, double* xT = nullptr);
int cr_inverse_dev(hipStream_t s, int m, const double* src, double* dst, int* info);

/* Preconditioner state (prec.hip: block Jacobi, prec_gs.hip: block Gauss-Seidel). */
struct BlockGS {
    int ready = 0;
    int kind = 0;                    /* 1: block-Jacobi, 2: block Gauss-Seidel           */
    int ts_sweeps = 3;               /* symmetric red-black sweeps on the T/S block     */
    DevBuf<double> dinv;             /* block-Jacobi: 6x6 inverses, slot-major          */
    /* structure (rebuilt when the identity-row pattern changes) */
    DevBuf<double> flags_d;          /* the same flags on the device (k_band_flags)       */
    std::vector<double> flags_h;     /* global (active column, U/V point) flags the      */
                                     /* structure was built for                         */
    int ncol = 0;                    /* active water columns                            */
    DevBuf<int> own_pos;             /* Schur index -> itself for this band's active     */
                                     /* columns, -1 otherwise                           */
    DevBuf<int> ocol;                /* (j*n+i) -> this band's Schur rhs entry, -2 - entry */
                                     /* for a pinned column (written 0), -1 for none     */
    DevBuf<double> gslot;            /* per cell: U/V rows' P couplings (8) and the W row's */
                                     /* P couplings (2), halo-filled                     */
    DevBuf<double> rcol;             /* per owned water column: the Schur right-hand side */
                                     /* as a linear form in rr (18 x l coefficients)     */
    DevBuf<uint8_t> known;           /* per row: identity row (z = r)                   */
    DevBuf<int> col_of_ij;           /* (j*n+i) -> Schur index i*m+j, or -1 (no water)   */
    DevBuf<int> ij_of_col;           /* Schur index -> j*n+i                            */
    DevBuf<uint8_t> pinned;          /* Schur index pinned to 0 (null-space pins)       */
    /* numeric factors */
    DevBuf<double> uvinv, tsinv;     /* 2x2 inverses per cell (U/V and T/S blocks)      */
    DevBuf<double> pw;               /* per P row: weight of the depth integral         */
    DevBuf<uint64_t> kmask;          /* per cell: slots coupling to identity columns     */
    DevBuf<double> tsoff;            /* compact T/S off-diagonal couplings, 16 x ncell  */
    DevBuf<double> tsc, tic, bc;     /* the same per colour (even n), T/S rhs per colour */
    DevBuf<double> zt, zs, tcell;    /* T/S iterates, per-cell work                      */
    DevBuf<double> S9;               /* Schur rows, 9 couplings per column (i*m+j)       */
    SchurCR cr;                      /* its cyclic-reduction factors                     */
    int dyn_iters = 1;               /* defect-correction passes on the dynamics block   */
    DevBuf<double> dres, zc;         /* dynamics defect and correction (ext rows)        */
    DevBuf<double> dvh;              /* bands: U/V/W/P coefficients of the two halo rows  */
    DevBuf<double> dvb;              /* the active cells' U/V/W/P coefficients, blocked:  */
                                     /* [act / 64][slot][act % 64] (the defect's stream)  */
    DevBuf<double> dq, dzero, dmr;   /* MR passes: -A_DD zc, a zero vector, dot partials  */
    int dyn_mr = 0;                  /* 1: minimal-residual step length per correction   */
    double dyn_omega = 1.0;          /* fixed step of the correction passes (dyn_mr = 0) */
    int ts_at = 0;                   /* T/S rhs after this many passes (0: after all)     */
    int schur_passes = 0;            /* passes solving the Schur system: first k-1 + last (0: all) */
    /* T/S aggregation multigrid (2x2 horizontal aggregates, full depth, band-local): level q
     * has mg_n[q] x mg_m[q] x l cells in the k-contiguous level layout (prec_gs.hip TsLev;
     * level 0 packed from tsoff/tsdiag) with 16 couplings, the 2x2 block, the z-line
     * factors (12), rhs and iterate */
    static constexpr int MG_MAX = 12;
    int ts_mg = 1, mg_sweeps = 1, mg_nlev = 0;
    int mg_n[MG_MAX] = {}, mg_m[MG_MAX] = {};
    int mg_par[MG_MAX] = {};         /* colour parity of the level's cell (0, 0): global   */
                                     /* column + row offset of the subdomain's aggregates  */
    DevBuf<double> tsdiag;           /* fine 2x2 T/S blocks (active entries)              */
    DevBuf<double> mg_off[MG_MAX], mg_diag[MG_MAX], mg_fac[MG_MAX], mg_b[MG_MAX], mg_z[MG_MAX];
    DevBuf<double> mg_zu[MG_MAX];    /* fused up leg (k_mg_up): the post-smoothed iterate      */
    DevBuf<double> mg_cinv;          /* coarsest level: dense inverse (2 ncl)^2          */
    /* subdomains: the coarsest T/S level solved globally (all ranks' coarsest cells plus
     * the cross-subdomain couplings; band LU + inverse on the device, on every rank) */
    int mg_glob = 0, mg_gN = 0, mg_gGX = 0, mg_gI0 = 0, mg_gJ0 = 0;
    DevBuf<double> mg_gX, mg_gband, mg_gvec, mg_gtmp, mg_glpan;
    DevBuf<int> mg_gpiv, mg_ginfo, mg_gcols;
    DevBuf<double> mg_cdense;        /* coarsest dense operator (device assembly)        */
    /* one rank: the coarsest level is the first of <= MG_CR_CELLS cells whose columns of
     * one longitude fit a cyclic-reduction block (2 mb l <= 192); its inverse (mg_cinv, in
     * the level's unknown order) comes from a whole-problem cyclic reduction over
     * longitudes (schur_cr.hip, the explicit "tail" inverse) */
    static constexpr int MG_CR_CELLS = 1024;
    int mg_crd = 0;
    int mg_hr = 0;                   /* bands: level 0 has 2 halo rows, and its colour-1   */
                                     /* lines on them are relaxed here too (mg_vcycle)      */
    SchurCR mg_cr;
    DevBuf<int> mg_cinfo;            /* its Gauss-Jordan pivot flag                      */
    /* the dynamics passes work on component-planar copies (plane q = unknown q of every ext
     * cell, plane stride next): known flags, iterate and right-hand side; dres, zc, dq and
     * dzero are planar too.  The AoS rr is kept for the T/S sweeps (ts_mg = 0) */
    DevBuf<uint8_t> knP;
    DevBuf<double> zP, rrP;
    DevBuf<double> colvT;            /* the Schur solution transposed (j * n + i)          */
    DevBuf<double> colvZ;            /* zeros of colvT's size: pbar of a pass without Schur  */
    DevBuf<double> rr, bts, colv, colv2, colv_own; /* work: Schur rhs (colv_own; bands:  */
                                     /* summed into colv), solution colv2               */
    /* owned cells with a non-identity row (the rest: land, all six rows identity), ascending:
     * FGMRES keeps its Arnoldi basis on these cells only (krylov.hip) */
    DevBuf<int> act;
    DevBuf<int> cmap;                /* per owned cell: its index in act, -1 (land)        */
    int64_t ric = -1;                /* compressed row of the integral condition (owned)   */
    DevBuf<uint8_t> actf;            /* per owned cell: 1 active (k_cell_active)           */
    int64_t nact = 0;
    std::vector<uint8_t> act_h;      /* the per-cell flags the list was built from        */
    /* the compressed SpMV (krylov.hip k_spmv7c): the active cells' 104 coefficients blocked
     * per tile (prec_gs.hip k_spmv_pack: no coefficient line holds a land cell or another
     * tile's), and the grid tiles that hold an active cell (8 ints each: tile, first | last
     * active lane << 8, first active cell, active cells, 64-bit active-lane mask, 0, 0) */
    DevBuf<double> spc;
    DevBuf<int> atl;
    DevBuf<int> apos;                /* per active cell: its tile's index in atl            */
    int natile = 0;
    /* the Jacobian the apply reads: the set-up one (prec_gs.hip gs_refresh).  A Jacobian
     * assembled while the block GS is set up goes into the other buffer (assemble_jacobian
     * swaps iemic_ctx::d_val with vold), so the preconditioner stays the operator of its
     * set-up Jacobian on every rank, as the reference's extracted blocks do */
    const double* vp = nullptr;
    DevBuf<double> vold;
    /* a Jacobian was assembled since the set-up: the compressed SpMV's stream spc and the
     * identity-row check are redone before the next apply or solve (gs_refresh) */
    int coef_stale = 0;
    int cmp_ok = 0;                  /* the active list matches the Jacobian's identity rows */
    DevBuf<double> chk;              /* gs_refresh: identity-row mismatches (1 double)     */
};

struct Krylov {
    int m = 0;                       /* allocated basis size                            */
    DevBuf<double> V, Z;             /* (m+1) x N and m x N                             */
    DevBuf<double> w, r;
    /* DCGS2 with the block GS: the Arnoldi basis compressed to the active cells
     * (BlockGS::act, 6 nact rows per vector), the preconditioner input rf (full, zero on
     * the land cells) and, for a right-hand side with land-cell entries, t and b' */
    int mc = 0;
    int64_t nc = 0;
    DevBuf<double> Vc, rf, t, bp;
    int zclean = 0;                  /* Z is zero on the identity rows of the current set-up */
};

constexpr int RED_BLOCKS = 1024;     /* partial-sum blocks of the reductions            */
constexpr int MAX_KRYLOV = 1000;     /* largest Krylov dimension                        */
/* reduction rows (DCGS2: 2 per basis vector + 3 sums + beta, h_jj; the coefficient area
 * d_hbuf[RED_ROWS..] holds 2 per basis vector and 1/beta, gamma at DCGS_SCAL) */
constexpr int RED_ROWS = 2 * MAX_KRYLOV + 8;
constexpr int DCGS_SCAL = 2 * MAX_KRYLOV + 2;

}  // namespace iemic

struct iemic_ctx {
    iemic_grid cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;      /* second stream: the early T/S V-cycles (one rank)  */
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int n = 0, m = 0, l = 0;
    int64_t ncell = 0, nrows = 0;    /* global cells / rows                               */
    /* Decomp2D subdomain (TRIOS_Domain.C:81-195; stencil.h ext layout): process grid
     * npx x npy, rank = py * npx + px, owned columns [ib0, ib1) and rows [jb0, jb1); hx x-halo
     * columns when npx > 1; neighbours nb[W, E, S, N] (-1: none; W/E wrap when periodic) */
    iemic::Sub sub;                  /* the same, as decomp.h computed it                  */
    int rank = 0, nranks = 1;
    int npx = 1, npy = 1, px = 0, py = 0;
    int jb0 = 0, jb1 = 0, ib0 = 0, ib1 = 0, nx = 0, hx = 0;
    int64_t xb = 0;                  /* first x-halo cell of an ext vector                */
    int nb[4] = {-1, -1, -1, -1};
    int64_t nloc = 0, nlrows = 0;    /* owned cells / rows                                */
    int64_t next = 0, nerows = 0;    /* cells / rows of an ext vector (+ halo rows/columns) */
    int64_t own0 = 0;                /* ext cell of the first owned cell                  */
    int64_t rowintcon = -1;          /* ext row of the integral condition if owned        */
    double int_correction = 0.0;     /* THCM::intCorrection_ (setIntCondCorrection)      */
    void* comm = nullptr;            /* ncclComm_t when nranks > 1 over RCCL              */
    void* group = nullptr;           /* in-process rank group (test facility), else null  */
    iemic_transport tp{};            /* host transport (tp.send != null), else RCCL/group  */
    iemic::DevBuf<double> d_stage;   /* packed strided messages (RCCL)                    */
    std::vector<double> h_stage;     /* host-staged messages (group / host transport)     */
    int64_t stat[4] = {0, 0, 0, 0};  /* exchange batches, messages, bytes sent, all-reduces */
    /* fail-fast (comm.hip): every host wait of an RCCL context (stream / event + async-error
     * polling, then ncclCommAbort) and every barrier of the in-process group is bounded by
     * this (IEMIC_COMM_TIMEOUT or 300 s at creation); the first all-reduce and halo batch
     * name their batch (bits of comm_checked: 1 all-reduce, 2 halo) */
    double comm_timeout_s = 300.0;
    int comm_checked = 0;
    iemic::host::Setup su;           /* grid tables, parameters, effective mask */
    /* device tables */
    iemic::DevBuf<int> d_landm;
    iemic::DevBuf<double> d_tab;     /* cos_y | cos_yv | tan_yv | sin_yv | amh_y | bmh_y |
                                        amh_yv | bmh_yv | bmhy_yv | dfzT | dfzW          */
    iemic::DevBuf<double> d_ftab;    /* forcing tables wfun(yv), temfun(y), salfun(y), spert */
    iemic::DevBuf<double> d_frc;     /* Frc (forcing.F90), before boundaries zeroing     */
    iemic::DevBuf<double> d_qcor;    /* qint corrections                                 */
    iemic::DevBuf<double> d_intc;    /* intcond coefficients (THCM.C:2549)               */
    iemic::DevBuf<double> d_atm;     /* coupled: tatm | qatm | albe (n*m each, surface)  */
    /* state and operator */
    iemic::DevBuf<double> d_x, d_F, d_B, d_val; /* d_val: NSLOT x ncell                    */
    iemic::DevBuf<double> d_tmp1, d_tmp2, d_red;
    /* reduction buffers (allocated at create): partial sums, results, pinned host copy */
    iemic::DevBuf<double> d_part, d_hbuf;
    double* h_red = nullptr;
    int jac_valid = 0;
    int refs = 1;                    /* the handle + dependents (atmosphere, coupled model) */
    iemic::BlockGS gs;
    iemic::Krylov kr;
    iemic::Geo geo() const;
    iemic_ctx() = default;
    iemic_ctx(const iemic_ctx&) = delete;
    iemic_ctx& operator=(const iemic_ctx&) = delete;
    ~iemic_ctx();
};

namespace iemic {
/* the host waits for the stream (e null) or an event: bounded under RCCL (comm.hip) */
int dev_wait(iemic_ctx* c, hipEvent_t e, const char* what);
#define DEV_SYNC(c)                                                     \
    do {                                                                \
        const int rs_ = ::iemic::dev_wait((c), nullptr, __func__);      \
        if (rs_) return rs_;                                            \
    } while (0)
#define DEV_WAIT_EVENT(c, e)                                            \
    do {                                                                \
        const int rs_ = ::iemic::dev_wait((c), (e), __func__);          \
        if (rs_) return rs_;                                            \
    } while (0)
/* Stream-ordered copies: every transfer goes through the context's stream and is complete
 * on return (the stream is non-blocking, so the legacy null stream must never be used). */
inline int h2d(iemic_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!bytes) return 0;
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    DEV_SYNC(c);
    return 0;
}
inline int d2h(iemic_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!bytes) return 0;
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    DEV_SYNC(c);
    return 0;
}
/* p[0 .. n) = 0 by a kernel of the library.  Used instead of hipMemsetAsync on the solve
 * path: the HIP runtime dispatches a memset as its own blit kernel, and rocprofv3's kernel
 * tracer (rocprofiler-sdk 7.2) faulted inside its dispatch intercept when several host
 * threads issued those concurrently (eight in-process band ranks) */
__global__ void k_zero(double* __restrict__ p, int64_t n);
inline int dev_zero(iemic_ctx* c, double* p, int64_t n);
/* two timing events, destroyed on every return path */
struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    int create()
    {
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return IEMIC_EDEVICE;
        return 0;
    }
    ~EventPair()
    {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};
/* Drains the stream when an entry point returns, also on error paths, so no kernel of
 * this context is still in flight when control goes back to the caller. */
inline int dev_zero(iemic_ctx* c, double* p, int64_t n)
{
    if (n <= 0) return 0;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_zero, dim3(g), dim3(256), 0, c->stream, p, n);
    HIP_OK(hipGetLastError());
    return 0;
}
struct StreamGuard {
    iemic_ctx* c;
    ~StreamGuard() { if (c && c->stream) (void)dev_wait(c, nullptr, "return"); }
};

/* the subdomain layout handed to the structured-grid kernels */
inline SubLay sub_lay(const iemic_ctx* c)
{
    SubLay X;
    X.n = c->n; X.m = c->m; X.l = c->l; X.periodic = c->cfg.periodic;
    X.jb0 = c->jb0; X.ib0 = c->ib0; X.nx = c->nx; X.hx = c->hx; X.xb = c->xb;
    return X;
}

/* comm.hip: sums over the ranks (no-op for one rank) and halo exchanges.  A message is
 * nblk blocks of len doubles, stride doubles apart, from base + off; one exchange is a
 * list of messages in two phases (x, then y: the y messages carry the x halo, so the
 * corner cells arrive too), each run as one batch by the transport. */
struct Seg {
    double* base;
    int64_t off, nblk, len, stride;
};
struct Msg {
    bool send;
    int peer;
    Seg s;
};
int allreduce_sum(iemic_ctx* c, double* dev, int count);
int comm_size(const iemic_ctx* c, int* size, int* kind);
/* depth latitude rows and x columns of the ext layout (width doubles per cell) */
int halo_exchange(iemic_ctx* c, double* ext_vec, int depth);
int halo_exchange_w(iemic_ctx* c, double* ext_cells, int width, int depth);
/* the two phases of an exchange of arrays of the ext layout (appended to x / y) */
int halo_exchange_planar(iemic_ctx* c, double* v, int nplanes, int64_t ps, int depth);
void halo_plan_ext(const iemic_ctx* c, double* v, int width, int depth, std::vector<Msg>& x,
                   std::vector<Msg>& y);
int run_msgs(iemic_ctx* c, const std::vector<Msg>& ops);
int comm_init(iemic_ctx* c, const unsigned char* id, int rank, int nranks);
/* collective check at creation that every rank's exchange plans pair up (the k-th message
 * a sends to b has the size of the k-th b receives from a): a mismatch is an error naming
 * the pair, before any exchange could hang */
int comm_verify_plans(iemic_ctx* c);
/* drop one reference to the context (iemic_destroy, a dependent's destroy); the last one
 * frees it */
void ctx_release(iemic_ctx* c);
int comm_unique_id(unsigned char* id128);
void* local_group_new(int nranks);
void local_group_free(void* g);
void local_group_join(iemic_ctx* c, void* g);
void local_group_leave(iemic_ctx* c);
void comm_destroy(iemic_ctx* c);

/* assembly.hip */
int assemble_jacobian(iemic_ctx* c, const double* x_dev);
int assemble_rhs(iemic_ctx* c, const double* x_dev, double* F_dev);
int compute_forcing(iemic_ctx* c);
int intcond_correction(iemic_ctx* c, const double* x_dev);
/* krylov.hip */
/* y = J x on the owned rows; x (ext layout) gets its halo rows exchanged first */
int spmv(iemic_ctx* c, double* x, double* y, hipStream_t s);
int spmv_kernel(iemic_ctx* c, const double* x, double* y);
double dot(iemic_ctx* c, const double* a, const double* b, int64_t n);
int dot_owned(iemic_ctx* c, const double* a, const double* b, double* out);
int idrs(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt, iemic_solve_info* info);
/* opt->method: 0 FGMRES, 1 IDR(s) */
int krylov_solve(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt,
                 iemic_solve_info* info);
int fgmres(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt,
           iemic_solve_info* info);
/* prec.hip */
int prec_compute(iemic_ctx* c, const iemic_krylov* opt);
int prec_apply(iemic_ctx* c, const double* r, double* z);
/* the block GS apply from a compressed input (6 rows per BlockGS::act cell, zero land rows) */
/* staged: rc is already in the block GS's planar right-hand side (k_dcgs_update) */
int gs_apply_c(iemic_ctx* c, const double* rc, double* z, bool staged = false);
/* repack the block GS's coefficient copies after a new Jacobian (BlockGS::coef_stale) */
int gs_refresh(iemic_ctx* c);
/* y = J x written compressed (rows of the active cells only; x full, halo current) */
int spmv_kernel_c(iemic_ctx* c, const double* x, double* yc, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
}  // namespace iemic

#endif
