/*
 * capi.hip -- the C ABI (include/iemic.h): context set-up and the Newton step.
 *
 * iemic_create restates the serial set-up of the THCM constructor
 * (src/ocean/THCM.C:178-798): init_ (usrc.F90:6-139: border handling of the land mask,
 * grid (grid.F90), QTnd/QSnd, stpnt + vmix_par, forcing), rowintcon and intcond
 * coefficients (THCM.C:661-717, thcm_utils.F90:285-312), then the Ocean mask-fix cycle
 * (Ocean.C:496-569, analyzeJacobian1 at the zero state).  The 1-D metric tables (cos, tan,
 * sin of the y grid, stretching derivatives) are evaluated once on the host with the same
 * libm the reference uses, so every per-cell expression evaluated on the device is
 * bit-identical to the reference; all per-cell and per-row work runs on the GPU.
 */
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>

#include "common.h"

namespace iemic {
static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
}  // namespace iemic

using namespace iemic;

extern "C" const char* iemic_last_error(void) { return g_err.c_str(); }

extern "C" int iemic_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

Geo iemic_ctx::geo() const { return su.geo(d_landm.p, d_tab.p); }

iemic_ctx::~iemic_ctx()
{
    if (stream) (void)hipStreamSynchronize(stream);
    if (h_red) (void)hipHostFree(h_red);
    h_red = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
    /* device buffers are members: released after this body, with the stream drained */
}

namespace {

int upload_forcing_tables(iemic_ctx* c)
{
    std::vector<double> t = c->su.forcing_tables();
    HIP_OK(hipMemcpyAsync(c->d_ftab.p, t.data(), sizeof(double) * t.size(), hipMemcpyHostToDevice,
                          c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return compute_forcing(c);
}

int upload_landm(iemic_ctx* c)
{
    int rc = h2d(c, c->d_landm.p, c->su.landm.data(), sizeof(int) * c->su.landm.size());
    if (rc) return rc;
    std::vector<double> ic = c->su.intcond_coeff();
    return h2d(c, c->d_intc.p, ic.data(), sizeof(double) * ic.size());
}

/* Ocean::analyzeJacobian1 (Ocean.C:273-340) + THCM::getLandMask(fix) (THCM.C:1298-1330):
 * P rows with at most 2 entries |v| > 1e-10 (and not a land identity row) become land. */
int mask_fix(iemic_ctx* c)
{
    const int n = c->n, m = c->m;
    HIP_OK(hipMemsetAsync(c->d_tmp1.p, 0, sizeof(double) * c->nrows, c->stream));
    const int pb = ROW_BEGIN[PP], pn = ROW_BEGIN[PP + 1] - ROW_BEGIN[PP];
    std::vector<double> pv((size_t)pn * c->ncell);
    for (int cyc = 0; cyc < std::max(1, c->cfg.max_mask_fixes); cyc++) {
        int rc = assemble_jacobian(c, c->d_tmp1.p);
        if (rc) return rc;
        if ((rc = d2h(c, pv.data(), c->d_val.p + (size_t)pb * c->ncell, sizeof(double) * pv.size())))
            return rc;
        int nfix = 0;
        for (int64_t cell = 0; cell < c->ncell; cell++) {
            if (NUN * cell + PP == c->rowintcon) continue;
            double sum = 0.0;
            int el = 0;
            for (int s = 0; s < pn; s++) {
                double v = pv[(size_t)s * c->ncell + cell];
                sum += v;
                if (std::fabs(v) > 1e-10) el++;
            }
            if (sum == 1) continue;
            if (el <= 2) {
                int i = (int)(cell % n) + 1, j = (int)((cell / n) % m) + 1, k = (int)(cell / ((int64_t)n * m)) + 1;
                c->su.landm[((size_t)k * (m + 2) + j) * (n + 2) + i] = LAND;
                nfix++;
            }
        }
        if (nfix == 0) break;
        int rc2 = upload_landm(c);
        if (rc2) return rc2;
        rc2 = upload_forcing_tables(c);
        if (rc2) return rc2;
    }
    c->jac_valid = 0;
    return 0;
}

}  // namespace

extern "C" int iemic_create(iemic_ctx** out, const iemic_grid* grid, const int* landm)
{
    if (!out || !grid || !landm) return IEMIC_EINVAL;
    *out = nullptr;
    int ndev = iemic_device_count();
    if (ndev <= 0) {
        set_error("iemic_create: no HIP device available (the library never runs on the CPU)");
        return IEMIC_ENODEV;
    }
    if (grid->vmix != 0) {
        set_error("iemic_create: Mixing != 0 not implemented yet (SURVEY.md §8f row 1)");
        return IEMIC_EINVAL;
    }
    if (grid->n < 3 || grid->m < 2 || grid->l < 2) {
        set_error("iemic_create: grid too small");
        return IEMIC_EINVAL;
    }
    iemic_ctx* c = new iemic_ctx();
    c->cfg = *grid;
    c->device = std::min(std::max(grid->device, 0), ndev - 1);
    if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("iemic_create: cannot initialise the HIP device");
        delete c;
        return IEMIC_EDEVICE;
    }
    c->n = grid->n; c->m = grid->m; c->l = grid->l;
    c->ncell = (int64_t)c->n * c->m * c->l;
    c->nrows = NUN * c->ncell;
    const int n = c->n, m = c->m, l = c->l;
    const size_t nl = (size_t)(n + 2) * (m + 2) * (l + 2);
    c->su.init(*grid, landm);
    c->rowintcon = c->su.rowintcon;
    int rc = 0;
    rc |= c->d_landm.alloc(nl);
    rc |= c->d_ftab.alloc((size_t)3 * (m + 2) + (size_t)n * m);
    rc |= c->d_frc.alloc(c->nrows);
    rc |= c->d_qcor.alloc(8);
    rc |= c->d_intc.alloc(c->nrows);
    rc |= c->d_x.alloc(c->nrows);
    rc |= c->d_F.alloc(c->nrows);
    rc |= c->d_B.alloc(c->nrows);
    rc |= c->d_val.alloc((size_t)NSLOT * c->ncell);
    rc |= c->d_tmp1.alloc(c->nrows);
    rc |= c->d_tmp2.alloc(c->nrows);
    rc |= c->d_red.alloc(2048);
    rc |= c->d_part.alloc((size_t)RED_BLOCKS * RED_ROWS);
    rc |= c->d_hbuf.alloc((size_t)2 * RED_ROWS);
    if (!rc && hipHostMalloc(&c->h_red, sizeof(double) * 2 * RED_ROWS) != hipSuccess) rc = 1;
    if (rc) {
        set_error("iemic_create: out of device memory");
        delete c;
        return IEMIC_ENOMEM;
    }
    (void)hipMemsetAsync(c->d_x.p, 0, sizeof(double) * c->nrows, c->stream);
    if (c->d_tab.alloc(c->su.tab.size()) ||
        h2d(c, c->d_tab.p, c->su.tab.data(), sizeof(double) * c->su.tab.size()) != 0) {
        set_error("iemic_create: cannot upload metric tables");
        delete c;
        return IEMIC_EDEVICE;
    }
    if ((rc = upload_landm(c))) {
        delete c;
        return rc;
    }
    if ((rc = upload_forcing_tables(c))) {
        delete c;
        return rc;
    }
    if (grid->analyze_jacobian) {
        if ((rc = mask_fix(c))) {
            delete c;
            return rc;
        }
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
        set_error("iemic_create: device error during set-up");
        delete c;
        return IEMIC_EDEVICE;
    }
    *out = c;
    return 0;
}

extern "C" void iemic_destroy(iemic_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    delete c; /* ~iemic_ctx drains the stream before any buffer is released */
}

#define CTX_CHECK(c)                                   \
    if (!(c)) return IEMIC_EINVAL;                     \
    if (hipSetDevice((c)->device) != hipSuccess) {     \
        set_error("hipSetDevice failed");              \
        return IEMIC_EDEVICE;                          \
    }                                                  \
    StreamGuard stream_guard_{(c)}

extern "C" int iemic_set_par(iemic_ctx* c, int idx, double value)
{
    CTX_CHECK(c);
    if (idx < 1 || idx > 30) {
        set_error("iemic_set_par: index out of range 1..30");
        return IEMIC_EINVAL;
    }
    c->su.par[idx] = value;       /* setparcs_ (usrc.F90:163-181): par, then forcing + lin */
    c->jac_valid = 0;
    int rc = upload_forcing_tables(c);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_get_par(iemic_ctx* c, int idx, double* value)
{
    if (!c || !value || idx < 1 || idx > 30) return IEMIC_EINVAL;
    *value = c->su.par[idx];
    return 0;
}

extern "C" int iemic_nrows(const iemic_ctx* c) { return c ? (int)c->nrows : IEMIC_EINVAL; }
extern "C" int iemic_rowintcon(const iemic_ctx* c) { return c ? c->rowintcon : IEMIC_EINVAL; }
extern "C" int iemic_landm(const iemic_ctx* c, int* out)
{
    if (!c || !out) return IEMIC_EINVAL;
    std::memcpy(out, c->su.landm.data(), sizeof(int) * c->su.landm.size());
    return 0;
}

/* Maximal-graph rows (THCM.C:2288-2521): sorted, de-duplicated columns */
extern "C" int64_t iemic_graph_nnz(const iemic_ctx* c)
{
    if (!c) return IEMIC_EINVAL;
    return c->su.to_csr(nullptr, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int iemic_set_state(iemic_ctx* c, const double* x)
{
    CTX_CHECK(c);
    if (!x) return IEMIC_EINVAL;
    int rc = h2d(c, c->d_x.p, x, sizeof(double) * c->nrows);
    if (rc) return rc;
    c->jac_valid = 0;
    return 0;
}
extern "C" int iemic_set_state_dev(iemic_ctx* c, const double* x_dev)
{
    CTX_CHECK(c);
    if (!x_dev) return IEMIC_EINVAL;
    HIP_OK(hipMemcpyAsync(c->d_x.p, x_dev, sizeof(double) * c->nrows, hipMemcpyDeviceToDevice,
                          c->stream));
    c->jac_valid = 0;
    return 0;
}
extern "C" int iemic_get_state(iemic_ctx* c, double* x)
{
    CTX_CHECK(c);
    return d2h(c, x, c->d_x.p, sizeof(double) * c->nrows);
    return 0;
}

extern "C" int iemic_jacobian(iemic_ctx* c)
{
    CTX_CHECK(c);
    int rc = assemble_jacobian(c, c->d_x.p);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_rhs(iemic_ctx* c, double* F)
{
    CTX_CHECK(c);
    int rc = assemble_rhs(c, c->d_x.p, c->d_F.p);
    if (rc) return rc;
    if (F) HIP_OK(hipMemcpyAsync(F, c->d_F.p, sizeof(double) * c->nrows, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_diag_b(iemic_ctx* c, double* B)
{
    CTX_CHECK(c);
    if (!c->jac_valid) return IEMIC_ESTATE;
    int rc = d2h(c, B, c->d_B.p, sizeof(double) * c->nrows);
    if (rc) return rc;
    return 0;
}

extern "C" int iemic_export_csr(iemic_ctx* c, int64_t* rowptr, int* col, double* val)
{
    CTX_CHECK(c);
    if (!c->jac_valid) {
        set_error("iemic_export_csr: no Jacobian assembled");
        return IEMIC_ESTATE;
    }
    std::vector<double> v((size_t)NSLOT * c->ncell);
    int rc = d2h(c, v.data(), c->d_val.p, sizeof(double) * v.size());
    if (rc) return rc;
    std::vector<double> ic;
    if (c->rowintcon >= 0) {
        ic.resize(c->nrows);
        if ((rc = d2h(c, ic.data(), c->d_intc.p, sizeof(double) * c->nrows))) return rc;
    }
    c->su.to_csr(v.data(), ic.data(), rowptr, col, val);
    return 0;
}

extern "C" int iemic_spmv(iemic_ctx* c, const double* x, double* y)
{
    CTX_CHECK(c);
    int rc = h2d(c, c->d_tmp1.p, x, sizeof(double) * c->nrows);
    if (rc) return rc;
    rc = spmv(c, c->d_tmp1.p, c->d_tmp2.p, c->stream);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(y, c->d_tmp2.p, sizeof(double) * c->nrows, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_spmv_dev(iemic_ctx* c, const double* x, double* y, void* stream)
{
    CTX_CHECK(c);
    return spmv(c, x, y, stream ? (hipStream_t)stream : c->stream);
}

extern "C" int iemic_prec_compute(iemic_ctx* c, const iemic_krylov* opt)
{
    CTX_CHECK(c);
    int rc = prec_compute(c, opt);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_prec_apply(iemic_ctx* c, const double* r, double* z)
{
    CTX_CHECK(c);
    int rc = h2d(c, c->d_tmp1.p, r, sizeof(double) * c->nrows);
    if (rc) return rc;
    rc = prec_apply(c, c->d_tmp1.p, c->d_tmp2.p);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(z, c->d_tmp2.p, sizeof(double) * c->nrows, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int iemic_solve_dev(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt,
                               iemic_solve_info* info)
{
    CTX_CHECK(c);
    if (!opt) return IEMIC_EINVAL;
    return fgmres(c, b, x, opt, info);
}

extern "C" int iemic_solve(iemic_ctx* c, const double* b, double* x, const iemic_krylov* opt,
                           iemic_solve_info* info)
{
    CTX_CHECK(c);
    if (!opt || !b || !x) return IEMIC_EINVAL;
    DevBuf<double> db, dx;
    if (db.alloc(c->nrows) || dx.alloc(c->nrows)) return IEMIC_ENOMEM;
    int rc = h2d(c, db.p, b, sizeof(double) * c->nrows);
    if (rc) return rc;
    rc = fgmres(c, db.p, dx.p, opt, info);
    if (rc) return rc;
    return d2h(c, x, dx.p, sizeof(double) * c->nrows);
}

namespace iemic {
__global__ void k_newton_update(double* __restrict__ x, const double* __restrict__ dx, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        x[q] += dx[q];
}
__global__ void k_neg(const double* __restrict__ a, double* __restrict__ b, int64_t N)
{
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N;
         q += (int64_t)gridDim.x * blockDim.x)
        b[q] = -a[q];
}
}  // namespace iemic

/* transient/Newton.H:92-99: F, J, solve J dx = -F, x += dx, F */
extern "C" int iemic_newton_step(iemic_ctx* c, const iemic_krylov* opt, iemic_newton_info* info)
{
    CTX_CHECK(c);
    if (!opt) return IEMIC_EINVAL;
    iemic_newton_info inf{};
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    auto T0 = clk::now();
    const int64_t N = c->nrows;
    const unsigned G = (unsigned)std::min<int64_t>((N + 255) / 256, 2048);
    auto t = clk::now();
    int rc = assemble_rhs(c, c->d_x.p, c->d_F.p);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    inf.t_rhs_ms += ms(t);
    inf.norm_f0 = std::sqrt(std::max(0.0, dot(c, c->d_F.p, c->d_F.p, N)));
    t = clk::now();
    if ((rc = assemble_jacobian(c, c->d_x.p))) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    inf.t_jac_ms = ms(t);
    t = clk::now();
    if (opt->prec > 0) {
        if ((rc = prec_compute(c, opt))) return rc;
        HIP_OK(hipStreamSynchronize(c->stream));
    }
    inf.t_prec_ms = ms(t);
    hipLaunchKernelGGL(k_neg, dim3(G), dim3(256), 0, c->stream, c->d_F.p, c->d_tmp1.p, N);
    t = clk::now();
    if ((rc = fgmres(c, c->d_tmp1.p, c->d_tmp2.p, opt, &inf.solve))) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    inf.t_solve_ms = ms(t);
    hipLaunchKernelGGL(k_newton_update, dim3(G), dim3(256), 0, c->stream, c->d_x.p, c->d_tmp2.p, N);
    t = clk::now();
    if ((rc = assemble_rhs(c, c->d_x.p, c->d_F.p))) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    inf.t_rhs_ms += ms(t);
    inf.norm_f1 = std::sqrt(std::max(0.0, dot(c, c->d_F.p, c->d_F.p, N)));
    c->jac_valid = 1;
    inf.t_total_ms = ms(T0);
    if (info) *info = inf;
    return 0;
}

extern "C" int iemic_time_spmv(iemic_ctx* c, int nrep, double* ms_per_launch)
{
    CTX_CHECK(c);
    if (!c->jac_valid || nrep < 1) return IEMIC_ESTATE;
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    int rc = spmv(c, c->d_x.p, c->d_tmp2.p, c->stream); /* warm */
    if (rc) return rc;
    HIP_OK(hipEventRecord(e0, c->stream));
    for (int r = 0; r < nrep; r++) {
        rc = spmv(c, c->d_x.p, c->d_tmp2.p, c->stream);
        if (rc) return rc;
    }
    HIP_OK(hipEventRecord(e1, c->stream));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    *ms_per_launch = ms / nrep;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}
