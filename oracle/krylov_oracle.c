/*
 * krylov_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU baseline + checker).
 *
 * CPU restatement of the linear-solve half of the Newton step:
 *  - 6x6 cell-block CSR built from the point Jacobian on the maximal graph
 *    (the Epetra_CrsMatrix of THCM.C:745 viewed cell-wise),
 *  - block ILU(0) under an arbitrary cell ordering (the preconditioner the build uses in
 *    place of TRIOS::BlockPreconditioner + ML/MRILU),
 *  - right-preconditioned flexible GMRES with classical Gram-Schmidt + one
 *    re-orthogonalisation pass (Belos BlockGmresSolMgr semantics used by
 *    Ocean::solve, src/ocean/Ocean.C:961-1137: "Flexible Gmres", DGKS, implicit residual
 *    scaled by the initial residual, x0 = 0), Givens least squares as in
 *    src/gmressolver/GMRESSolver.H:81-255.
 */
#include "thcm_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NB 6
#define BB 36

/* ---- block CSR -------------------------------------------------------------- */
/* Build the cell-block pattern from a point CSR with 6 rows per cell.  Returns number
 * of blocks; fills bptr (ncell+1), bcol (cap), bval (cap*36, row-major per block). */
int64_t orc_bcsr_build(int ncell, const int64_t* rowptr, const int* col, const double* val,
                       int64_t* bptr, int* bcol, double* bval, int64_t cap)
{
    int64_t nb = 0;
    int* mark = (int*)malloc(sizeof(int) * ncell);
    for (int c = 0; c < ncell; c++) mark[c] = -1;
    int* list = (int*)malloc(sizeof(int) * 4096);
    for (int c = 0; c < ncell; c++) {
        int cnt = 0;
        for (int r = 0; r < NB; r++) {
            int row = c * NB + r;
            for (int64_t p = rowptr[row]; p < rowptr[row + 1]; p++) {
                int cc = col[p] / NB;
                if (mark[cc] != c) { mark[cc] = c; list[cnt++] = cc; }
            }
        }
        /* diagonal block always present */
        if (mark[c] != c) { mark[c] = c; list[cnt++] = c; }
        for (int a = 1; a < cnt; a++) {
            int v = list[a], b = a - 1;
            while (b >= 0 && list[b] > v) { list[b + 1] = list[b]; b--; }
            list[b + 1] = v;
        }
        if (bptr) bptr[c] = nb;
        for (int a = 0; a < cnt; a++) {
            if (bcol && nb < cap) {
                bcol[nb] = list[a];
                memset(bval + nb * BB, 0, sizeof(double) * BB);
            }
            nb++;
        }
    }
    if (bptr) bptr[ncell] = nb;
    if (bcol && bval && nb <= cap) {
        for (int c = 0; c < ncell; c++)
            for (int r = 0; r < NB; r++) {
                int row = c * NB + r;
                for (int64_t p = rowptr[row]; p < rowptr[row + 1]; p++) {
                    int cc = col[p] / NB, cr = col[p] % NB;
                    int64_t lo = bptr[c], hi = bptr[c + 1] - 1;
                    while (lo < hi) {
                        int64_t mid = (lo + hi) / 2;
                        if (bcol[mid] < cc) lo = mid + 1; else hi = mid;
                    }
                    bval[lo * BB + r * NB + cr] += val[p];
                }
            }
    }
    free(mark);
    free(list);
    return nb;
}

static int inv6(const double* A, double* Ainv)
{
    double M[NB][2 * NB];
    for (int i = 0; i < NB; i++)
        for (int j = 0; j < NB; j++) {
            M[i][j] = A[i * NB + j];
            M[i][NB + j] = (i == j) ? 1.0 : 0.0;
        }
    for (int k = 0; k < NB; k++) {
        int piv = k;
        double best = fabs(M[k][k]);
        for (int i = k + 1; i < NB; i++)
            if (fabs(M[i][k]) > best) { best = fabs(M[i][k]); piv = i; }
        if (best == 0.0) return -1;
        if (piv != k)
            for (int j = 0; j < 2 * NB; j++) { double t = M[k][j]; M[k][j] = M[piv][j]; M[piv][j] = t; }
        double d = 1.0 / M[k][k];
        for (int j = 0; j < 2 * NB; j++) M[k][j] *= d;
        for (int i = 0; i < NB; i++)
            if (i != k) {
                double f = M[i][k];
                if (f != 0.0)
                    for (int j = 0; j < 2 * NB; j++) M[i][j] -= f * M[k][j];
            }
    }
    for (int i = 0; i < NB; i++)
        for (int j = 0; j < NB; j++) Ainv[i * NB + j] = M[i][NB + j];
    return 0;
}

static inline void mm6(const double* A, const double* B, double* C) /* C = A*B */
{
    for (int i = 0; i < NB; i++)
        for (int j = 0; j < NB; j++) {
            double s = 0.0;
            for (int k = 0; k < NB; k++) s += A[i * NB + k] * B[k * NB + j];
            C[i * NB + j] = s;
        }
}

/* Block ILU(0) in the order given by rank[cell] (position of the cell in the
 * elimination order).  On exit bval holds L (strictly lower, unit diagonal implied)
 * and U (upper), and dinv[c*36] the inverse of the pivot block.  Returns 0 or the
 * (1+cell) of a singular pivot. */
int orc_bilu0_factor(int ncell, const int64_t* bptr, const int* bcol, double* bval,
                     const int* order, const int* rank, double* dinv)
{
    double tmp[BB];
    int64_t maxrow = 0;
    for (int c = 0; c < ncell; c++)
        if (bptr[c + 1] - bptr[c] > maxrow) maxrow = bptr[c + 1] - bptr[c];
    int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (maxrow + 1));
    for (int q = 0; q < ncell; q++) {
        int i = order[q];
        int64_t b = bptr[i], e = bptr[i + 1];
        int nk = (int)(e - b);
        /* L blocks sorted by rank */
        int nl = 0;
        for (int64_t p = b; p < e; p++)
            if (rank[bcol[p]] < q) idx[nl++] = p;
        for (int a = 1; a < nl; a++) {
            int64_t v = idx[a];
            int c = a - 1;
            while (c >= 0 && rank[bcol[idx[c]]] > rank[bcol[v]]) { idx[c + 1] = idx[c]; c--; }
            idx[c + 1] = v;
        }
        (void)nk;
        for (int a = 0; a < nl; a++) {
            int64_t pik = idx[a];
            int k = bcol[pik];
            mm6(bval + pik * BB, dinv + (int64_t)k * BB, tmp);
            memcpy(bval + pik * BB, tmp, sizeof(tmp));
            /* A_ij -= L_ik U_kj for j in row i with rank[j] > rank[k] */
            for (int64_t pj = b; pj < e; pj++) {
                int j = bcol[pj];
                if (rank[j] <= rank[k]) continue;
                int64_t lo = bptr[k], hi = bptr[k + 1] - 1, hit = -1;
                while (lo <= hi) {
                    int64_t mid = (lo + hi) / 2;
                    if (bcol[mid] == j) { hit = mid; break; }
                    if (bcol[mid] < j) lo = mid + 1; else hi = mid - 1;
                }
                if (hit < 0) continue;
                double prod[BB];
                mm6(bval + pik * BB, bval + hit * BB, prod);
                for (int t = 0; t < BB; t++) bval[pj * BB + t] -= prod[t];
            }
        }
        int64_t pd = -1;
        for (int64_t p = b; p < e; p++)
            if (bcol[p] == i) pd = p;
        if (inv6(bval + pd * BB, dinv + (int64_t)i * BB)) { free(idx); return i + 1; }
    }
    free(idx);
    return 0;
}

void orc_bilu0_apply(int ncell, const int64_t* bptr, const int* bcol, const double* bval,
                     const int* order, const int* rank, const double* dinv, const double* r,
                     double* z)
{
    double* y = z;
    for (int q = 0; q < ncell; q++) {
        int i = order[q];
        double s[NB];
        for (int t = 0; t < NB; t++) s[t] = r[i * NB + t];
        for (int64_t p = bptr[i]; p < bptr[i + 1]; p++) {
            int k = bcol[p];
            if (rank[k] >= q) continue;
            const double* L = bval + p * BB;
            for (int a = 0; a < NB; a++) {
                double acc = 0.0;
                for (int c = 0; c < NB; c++) acc += L[a * NB + c] * y[k * NB + c];
                s[a] -= acc;
            }
        }
        for (int t = 0; t < NB; t++) y[i * NB + t] = s[t];
    }
    for (int q = ncell - 1; q >= 0; q--) {
        int i = order[q];
        double s[NB];
        for (int t = 0; t < NB; t++) s[t] = y[i * NB + t];
        for (int64_t p = bptr[i]; p < bptr[i + 1]; p++) {
            int j = bcol[p];
            if (rank[j] <= q) continue;
            const double* U = bval + p * BB;
            for (int a = 0; a < NB; a++) {
                double acc = 0.0;
                for (int c = 0; c < NB; c++) acc += U[a * NB + c] * z[j * NB + c];
                s[a] -= acc;
            }
        }
        const double* D = dinv + (int64_t)i * BB;
        for (int a = 0; a < NB; a++) {
            double acc = 0.0;
            for (int c = 0; c < NB; c++) acc += D[a * NB + c] * s[c];
            z[i * NB + a] = acc;
        }
    }
}

/* ---- preconditioners behind one callback --------------------------------------- */
typedef void (*orc_prec_fn)(const void* ctx, const double* r, double* z);

typedef struct {
    int ncell;
    const int64_t* bptr;
    const int *bcol, *order, *rank;
    const double *bval, *dinv;
} bilu_t;

static void bilu_apply_cb(const void* ctx, const double* r, double* z)
{
    const bilu_t* s = (const bilu_t*)ctx;
    orc_bilu0_apply(s->ncell, s->bptr, s->bcol, s->bval, s->order, s->rank, s->dinv, r, z);
}

/* Block Jacobi: inverse of each cell's 6x6 diagonal block (identity if singular) --
 * the CPU twin of prec.hip k_bj_compute/k_bj_apply. */
void orc_bj_compute(int ncell, const int64_t* rowptr, const int* col, const double* val,
                    double* dinv)
{
#pragma omp parallel for schedule(static)
    for (int cell = 0; cell < ncell; cell++) {
        double A[BB] = {0};
        for (int a = 0; a < NB; a++) {
            const int64_t row = (int64_t)cell * NB + a;
            for (int64_t p = rowptr[row]; p < rowptr[row + 1]; p++) {
                const int c = col[p];
                if (c / NB == cell) A[a * NB + c % NB] += val[p];
            }
        }
        double* D = dinv + (int64_t)cell * BB;
        if (inv6(A, D)) {
            for (int q = 0; q < BB; q++) D[q] = 0.0;
            for (int a = 0; a < NB; a++) D[a * NB + a] = 1.0;
        }
    }
}

typedef struct {
    int ncell;
    const double* dinv;
} bj_t;

static void bj_apply_cb(const void* ctx, const double* r, double* z)
{
    const bj_t* s = (const bj_t*)ctx;
#pragma omp parallel for schedule(static)
    for (int cell = 0; cell < s->ncell; cell++) {
        const double* D = s->dinv + (int64_t)cell * BB;
        for (int a = 0; a < NB; a++) {
            double acc = 0.0;
            for (int c = 0; c < NB; c++) acc += D[a * NB + c] * r[(int64_t)cell * NB + c];
            z[(int64_t)cell * NB + a] = acc;
        }
    }
}

void orc_bj_apply(int ncell, const double* dinv, const double* r, double* z)
{
    bj_t s = {ncell, dinv};
    bj_apply_cb(&s, r, z);
}

static double dot(int n, const double* a, const double* b)
{
    double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}

/* Right-preconditioned FGMRES(m) with restarts, CGS2.  Tolerance relative to ||b||
 * (x0 = 0).  Returns iterations; *relres = ||b - A x|| / ||b|| (true residual). */
static int fgmres_core(int N, const int64_t* rowptr, const int* col, const double* val,
                       orc_prec_fn prec, const void* pctx, const double* b, double* x,
                       double tol, int m, int maxit, double* relres, double* hist)
{
    double* V = (double*)malloc(sizeof(double) * (size_t)N * (m + 1));
    double* Z = (double*)malloc(sizeof(double) * (size_t)N * m);
    double* H = (double*)calloc((size_t)(m + 1) * m, sizeof(double));
    double* cs = (double*)malloc(sizeof(double) * m);
    double* sn = (double*)malloc(sizeof(double) * m);
    double* g = (double*)malloc(sizeof(double) * (m + 1));
    double* hcol = (double*)malloc(sizeof(double) * (m + 1));
    double* r = (double*)malloc(sizeof(double) * N);
    memset(x, 0, sizeof(double) * N);
    double bnorm = sqrt(dot(N, b, b));
    if (bnorm == 0.0) bnorm = 1.0;
    int it = 0;
    double res = 1.0;
    while (it < maxit) {
        /* r = b - A x */
        orc_csr_spmv(N, rowptr, col, val, x, r);
        for (int i = 0; i < N; i++) r[i] = b[i] - r[i];
        double beta = sqrt(dot(N, r, r));
        res = beta / bnorm;
        if (res <= tol) break;
        for (int i = 0; i < N; i++) V[i] = r[i] / beta;
        memset(g, 0, sizeof(double) * (m + 1));
        g[0] = beta;
        int j;
        for (j = 0; j < m && it < maxit; j++, it++) {
            double* vj = V + (size_t)j * N;
            double* zj = Z + (size_t)j * N;
            double* w = V + (size_t)(j + 1) * N;
            if (prec) prec(pctx, vj, zj);
            else memcpy(zj, vj, sizeof(double) * N);
            orc_csr_spmv(N, rowptr, col, val, zj, w);
            for (int i = 0; i <= j; i++) hcol[i] = 0.0;
            for (int pass = 0; pass < 2; pass++) {
                for (int i = 0; i <= j; i++) {
                    double h = dot(N, V + (size_t)i * N, w);
                    hcol[i] += h;
                }
                /* CGS: subtract with the coefficients of this pass */
                for (int i = 0; i <= j; i++) {
                    double h = pass == 0 ? hcol[i] : hcol[i] - H[(size_t)i * m + j];
                    const double* vi = V + (size_t)i * N;
#pragma omp parallel for schedule(static)
                    for (int q = 0; q < N; q++) w[q] -= h * vi[q];
                }
                for (int i = 0; i <= j; i++) H[(size_t)i * m + j] = hcol[i];
            }
            double hn = sqrt(dot(N, w, w));
            H[(size_t)(j + 1) * m + j] = hn;
            if (hn > 0)
                for (int q = 0; q < N; q++) w[q] /= hn;
            /* Givens */
            for (int i = 0; i < j; i++) {
                double a = H[(size_t)i * m + j], c = H[(size_t)(i + 1) * m + j];
                H[(size_t)i * m + j] = cs[i] * a + sn[i] * c;
                H[(size_t)(i + 1) * m + j] = -sn[i] * a + cs[i] * c;
            }
            double a = H[(size_t)j * m + j], c = H[(size_t)(j + 1) * m + j];
            double d = sqrt(a * a + c * c);
            cs[j] = a / d;
            sn[j] = c / d;
            H[(size_t)j * m + j] = d;
            H[(size_t)(j + 1) * m + j] = 0.0;
            g[j + 1] = -sn[j] * g[j];
            g[j] = cs[j] * g[j];
            res = fabs(g[j + 1]) / bnorm;
            if (hist) hist[it] = res;
            if (res <= tol) { j++; it++; break; }
        }
        /* solve H y = g, x += Z y */
        int k = j;
        double* y = hcol;
        for (int i = k - 1; i >= 0; i--) {
            double t = g[i];
            for (int q = i + 1; q < k; q++) t -= H[(size_t)i * m + q] * y[q];
            y[i] = t / H[(size_t)i * m + i];
        }
        for (int i = 0; i < k; i++) {
            const double* zi = Z + (size_t)i * N;
            for (int q = 0; q < N; q++) x[q] += y[i] * zi[q];
        }
        if (res <= tol) break;
    }
    orc_csr_spmv(N, rowptr, col, val, x, r);
    for (int i = 0; i < N; i++) r[i] = b[i] - r[i];
    *relres = sqrt(dot(N, r, r)) / bnorm;
    free(V); free(Z); free(H); free(cs); free(sn); free(g); free(hcol); free(r);
    return it;
}

int orc_fgmres(int ncell, const int64_t* rowptr, const int* col, const double* val,
               const int64_t* bptr, const int* bcol, const double* bval, const int* order,
               const int* rank, const double* dinv, const double* b, double* x, double tol,
               int m, int maxit, double* relres, double* hist)
{
    bilu_t s = {ncell, bptr, bcol, order, rank, bval, dinv};
    return fgmres_core(ncell * NB, rowptr, col, val, bval ? bilu_apply_cb : NULL, &s, b, x, tol,
                       m, maxit, relres, hist);
}

/* FGMRES with the block-Jacobi preconditioner (dinv from orc_bj_compute) */
int orc_fgmres_bj(int ncell, const int64_t* rowptr, const int* col, const double* val,
                  const double* dinv, const double* b, double* x, double tol, int m, int maxit,
                  double* relres, double* hist)
{
    bj_t s = {ncell, dinv};
    return fgmres_core(ncell * NB, rowptr, col, val, bj_apply_cb, &s, b, x, tol, m, maxit,
                       relres, hist);
}

/* FGMRES with the block Gauss-Seidel preconditioner of prec_oracle.c */
void orc_gs_apply(void* h, const double* r, double* z);
static void gs_apply_cb(const void* ctx, const double* r, double* z)
{
    orc_gs_apply((void*)ctx, r, z);
}
int orc_fgmres_gs(int ncell, const int64_t* rowptr, const int* col, const double* val, void* gs,
                  const double* b, double* x, double tol, int m, int maxit, double* relres,
                  double* hist)
{
    return fgmres_core(ncell * NB, rowptr, col, val, gs_apply_cb, gs, b, x, tol, m, maxit, relres,
                       hist);
}
