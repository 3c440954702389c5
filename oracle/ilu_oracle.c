/*
 * ilu_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of the block ILU(0) of
 * i-emic_amd/csrc/ilu.hip (the build's replacement for the reference's MRILU seam,
 * src/mrilucpp/Ifpack_MRILU.cpp:22-39): same block pattern (bs x bs blocks of a 0-based
 * CSR, diagonal block always present), IKJ elimination without fill, pivot blocks inverted
 * by Gauss-Jordan with partial pivoting, unit-lower / block-upper solves.  Sequential; the
 * checker of the GPU factor and apply.  The reference's MRILU itself is not restated
 * (multilevel ILU, parity unpinned for this row).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int n, bs, nb, perturbed;
    int *rp, *cl, *dg;
    double *val, *dinv;
} oilu_t;

static int cmpint(const void* a, const void* b) { return *(const int*)a - *(const int*)b; }

void orc_ilu_destroy(void* h)
{
    oilu_t* f = (oilu_t*)h;
    if (!f) return;
    free(f->rp); free(f->cl); free(f->dg); free(f->val); free(f->dinv);
    free(f);
}

static int inv_gj(const double* A, double* X, int bs)
{
    int zero = 0;
    double a[64];
    memcpy(a, A, sizeof(double) * bs * bs);
    memset(X, 0, sizeof(double) * bs * bs);
    for (int e = 0; e < bs; e++) X[e * bs + e] = 1.0;
    for (int k = 0; k < bs; k++) {
        int p = k;
        for (int i = k + 1; i < bs; i++)
            if (fabs(a[i * bs + k]) > fabs(a[p * bs + k])) p = i;
        if (a[p * bs + k] == 0.0) { p = k; a[k * bs + k] = 1.0; zero++; }
        if (p != k)
            for (int j = 0; j < bs; j++) {
                double t = a[p * bs + j]; a[p * bs + j] = a[k * bs + j]; a[k * bs + j] = t;
                t = X[p * bs + j]; X[p * bs + j] = X[k * bs + j]; X[k * bs + j] = t;
            }
        const double iv = 1.0 / a[k * bs + k];
        for (int j = 0; j < bs; j++) { a[k * bs + j] *= iv; X[k * bs + j] *= iv; }
        for (int i = 0; i < bs; i++) {
            if (i == k) continue;
            const double fct = a[i * bs + k];
            if (fct == 0.0) continue;
            for (int j = 0; j < bs; j++) { a[i * bs + j] -= fct * a[k * bs + j]; X[i * bs + j] -= fct * X[k * bs + j]; }
        }
    }
    return zero;
}

/* factorised handle, or NULL (bad arguments or a singular pivot block) */
void* orc_ilu_create(int n, const int64_t* rowptr, const int* col, const double* val, int bs)
{
    if (bs < 1 || bs > 8 || n % bs) return NULL;
    oilu_t* f = (oilu_t*)calloc(1, sizeof(oilu_t));
    f->n = n; f->bs = bs; f->nb = n / bs;
    const int nb = f->nb, bb = bs * bs;
    f->rp = (int*)calloc(nb + 1, sizeof(int));
    int cap = 64, cnt = 0;
    f->cl = (int*)malloc(sizeof(int) * cap);
    int* mark = (int*)malloc(sizeof(int) * nb);
    int* tmp = (int*)malloc(sizeof(int) * (nb + 1));
    for (int i = 0; i < nb; i++) mark[i] = -1;
    for (int I = 0; I < nb; I++) {
        int nt = 0;
        for (int r = I * bs; r < (I + 1) * bs; r++)
            for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) {
                if (col[p] < 0 || col[p] >= n) continue;
                const int J = col[p] / bs;
                if (mark[J] != I) { mark[J] = I; tmp[nt++] = J; }
            }
        if (mark[I] != I) { mark[I] = I; tmp[nt++] = I; }
        qsort(tmp, nt, sizeof(int), cmpint);
        if (cnt + nt > cap) { while (cnt + nt > cap) cap *= 2; f->cl = (int*)realloc(f->cl, sizeof(int) * cap); }
        memcpy(f->cl + cnt, tmp, sizeof(int) * nt);
        cnt += nt;
        f->rp[I + 1] = cnt;
    }
    free(mark); free(tmp);
    f->dg = (int*)malloc(sizeof(int) * nb);
    f->val = (double*)calloc((size_t)cnt * bb, sizeof(double));
    f->dinv = (double*)calloc((size_t)nb * bb, sizeof(double));
    for (int I = 0; I < nb; I++) {
        for (int p = f->rp[I]; p < f->rp[I + 1]; p++)
            if (f->cl[p] == I) f->dg[I] = p;
        for (int r = I * bs; r < (I + 1) * bs; r++)
            for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) {
                if (col[p] < 0 || col[p] >= n) continue;
                const int J = col[p] / bs;
                int lo = f->rp[I], hi = f->rp[I + 1] - 1, pos = -1;
                while (lo <= hi) { int mid = (lo + hi) / 2; if (f->cl[mid] == J) { pos = mid; break; } if (f->cl[mid] < J) lo = mid + 1; else hi = mid - 1; }
                f->val[(size_t)pos * bb + (r - I * bs) * bs + (col[p] - J * bs)] += val[p];
            }
    }
    double tmpb[64];
    for (int I = 0; I < nb; I++) {
        for (int p = f->rp[I]; p < f->dg[I]; p++) {
            const int K = f->cl[p];
            double* aik = f->val + (size_t)p * bb;
            const double* dk = f->dinv + (size_t)K * bb;
            for (int r = 0; r < bs; r++)
                for (int c = 0; c < bs; c++) {
                    double v = 0.0;
                    for (int t = 0; t < bs; t++) v += aik[r * bs + t] * dk[t * bs + c];
                    tmpb[r * bs + c] = v;
                }
            memcpy(aik, tmpb, sizeof(double) * bb);
            int a = p + 1, b = f->dg[K] + 1;
            while (a < f->rp[I + 1] && b < f->rp[K + 1]) {
                if (f->cl[a] < f->cl[b]) a++;
                else if (f->cl[a] > f->cl[b]) b++;
                else {
                    double* aij = f->val + (size_t)a * bb;
                    const double* akj = f->val + (size_t)b * bb;
                    for (int r = 0; r < bs; r++)
                        for (int c = 0; c < bs; c++) {
                            double s = 0.0;
                            for (int t = 0; t < bs; t++) s += aik[r * bs + t] * akj[t * bs + c];
                            aij[r * bs + c] -= s;
                        }
                    a++; b++;
                }
            }
        }
        f->perturbed += inv_gj(f->val + (size_t)f->dg[I] * bb, f->dinv + (size_t)I * bb, bs);
    }
    return f;
}

void orc_ilu_apply(void* h, const double* rhs, double* sol)
{
    oilu_t* f = (oilu_t*)h;
    const int bs = f->bs, bb = bs * bs, nb = f->nb;
    double* y = (double*)malloc(sizeof(double) * f->n);
    double t[8];
    for (int I = 0; I < nb; I++) {
        for (int r = 0; r < bs; r++) t[r] = rhs[I * bs + r];
        for (int p = f->rp[I]; p < f->dg[I]; p++) {
            const int K = f->cl[p];
            const double* a = f->val + (size_t)p * bb;
            for (int r = 0; r < bs; r++)
                for (int c = 0; c < bs; c++) t[r] -= a[r * bs + c] * y[K * bs + c];
        }
        for (int r = 0; r < bs; r++) y[I * bs + r] = t[r];
    }
    for (int I = nb - 1; I >= 0; I--) {
        for (int r = 0; r < bs; r++) t[r] = y[I * bs + r];
        for (int p = f->dg[I] + 1; p < f->rp[I + 1]; p++) {
            const int J = f->cl[p];
            const double* a = f->val + (size_t)p * bb;
            for (int r = 0; r < bs; r++)
                for (int c = 0; c < bs; c++) t[r] -= a[r * bs + c] * sol[J * bs + c];
        }
        const double* di = f->dinv + (size_t)I * bb;
        for (int r = 0; r < bs; r++) {
            double s = 0.0;
            for (int c = 0; c < bs; c++) s += di[r * bs + c] * t[c];
            sol[I * bs + r] = s;
        }
    }
    free(y);
}

int orc_ilu_perturbed(void* h) { return ((oilu_t*)h)->perturbed; }
