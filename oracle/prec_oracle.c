/*
 * prec_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of the block Gauss-Seidel
 * preconditioner of i-emic_amd/csrc/prec_gs.hip, written independently on the
 * Epetra-shaped CSR Jacobian (entries looked up by (row, column)), with the 2-D Schur
 * complement solved by a band LU per application instead of the GPU's dense inverse.
 * It is the checker for the GPU's prec apply and the preconditioner of the CPU
 * baseline's FGMRES.  This is the build's own preconditioner design (the reference's
 * TRIOS/MRILU path cannot be built here), so its parity is against this restatement,
 * not against the reference: "parity unpinned" w.r.t. the reference for this row.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { NUN = 6, UU = 0, VV = 1, WW = 2, PP = 3, TT = 4, SS = 5 };

typedef struct {
    int n, m, l, periodic, ts_sweeps;
    int64_t N, ncell;
    const int64_t* rowptr;
    const int* col;
    const double* val;
    int64_t rowintcon;
    int int_sign;
    const double* intc;
    uint8_t* known;
    /* columns */
    int ncol, bl, bu;
    int* colid;      /* j*n+i -> index */
    int* ij_of_col;
    uint8_t* pinned;
    double* band;    /* row-wise LU factors, width 2bl+bu+1 */
    double* band0;   /* the Schur band before the LU (exported for studies/tests) */
    int* piv;
    double *uvinv, *tsinv, *pw, *rr, *bts, *colv;
} gs_t;

static double A(const gs_t* g, int64_t row, int64_t c)
{
    int64_t lo = g->rowptr[row], hi = g->rowptr[row + 1] - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) / 2;
        int cm = g->col[mid];
        if (cm == c) return g->val[mid];
        if (cm < c) lo = mid + 1;
        else hi = mid - 1;
    }
    return 0.0;
}
static int64_t cel(const gs_t* g, int i, int j, int k) { return ((int64_t)k * g->m + j) * g->n + i; }
static int wrap(const gs_t* g, int* i, int* j)
{
    if (*j < 0 || *j >= g->m) return 0;
    if (*i < 0 || *i >= g->n) {
        if (!g->periodic) return 0;
        *i = (*i + g->n) % g->n;
    }
    return 1;
}
static void inv2(double a, double b, double c, double d, int ia, int ib, double* o)
{
    o[0] = o[1] = o[2] = o[3] = 0.0;
    if (ia && ib) {
        double det = a * d - b * c;
        if (det != 0.0) { o[0] = d / det; o[1] = -b / det; o[2] = -c / det; o[3] = a / det; }
    } else if (ia) {
        if (a != 0.0) o[0] = 1.0 / a;
    } else if (ib) {
        if (d != 0.0) o[3] = 1.0 / d;
    }
}

static int cmp64(const void* a, const void* b)
{
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

void orc_gs_destroy(void* h)
{
    gs_t* g = (gs_t*)h;
    if (!g) return;
    free(g->known); free(g->colid); free(g->ij_of_col); free(g->pinned); free(g->band);
    free(g->piv); free(g->uvinv); free(g->tsinv); free(g->pw); free(g->rr); free(g->bts);
    free(g->colv); free(g->band0);
    free(g);
}

/* Returns NULL on a singular Schur complement. */
void* orc_gs_create(int n, int m, int l, int periodic, const int64_t* rowptr, const int* col,
                    const double* val, int64_t rowintcon, int int_sign, const double* intc,
                    int ts_sweeps)
{
    gs_t* g = (gs_t*)calloc(1, sizeof(gs_t));
    g->n = n; g->m = m; g->l = l; g->periodic = periodic; g->ts_sweeps = ts_sweeps;
    g->ncell = (int64_t)n * m * l;
    g->N = NUN * g->ncell;
    g->rowptr = rowptr; g->col = col; g->val = val;
    g->rowintcon = rowintcon; g->int_sign = int_sign; g->intc = intc;
    const int64_t N = g->N, nc = g->ncell;
    /* identity rows */
    g->known = (uint8_t*)calloc(N, 1);
    for (int64_t r = 0; r < N; r++) {
        int id = 1, diag = 0;
        for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) {
            if (col[p] == r) diag = val[p] == 1.0;
            else if (val[p] != 0.0) id = 0;
        }
        g->known[r] = (id && diag && r != rowintcon) ? 1 : 0;
    }
    uint8_t* kn = g->known;
    /* cell factors */
    g->uvinv = (double*)calloc(4 * nc, sizeof(double));
    g->tsinv = (double*)calloc(4 * nc, sizeof(double));
    g->pw = (double*)calloc(nc, sizeof(double));
    for (int64_t c = 0; c < nc; c++) {
        const int64_t u = NUN * c;
        inv2(A(g, u + UU, u + UU), A(g, u + UU, u + VV), A(g, u + VV, u + UU), A(g, u + VV, u + VV),
             !kn[u + UU], !kn[u + VV], g->uvinv + 4 * c);
        double sd = A(g, u + SS, u + SS), st = A(g, u + SS, u + TT);
        if (u + SS == rowintcon) { sd = int_sign * intc[u + SS]; st = 0.0; }
        inv2(A(g, u + TT, u + TT), A(g, u + TT, u + SS), st, sd, !kn[u + TT], !kn[u + SS],
             g->tsinv + 4 * c);
        if (!kn[u + PP]) {
            const int64_t below = c - (int64_t)n * m;
            double a = A(g, u + PP, u + WW);
            double b = below >= 0 ? A(g, u + PP, NUN * below + WW) : 0.0;
            if (!kn[u + WW] && a != 0.0) g->pw[c] = 1.0 / a;
            else if (below >= 0 && !kn[NUN * below + WW] && b != 0.0) g->pw[c] = -1.0 / b;
            else g->pw[c] = 1.0;
        }
    }
    /* water columns in band order (periodic: i folded 0,n-1,1,n-2,...; j fastest) */
    g->colid = (int*)malloc(sizeof(int) * n * m);
    int* ipos = (int*)malloc(sizeof(int) * n);
    if (periodic) {
        int a = 0, b = n - 1, q = 0;
        while (a <= b) { ipos[a] = q++; if (a != b) ipos[b] = q++; a++; b--; }
    } else
        for (int i = 0; i < n; i++) ipos[i] = i;
    int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * n * m);
    int ncol = 0;
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++) {
            g->colid[j * n + i] = -1;
            int act = 0;
            for (int k = 0; k < l && !act; k++) act = !kn[NUN * cel(g, i, j, k) + PP];
            if (act) keys[ncol++] = ((int64_t)ipos[i] * m + j) * ((int64_t)n * m) + (j * n + i);
        }
    qsort(keys, ncol, sizeof(int64_t), cmp64);
    g->ncol = ncol;
    g->ij_of_col = (int*)malloc(sizeof(int) * (ncol ? ncol : 1));
    for (int q = 0; q < ncol; q++) {
        g->ij_of_col[q] = (int)(keys[q] % ((int64_t)n * m));
        g->colid[g->ij_of_col[q]] = q;
    }
    free(keys);
    free(ipos);
    /* U/V point active at some level */
    uint8_t* uva = (uint8_t*)calloc(n * m, 1);
    for (int j = 0; j < m; j++)
        for (int i = 0; i < n; i++)
            for (int k = 0; k < l; k++) {
                int64_t c = cel(g, i, j, k);
                if (!kn[NUN * c + UU] || !kn[NUN * c + VV]) { uva[j * n + i] = 1; break; }
            }
    /* adjacency (sharing an active corner), bandwidth, basins + pins */
    int* adj = (int*)malloc(sizeof(int) * 9 * (ncol ? ncol : 1));
    int* nadj = (int*)calloc(ncol ? ncol : 1, sizeof(int));
    int bw = 0;
    for (int q = 0; q < ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        for (int dj = -1; dj <= 1; dj++)
            for (int di = -1; di <= 1; di++) {
                int ti = i + di, tj = j + dj;
                if (!wrap(g, &ti, &tj)) continue;
                int q2 = g->colid[tj * n + ti];
                if (q2 < 0 || q2 == q) continue;
                int shared = 0;
                for (int a = -1; a <= 0; a++)
                    for (int b = -1; b <= 0; b++) {
                        int e = di - a, f = dj - b;
                        if (e < 0 || e > 1 || f < 0 || f > 1) continue;
                        int qi = i + a, qj = j + b;
                        if (wrap(g, &qi, &qj) && uva[qj * n + qi]) shared = 1;
                    }
                if (!shared) continue;
                adj[9 * q + nadj[q]++] = q2;
                if (abs(q2 - q) > bw) bw = abs(q2 - q);
            }
    }
    g->pinned = (uint8_t*)calloc(ncol ? ncol : 1, 1);
    int* comp = (int*)malloc(sizeof(int) * (ncol ? ncol : 1));
    int* stack = (int*)malloc(sizeof(int) * (ncol ? ncol : 1));
    /* null space of the B-grid pressure Schur: constant on each connected set of
     * same-colour columns linked diagonally through an active U/V corner -> one pin each */
    for (int q = 0; q < ncol; q++) comp[q] = -1;
    for (int s = 0; s < ncol; s++) {
        if (comp[s] >= 0) continue;
        int sp = 0;
        stack[sp++] = s;
        comp[s] = s;
        g->pinned[s] = 1; /* band order: s is the component's first column */
        while (sp) {
            int q = stack[--sp];
            int qi0 = g->ij_of_col[q] % n, qj0 = g->ij_of_col[q] / n;
            for (int t = 0; t < nadj[q]; t++) {
                int q2 = adj[9 * q + t];
                int di = g->ij_of_col[q2] % n - qi0, dj = g->ij_of_col[q2] / n - qj0;
                if (di > 1) di -= n;
                if (di < -1) di += n;
                if (di == 0 || dj == 0) continue; /* other colour */
                if (comp[q2] < 0) { comp[q2] = s; stack[sp++] = q2; }
            }
        }
    }
    free(comp); free(stack); free(adj); free(nadj); free(uva);
    g->bl = g->bu = bw > 0 ? bw : 1;
    const int bl = g->bl, bu = g->bu, W = 2 * bl + bu + 1;
    /* Schur S = Mz2 Duv D^-1 Guv Mz1^T */
    g->band = (double*)calloc((size_t)(ncol ? ncol : 1) * W, sizeof(double));
    for (int q = 0; q < ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        double* row = g->band + (size_t)q * W;
        if (g->pinned[q]) { row[bl] = 1.0; continue; }
        for (int dj = -1; dj <= 1; dj++)
            for (int di = -1; di <= 1; di++) {
                int ti = i + di, tj = j + dj;
                if (!wrap(g, &ti, &tj)) continue;
                int q2 = g->colid[tj * n + ti];
                if (q2 < 0 || g->pinned[q2] || q2 - q < -bl || q2 - q > bl + bu) continue;
                double s = 0.0;
                for (int k = 0; k < l; k++) {
                    int64_t pc = cel(g, i, j, k), tc = cel(g, ti, tj, k);
                    if (kn[NUN * pc + PP] || kn[NUN * tc + PP]) continue;
                    double acc = 0.0;
                    for (int a = -1; a <= 0; a++)
                        for (int b = -1; b <= 0; b++) {
                            int e = di - a, f = dj - b;
                            if (e < 0 || e > 1 || f < 0 || f > 1) continue;
                            int qi = i + a, qj = j + b;
                            if (!wrap(g, &qi, &qj)) continue;
                            int64_t qc = cel(g, qi, qj, k);
                            int ua = !kn[NUN * qc + UU], va = !kn[NUN * qc + VV];
                            double du = ua ? A(g, NUN * pc + PP, NUN * qc + UU) : 0.0;
                            double dv = va ? A(g, NUN * pc + PP, NUN * qc + VV) : 0.0;
                            const double* D = g->uvinv + 4 * qc;
                            double yu = du * D[0] + dv * D[2], yv = du * D[1] + dv * D[3];
                            double gu = ua ? A(g, NUN * qc + UU, NUN * tc + PP) : 0.0;
                            double gv = va ? A(g, NUN * qc + VV, NUN * tc + PP) : 0.0;
                            acc += yu * gu + yv * gv;
                        }
                    s += g->pw[pc] * acc;
                }
                row[q2 - q + bl] += s;
            }
    }
    g->band0 = (double*)malloc(sizeof(double) * (size_t)(ncol ? ncol : 1) * W);
    memcpy(g->band0, g->band, sizeof(double) * (size_t)(ncol ? ncol : 1) * W);
    /* band LU, partial pivoting (same scheme as k_band_lu) */
    g->piv = (int*)malloc(sizeof(int) * (ncol ? ncol : 1));
    double* ab = g->band;
    for (int k = 0; k < ncol; k++) {
        int iend = k + bl < ncol - 1 ? k + bl : ncol - 1, jend = k + bl + bu < ncol - 1 ? k + bl + bu : ncol - 1;
        int p = k;
        double best = -1.0;
        for (int i = k; i <= iend; i++) {
            double v = fabs(ab[(size_t)i * W + (k - i + bl)]);
            if (v > best) { best = v; p = i; }
        }
        if (best == 0.0) { orc_gs_destroy(g); return NULL; }
        g->piv[k] = p;
        if (p != k)
            for (int j = k; j <= jend; j++) {
                double t = ab[(size_t)k * W + (j - k + bl)];
                ab[(size_t)k * W + (j - k + bl)] = ab[(size_t)p * W + (j - p + bl)];
                ab[(size_t)p * W + (j - p + bl)] = t;
            }
        double piv = ab[(size_t)k * W + bl];
        for (int i = k + 1; i <= iend; i++) {
            double lik = (ab[(size_t)i * W + (k - i + bl)] /= piv);
            if (lik == 0.0) continue;
            for (int j = k + 1; j <= jend; j++)
                ab[(size_t)i * W + (j - i + bl)] -= lik * ab[(size_t)k * W + (j - k + bl)];
        }
    }
    g->rr = (double*)calloc(N, sizeof(double));
    g->bts = (double*)calloc(N, sizeof(double));
    g->colv = (double*)calloc(ncol ? ncol : 1, sizeof(double));
    return g;
}

/* Duv uv at P cell pc */
static double duv_uv(const gs_t* g, int i, int j, int k, const double* z)
{
    const int64_t pc = cel(g, i, j, k);
    double acc = 0.0;
    for (int a = -1; a <= 0; a++)
        for (int b = -1; b <= 0; b++) {
            int qi = i + a, qj = j + b;
            if (!wrap(g, &qi, &qj)) continue;
            int64_t qc = cel(g, qi, qj, k);
            if (!g->known[NUN * qc + UU]) acc += A(g, NUN * pc + PP, NUN * qc + UU) * z[NUN * qc + UU];
            if (!g->known[NUN * qc + VV]) acc += A(g, NUN * pc + PP, NUN * qc + VV) * z[NUN * qc + VV];
        }
    return acc;
}

/* Guv p over the 4 P corners of the U/V point (i,j,k); p from z (ptil) or per column */
static void guv(const gs_t* g, int i, int j, int k, const double* z, const double* pcol, double* gu,
                double* gv)
{
    const int64_t qc = cel(g, i, j, k);
    *gu = *gv = 0.0;
    for (int e = 0; e <= 1; e++)
        for (int f = 0; f <= 1; f++) {
            int pi = i + e, pj = j + f;
            if (!wrap(g, &pi, &pj)) continue;
            int64_t pc = cel(g, pi, pj, k);
            if (g->known[NUN * pc + PP]) continue;
            double p;
            if (pcol) {
                int c = g->colid[pj * g->n + pi];
                if (c < 0) continue;
                p = pcol[c];
            } else
                p = z[NUN * pc + PP];
            *gu += A(g, NUN * qc + UU, NUN * pc + PP) * p;
            *gv += A(g, NUN * qc + VV, NUN * pc + PP) * p;
        }
}

void orc_gs_apply(void* h, const double* r, double* z)
{
    gs_t* g = (gs_t*)h;
    const int n = g->n, m = g->m, l = g->l;
    const int64_t N = g->N, nc = g->ncell;
    const uint8_t* kn = g->known;
    memset(z, 0, sizeof(double) * N);
    /* known rows and rr */
    for (int64_t row = 0; row < N; row++) {
        if (kn[row]) { z[row] = r[row]; g->rr[row] = 0.0; continue; }
        double acc = r[row];
        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++)
            if (kn[g->col[p]]) acc -= g->val[p] * r[g->col[p]];
        g->rr[row] = acc;
    }
    double* rr = g->rr;
    /* 1. ptil */
    for (int q = 0; q < g->ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        double pabove = 0.0;
        for (int k = l - 1; k >= 0; k--) {
            int64_t c = cel(g, i, j, k);
            int pa = !kn[NUN * c + PP];
            double p = 0.0;
            if (pa && k < l - 1 && !kn[NUN * c + WW]) {
                double g0 = A(g, NUN * c + WW, NUN * c + PP);
                double g1 = A(g, NUN * c + WW, NUN * cel(g, i, j, k + 1) + PP);
                if (g0 != 0.0) p = (rr[NUN * c + WW] - g1 * pabove) / g0;
            }
            if (pa) z[NUN * c + PP] = p;
            pabove = pa ? p : 0.0;
        }
    }
    /* 2. uv* */
    for (int64_t c = 0; c < nc; c++) {
        int ua = !kn[NUN * c + UU], va = !kn[NUN * c + VV];
        if (!ua && !va) continue;
        int i = (int)(c % n), j = (int)((c / n) % m), k = (int)(c / ((int64_t)n * m));
        double gu, gv;
        guv(g, i, j, k, z, NULL, &gu, &gv);
        double ru = ua ? rr[NUN * c + UU] - gu : 0.0, rv = va ? rr[NUN * c + VV] - gv : 0.0;
        const double* D = g->uvinv + 4 * c;
        if (ua) z[NUN * c + UU] = D[0] * ru + D[1] * rv;
        if (va) z[NUN * c + VV] = D[2] * ru + D[3] * rv;
    }
    /* 3. Schur rhs and band solve */
    for (int q = 0; q < g->ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        double s = 0.0;
        for (int k = 0; k < l; k++) {
            int64_t c = cel(g, i, j, k);
            if (kn[NUN * c + PP]) continue;
            s += g->pw[c] * (duv_uv(g, i, j, k, z) - rr[NUN * c + PP]);
        }
        g->colv[q] = g->pinned[q] ? 0.0 : s;
    }
    {
        const int ncol = g->ncol, bl = g->bl, bu = g->bu, W = 2 * bl + bu + 1;
        const double* ab = g->band;
        double* b = g->colv;
        for (int k = 0; k < ncol; k++) {
            int p = g->piv[k];
            if (p != k) { double t = b[k]; b[k] = b[p]; b[p] = t; }
            int iend = k + bl < ncol - 1 ? k + bl : ncol - 1;
            for (int i = k + 1; i <= iend; i++) b[i] -= ab[(size_t)i * W + (k - i + bl)] * b[k];
        }
        for (int i = ncol - 1; i >= 0; i--) {
            double s = b[i];
            int jend = i + bl + bu < ncol - 1 ? i + bl + bu : ncol - 1;
            for (int j = i + 1; j <= jend; j++) s -= ab[(size_t)i * W + (j - i + bl)] * b[j];
            b[i] = s / ab[(size_t)i * W + bl];
        }
    }
    /* 4. uv correction */
    for (int64_t c = 0; c < nc; c++) {
        int ua = !kn[NUN * c + UU], va = !kn[NUN * c + VV];
        if (!ua && !va) continue;
        int i = (int)(c % n), j = (int)((c / n) % m), k = (int)(c / ((int64_t)n * m));
        double gu, gv;
        guv(g, i, j, k, z, g->colv, &gu, &gv);
        if (!ua) gu = 0.0;
        if (!va) gv = 0.0;
        const double* D = g->uvinv + 4 * c;
        if (ua) z[NUN * c + UU] -= D[0] * gu + D[1] * gv;
        if (va) z[NUN * c + VV] -= D[2] * gu + D[3] * gv;
    }
    /* 4b/5. p and w */
    for (int q = 0; q < g->ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        double wbelow = 0.0;
        for (int k = 0; k < l; k++) {
            int64_t c = cel(g, i, j, k);
            int pa = !kn[NUN * c + PP], wa = !kn[NUN * c + WW];
            if (pa) z[NUN * c + PP] += g->colv[q];
            double w = 0.0;
            if (pa && wa) {
                double a = A(g, NUN * c + PP, NUN * c + WW);
                double b = k > 0 ? A(g, NUN * c + PP, NUN * cel(g, i, j, k - 1) + WW) : 0.0;
                double rhs = rr[NUN * c + PP] - duv_uv(g, i, j, k, z);
                if (a != 0.0) w = (rhs - b * wbelow) / a;
                z[NUN * c + WW] = w;
            } else if (wa)
                z[NUN * c + WW] = 0.0;
            wbelow = wa ? w : 0.0;
        }
    }
    /* 6. T/S */
    for (int64_t row = 0; row < N; row++) {
        int var = (int)(row % NUN);
        if (var < TT || kn[row]) continue;
        double acc = rr[row];
        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++) {
            int cv = g->col[p] % NUN;
            if (cv == TT || cv == SS || kn[g->col[p]]) continue;
            acc -= g->val[p] * z[g->col[p]];
        }
        g->bts[row] = acc;
        z[row] = 0.0;
    }
    /* colours: parity of i+j+k; odd periodic n: column n-1 gets colours 2/3 */
    const int four = g->periodic && (n & 1);
    const int seq2[4] = {0, 1, 1, 0}, seq4[8] = {0, 1, 2, 3, 3, 2, 1, 0};
    const int* seq = four ? seq4 : seq2;
    const int ns = four ? 8 : 4;
    int nsw = g->ts_sweeps > 1 ? g->ts_sweeps : 1;
    for (int sw = 0; sw < nsw; sw++)
        for (int hh = 0; hh < ns; hh++) {
            const int color = seq[hh];
#pragma omp parallel for schedule(static)
            for (int64_t c = 0; c < nc; c++) {
                int i = (int)(c % n), j = (int)((c / n) % m), k = (int)(c / ((int64_t)n * m));
                int cc = (four && i == n - 1) ? 2 + ((j + k) & 1) : ((i + j + k) & 1);
                if (cc != color) continue;
                int ta = !kn[NUN * c + TT], sa = !kn[NUN * c + SS];
                if (!ta && !sa) continue;
                double res[2] = {0.0, 0.0};
                for (int R = TT; R <= SS; R++) {
                    int64_t row = NUN * c + R;
                    if (kn[row]) continue;
                    double acc = g->bts[row];
                    if (row != g->rowintcon)
                        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++) {
                            int cl = g->col[p], cv = cl % NUN;
                            if (cv != TT && cv != SS) continue;
                            if (cl / NUN == c || kn[cl]) continue;
                            acc -= g->val[p] * z[cl];
                        }
                    res[R - TT] = acc;
                }
                const double* D = g->tsinv + 4 * c;
                if (ta) z[NUN * c + TT] = D[0] * res[0] + D[1] * res[1];
                if (sa) z[NUN * c + SS] = D[2] * res[0] + D[3] * res[1];
            }
        }
}

int orc_gs_ncol(void* h) { return ((gs_t*)h)->ncol; }
int orc_gs_band(void* h) { return ((gs_t*)h)->bl; }

/* the pinned Schur matrix before factorisation: band rows (width 2bl+bu+1, offset bl),
 * the (j*n+i) position and pin flag of every column */
void orc_gs_schur(void* h, double* band, int* ij_of_col, uint8_t* pinned)
{
    gs_t* g = (gs_t*)h;
    const size_t W = (size_t)(2 * g->bl + g->bu + 1);
    memcpy(band, g->band0, sizeof(double) * (size_t)g->ncol * W);
    memcpy(ij_of_col, g->ij_of_col, sizeof(int) * (size_t)g->ncol);
    memcpy(pinned, g->pinned, (size_t)g->ncol);
}
