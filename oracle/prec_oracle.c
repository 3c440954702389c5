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
    /* variant of prec_gs.hip's defaults: defect-correction passes on the dynamics block,
     * T/S by aggregation-multigrid V-cycles (orc_gs_config) */
    int dyn_iters, ts_mg;
    int ts_at;                       /* T/S right-hand side after this many dynamics passes */
    double dyn_omega;
    double *dres, *zc;
    int dyn_krylov;                  /* 1: the dynamics passes as right-preconditioned GMRES */
    int schur_passes;                /* passes that solve the Schur system: the first k - 1 and the last (0: all) */
    int schur_mask;                  /* study: bit k set = correction pass k solves it (0: schur_passes decides) */
    int skip_schur;
    double *kv, *kz;                 /* its basis (dyn_iters + 1) and M_D^-1 images (dyn_iters) */
    void* mg;
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

static void mg_free(void* p);

void orc_gs_destroy(void* h)
{
    gs_t* g = (gs_t*)h;
    if (!g) return;
    free(g->known); free(g->colid); free(g->ij_of_col); free(g->pinned); free(g->band);
    free(g->piv); free(g->uvinv); free(g->tsinv); free(g->pw); free(g->rr); free(g->bts);
    free(g->colv); free(g->band0); free(g->dres); free(g->zc); free(g->kv); free(g->kz);
    mg_free(g->mg);
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
    g->dyn_iters = 1;
    g->dyn_omega = 1.0;
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

/* dynamics block (steps 1-5): z at the active U/V/W/P rows from the right-hand side rr
 * (active rows; identity rows of z untouched) */
static void dyn_solve(gs_t* g, const double* rr, double* z)
{
    const int n = g->n, m = g->m, l = g->l;
    const int64_t nc = g->ncell;
    const uint8_t* kn = g->known;
    /* 1. ptil */
#pragma omp parallel for schedule(static)
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
#pragma omp parallel for schedule(static)
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
#pragma omp parallel for schedule(static)
    for (int q = 0; q < g->ncol; q++) {
        int i = g->ij_of_col[q] % n, j = g->ij_of_col[q] / n;
        double s = 0.0;
        for (int k = 0; k < l; k++) {
            int64_t c = cel(g, i, j, k);
            if (kn[NUN * c + PP]) continue;
            s += g->pw[c] * (duv_uv(g, i, j, k, z) - rr[NUN * c + PP]);
        }
        g->colv[q] = (g->pinned[q] || g->skip_schur) ? 0.0 : s;
    }
    if (!g->skip_schur) {
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
#pragma omp parallel for schedule(static)
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
#pragma omp parallel for schedule(static)
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
}

/* the dynamics rows of rr - A z (z: identity rows = r, T/S = 0), 0 elsewhere */
static void dyn_defect(gs_t* g, const double* z, double* d)
{
    const int64_t N = g->N;
#pragma omp parallel for schedule(static)
    for (int64_t row = 0; row < N; row++) {
        const int var = (int)(row % NUN);
        if (var > PP || g->known[row]) { d[row] = 0.0; continue; }
        double acc = g->rr[row];
        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++) {
            const int cl = g->col[p], cv = cl % NUN;
            if (cv > PP || g->known[cl]) continue;
            acc -= g->val[p] * z[cl];
        }
        d[row] = acc;
    }
}



/* ---- T/S aggregation multigrid (prec_gs.hip's mg_setup / mg_vcycle restated on the
 * CPU, one band): levels of n x m x l cells merging 2x2 horizontal neighbours over the
 * full depth, Galerkin coarse operators with piecewise-constant transfers, z-line
 * (block-tridiagonal along k) relaxation by horizontal colour, forward before and
 * backward after the coarse correction, a dense inverse on the coarsest level (<= 128
 * cells).  Cell index on every level: (j*l + k)*n + i. ------------------------------- */
enum { MG_MAXL = 12 };
typedef struct {
    int nlev, l, periodic;
    int n[MG_MAXL], m[MG_MAXL];
    double *off[MG_MAXL], *diag[MG_MAXL], *dinv[MG_MAXL], *b[MG_MAXL], *z[MG_MAXL];
    double* cinv;
} mg_t;

static void mg_free(void* p)
{
    mg_t* M = (mg_t*)p;
    if (!M) return;
    for (int q = 0; q < M->nlev; q++) {
        free(M->off[q]); free(M->diag[q]); free(M->dinv[q]); free(M->b[q]); free(M->z[q]);
    }
    free(M->cinv);
    free(M);
}

static int64_t mg_ncl(const mg_t* M, int q) { return (int64_t)M->n[q] * M->m[q] * M->l; }

/* neighbour q (-i,+i,-j,+j,-k,+k) of (i,j,k) on level lv; 0 outside */
static int mg_nb(const mg_t* M, int lv, int q, int* i, int* j, int* k)
{
    switch (q) {
    case 0: (*i)--; break;
    case 1: (*i)++; break;
    case 2: (*j)--; break;
    case 3: (*j)++; break;
    case 4: (*k)--; break;
    default: (*k)++; break;
    }
    if (*j < 0 || *j >= M->m[lv] || *k < 0 || *k >= M->l) return 0;
    if (*i < 0 || *i >= M->n[lv]) {
        if (!M->periodic) return 0;
        *i = (*i + M->n[lv]) % M->n[lv];
    }
    return 1;
}

/* Gauss-Jordan inverse with partial pivoting; rows without coupling become identity rows */
static void dense_inverse(double* A, int N, double* X)
{
    memset(X, 0, sizeof(double) * (size_t)N * N);
    for (int i = 0; i < N; i++) {
        X[(size_t)i * N + i] = 1.0;
        int any = 0;
        for (int j = 0; j < N; j++) any |= A[(size_t)i * N + j] != 0.0;
        if (!any) A[(size_t)i * N + i] = 1.0;
    }
    for (int k = 0; k < N; k++) {
        int p = k;
        for (int i = k + 1; i < N; i++)
            if (fabs(A[(size_t)i * N + k]) > fabs(A[(size_t)p * N + k])) p = i;
        if (p != k)
            for (int j = 0; j < N; j++) {
                double t = A[(size_t)p * N + j]; A[(size_t)p * N + j] = A[(size_t)k * N + j]; A[(size_t)k * N + j] = t;
                t = X[(size_t)p * N + j]; X[(size_t)p * N + j] = X[(size_t)k * N + j]; X[(size_t)k * N + j] = t;
            }
        const double d = A[(size_t)k * N + k];
        const double qd = d != 0.0 ? 1.0 / d : 0.0;
        for (int j = 0; j < N; j++) { A[(size_t)k * N + j] *= qd; X[(size_t)k * N + j] *= qd; }
#pragma omp parallel for schedule(static) if (N > 256)
        for (int i = 0; i < N; i++) {
            if (i == k) continue;
            const double f = A[(size_t)i * N + k];
            if (f == 0.0) continue;
            for (int j = 0; j < N; j++) {
                A[(size_t)i * N + j] -= f * A[(size_t)k * N + j];
                X[(size_t)i * N + j] -= f * X[(size_t)k * N + j];
            }
        }
    }
}

static void* mg_build(gs_t* g)
{
    const int n = g->n, m = g->m, l = g->l;
    mg_t* M = (mg_t*)calloc(1, sizeof(mg_t));
    M->l = l;
    M->periodic = g->periodic;
    int nn = n, mm = m, q = 0;
    M->n[0] = n; M->m[0] = m;
    /* the GPU's one-rank rule (prec_gs.hip mg_setup): stop at the first level of <= 1024
     * cells whose longitudes fit a cyclic-reduction block (2 mm l <= 192, >= 2 longitudes),
     * solved exactly (the GPU by whole-problem cyclic reduction, here Gauss-Jordan) */
#define MG_CR_OK(a, b) ((int64_t)(a) * (b) * l <= 1024 && 2 * (b) * l <= 192 && (a) >= 2)
    while (q + 1 < MG_MAXL && (q == 0 || (int64_t)nn * mm * l > 128) && (nn > 1 || mm > 1) &&
           !(q > 0 && MG_CR_OK(nn, mm))) {
        nn = (nn + 1) / 2; mm = (mm + 1) / 2; q++;
        M->n[q] = nn; M->m[q] = mm;
    }
    if (q == 0) { free(M); return NULL; }
    M->nlev = q + 1;
    for (int lv = 0; lv < M->nlev; lv++) {
        const int64_t ncl = mg_ncl(M, lv);
        M->off[lv] = (double*)calloc(16 * ncl, sizeof(double));
        M->diag[lv] = (double*)calloc(4 * ncl, sizeof(double));
        M->dinv[lv] = (double*)calloc(4 * ncl, sizeof(double));
        M->b[lv] = (double*)calloc(2 * ncl, sizeof(double));
        M->z[lv] = (double*)calloc(2 * ncl, sizeof(double));
    }
    /* level 0: the T/S block of the Jacobian (k_ts_compact / k_cell_factors) */
    const uint8_t* kn = g->known;
    const int64_t nc0 = mg_ncl(M, 0);
    static const int dd[8][4] = {{-1, 0, 0, 0}, {1, 0, 0, 0}, {0, -1, 0, 0}, {0, 1, 0, 0},
                                 {0, 0, -1, 0}, {0, 0, 1, 0}, {0, 0, -1, 1}, {0, 0, 1, 1}};
    for (int j = 0; j < m; j++)
        for (int k = 0; k < l; k++)
            for (int i = 0; i < n; i++) {
                const int64_t c = ((int64_t)j * l + k) * n + i, rc = cel(g, i, j, k);
                for (int R = 0; R < 2; R++) {
                    const int var = TT + R, oth = SS - R;
                    const int64_t row = NUN * rc + var;
                    const int act = !kn[row] && row != g->rowintcon;
                    for (int qq = 0; qq < 8; qq++) {
                        double v = 0.0;
                        if (act) {
                            int ii = i + dd[qq][0], jj = j + dd[qq][1];
                            const int kk = k + dd[qq][2];
                            if (kk >= 0 && kk < l && wrap(g, &ii, &jj)) {
                                const int64_t cl = NUN * cel(g, ii, jj, kk) + (dd[qq][3] ? oth : var);
                                if (!kn[cl]) v = A(g, row, cl);
                            }
                        }
                        M->off[0][(int64_t)(R * 8 + qq) * nc0 + c] = v;
                    }
                }
                const int64_t u = NUN * rc;
                const int ta = !kn[u + TT], sa = !kn[u + SS];
                double sd = A(g, u + SS, u + SS), st = A(g, u + SS, u + TT);
                if (u + SS == g->rowintcon) { sd = g->int_sign * g->intc[u + SS]; st = 0.0; }
                M->diag[0][c] = ta ? A(g, u + TT, u + TT) : 0.0;
                M->diag[0][nc0 + c] = ta && sa ? A(g, u + TT, u + SS) : 0.0;
                M->diag[0][2 * nc0 + c] = ta && sa ? st : 0.0;
                M->diag[0][3 * nc0 + c] = sa ? sd : 0.0;
                for (int e = 0; e < 4; e++) M->dinv[0][e * nc0 + c] = g->tsinv[4 * rc + e];
            }
    /* Galerkin coarse levels (k_mg_galerkin) */
    for (int lv = 1; lv < M->nlev; lv++) {
        const int Fn = M->n[lv - 1], Fm = M->m[lv - 1];
        const int64_t fcl = mg_ncl(M, lv - 1), ccl = mg_ncl(M, lv);
        for (int64_t t = 0; t < ccl; t++) {
            const int I = (int)(t % M->n[lv]), k = (int)((t / M->n[lv]) % l), J = (int)(t / ((int64_t)M->n[lv] * l));
            double o[16] = {0}, d[4] = {0};
            for (int bb = 0; bb < 2; bb++)
                for (int a = 0; a < 2; a++) {
                    const int i = 2 * I + a, j = 2 * J + bb;
                    if (i >= Fn || j >= Fm) continue;
                    const int64_t c = ((int64_t)j * l + k) * Fn + i;
                    for (int e = 0; e < 4; e++) d[e] += M->diag[lv - 1][e * fcl + c];
                    for (int R = 0; R < 2; R++)
                        for (int qq = 0; qq < 8; qq++) {
                            const double v = M->off[lv - 1][(int64_t)(8 * R + qq) * fcl + c];
                            if (v == 0.0) continue;
                            int ii = i, jj = j, kk = k;
                            if (!mg_nb(M, lv - 1, qq < 6 ? qq : qq - 2, &ii, &jj, &kk)) continue;
                            if (qq < 6 && (ii >> 1) == I && (jj >> 1) == J && kk == k) d[3 * R] += v;
                            else o[8 * R + qq] += v;
                        }
                }
            const int at = d[0] != 0.0, as = d[3] != 0.0;
            if (!at) { d[1] = d[2] = 0.0; for (int qq = 0; qq < 8; qq++) o[qq] = 0.0; }
            if (!as) { d[1] = d[2] = 0.0; for (int qq = 8; qq < 16; qq++) o[qq] = 0.0; }
            for (int e = 0; e < 16; e++) M->off[lv][e * ccl + t] = o[e];
            for (int e = 0; e < 4; e++) M->diag[lv][e * ccl + t] = d[e];
            double inv[4];
            inv2(d[0], d[1], d[2], d[3], at, as, inv);
            for (int e = 0; e < 4; e++) M->dinv[lv][e * ccl + t] = inv[e];
        }
    }
    /* coarsest: dense operator and its inverse */
    const int qc = M->nlev - 1;
    const int64_t ncl = mg_ncl(M, qc);
    const int N = (int)(2 * ncl);
    double* Ad = (double*)calloc((size_t)N * N, sizeof(double));
    M->cinv = (double*)calloc((size_t)N * N, sizeof(double));
    for (int64_t t = 0; t < ncl; t++) {
        const int i = (int)(t % M->n[qc]), k = (int)((t / M->n[qc]) % l), jl = (int)(t / ((int64_t)M->n[qc] * l));
        for (int R = 0; R < 2; R++) {
            const int64_t row = R * ncl + t;
            Ad[row * N + R * ncl + t] += M->diag[qc][(3 * R) * ncl + t];
            Ad[row * N + (1 - R) * ncl + t] += M->diag[qc][(1 + R) * ncl + t];
            for (int qq = 0; qq < 8; qq++) {
                const double v = M->off[qc][(8 * R + qq) * ncl + t];
                if (v == 0.0) continue;
                int ii = i, jj = jl, kk = k;
                if (!mg_nb(M, qc, qq < 6 ? qq : qq - 2, &ii, &jj, &kk)) continue;
                const int64_t nb = ((int64_t)jj * l + kk) * M->n[qc] + ii;
                Ad[row * N + (qq < 6 ? R : 1 - R) * ncl + nb] += v;
            }
        }
    }
    dense_inverse(Ad, N, M->cinv);
    free(Ad);
    return M;
}

/* off-diagonal part of (T, S) rows at cell c of level lv applied to the iterate */
static void mg_offmul(const mg_t* M, int lv, int i, int j, int k, int64_t c, double* at, double* as)
{
    const int64_t ncl = mg_ncl(M, lv);
    const double *off = M->off[lv], *zt = M->z[lv], *zs = M->z[lv] + ncl;
    *at = *as = 0.0;
    for (int q = 0; q < 6; q++) {
        int ii = i, jj = j, kk = k;
        if (!mg_nb(M, lv, q, &ii, &jj, &kk)) continue;
        const int64_t nc = ((int64_t)jj * M->l + kk) * M->n[lv] + ii;
        *at += off[q * ncl + c] * zt[nc];
        *as += off[(8 + q) * ncl + c] * zs[nc];
        if (q == 4) { *at += off[6 * ncl + c] * zs[nc]; *as += off[14 * ncl + c] * zt[nc]; }
        else if (q == 5) { *at += off[7 * ncl + c] * zs[nc]; *as += off[15 * ncl + c] * zt[nc]; }
    }
}

/* z-line relaxation of the columns of one horizontal colour (block Thomas along k) */
static void mg_zline(mg_t* M, int lv, int colour)
{
    const int n = M->n[lv], mb = M->m[lv], l = M->l;
    const int64_t ncl = mg_ncl(M, lv);
    const double *off = M->off[lv], *dg = M->diag[lv], *bt = M->b[lv], *bs = M->b[lv] + ncl;
    double *zt = M->z[lv], *zs = M->z[lv] + ncl;
    const int odd = M->periodic && (n & 1);
#pragma omp parallel for schedule(static)
    for (int col = 0; col < n * mb; col++) {
        const int i = col % n, j = col / n;
        const int cc = (odd && i == n - 1) ? 2 + (j & 1) : ((i + j) & 1);
        if (cc != colour) continue;
        double Cp[64][4], dp[64][2];
        for (int k = 0; k < l; k++) {
            const int64_t c = ((int64_t)j * l + k) * n + i;
            double rt = bt[c], rs = bs[c];
            for (int q = 0; q < 4; q++) {
                int ii = i, jj = j, kk = k;
                if (!mg_nb(M, lv, q, &ii, &jj, &kk)) continue;
                const int64_t nc = ((int64_t)jj * l + kk) * n + ii;
                rt -= off[q * ncl + c] * zt[nc];
                rs -= off[(8 + q) * ncl + c] * zs[nc];
            }
            double Am[4] = {dg[c], dg[ncl + c], dg[2 * ncl + c], dg[3 * ncl + c]};
            double Bm[4] = {off[4 * ncl + c], off[6 * ncl + c], off[14 * ncl + c], off[12 * ncl + c]};
            double Cm[4] = {off[5 * ncl + c], off[7 * ncl + c], off[15 * ncl + c], off[13 * ncl + c]};
            const int at = dg[c] != 0.0, as = dg[3 * ncl + c] != 0.0;
            if (!at) { Am[0] = 1.0; Am[1] = Am[2] = 0.0; Bm[0] = Bm[1] = 0.0; Cm[0] = Cm[1] = 0.0; rt = 0.0; }
            if (!as) { Am[3] = 1.0; Am[1] = Am[2] = 0.0; Bm[2] = Bm[3] = 0.0; Cm[2] = Cm[3] = 0.0; rs = 0.0; }
            if (k > 0) {       /* Am -= Bm Cp[k-1], r -= Bm dp[k-1] */
                const double* P = Cp[k - 1];
                const double a0 = Am[0] - (Bm[0] * P[0] + Bm[1] * P[2]), a1 = Am[1] - (Bm[0] * P[1] + Bm[1] * P[3]);
                const double a2 = Am[2] - (Bm[2] * P[0] + Bm[3] * P[2]), a3 = Am[3] - (Bm[2] * P[1] + Bm[3] * P[3]);
                Am[0] = a0; Am[1] = a1; Am[2] = a2; Am[3] = a3;
                rt -= Bm[0] * dp[k - 1][0] + Bm[1] * dp[k - 1][1];
                rs -= Bm[2] * dp[k - 1][0] + Bm[3] * dp[k - 1][1];
            }
            const double det = Am[0] * Am[3] - Am[1] * Am[2];
            const double qd = det != 0.0 ? 1.0 / det : 0.0;
            const double I0 = Am[3] * qd, I1 = -Am[1] * qd, I2 = -Am[2] * qd, I3 = Am[0] * qd;
            Cp[k][0] = I0 * Cm[0] + I1 * Cm[2]; Cp[k][1] = I0 * Cm[1] + I1 * Cm[3];
            Cp[k][2] = I2 * Cm[0] + I3 * Cm[2]; Cp[k][3] = I2 * Cm[1] + I3 * Cm[3];
            dp[k][0] = I0 * rt + I1 * rs;
            dp[k][1] = I2 * rt + I3 * rs;
        }
        double x0 = 0.0, x1 = 0.0;
        for (int k = l - 1; k >= 0; k--) {
            const int64_t c = ((int64_t)j * l + k) * n + i;
            const double y0 = dp[k][0] - (Cp[k][0] * x0 + Cp[k][1] * x1);
            const double y1 = dp[k][1] - (Cp[k][2] * x0 + Cp[k][3] * x1);
            x0 = y0; x1 = y1;
            zt[c] = x0; zs[c] = x1;
        }
    }
}

static void mg_smooth(mg_t* M, int lv, int post)
{
    const int ncol = (M->periodic && (M->n[lv] & 1)) ? 4 : 2;
    for (int h = 0; h < ncol; h++) mg_zline(M, lv, post ? ncol - 1 - h : h);
}

static void mg_vcycle(gs_t* g, void* mgp, int q)
{
    (void)g;
    mg_t* M = (mg_t*)mgp;
    if (q == M->nlev - 1) {
        const int64_t ncl = mg_ncl(M, q);
        const int N = (int)(2 * ncl);
#pragma omp parallel for schedule(static)
        for (int r = 0; r < N; r++) {
            double acc = 0.0;
            for (int c = 0; c < N; c++) acc += M->cinv[(size_t)r * N + c] * M->b[q][c];
            M->z[q][r] = acc;
        }
        return;
    }
    mg_smooth(M, q, 0);
    /* restriction: coarse rhs = sum of the children's residuals, coarse iterate 0 */
    const int Fn = M->n[q], Fm = M->m[q], l = M->l;
    const int64_t fcl = mg_ncl(M, q), ccl = mg_ncl(M, q + 1);
    const double* dg = M->diag[q];
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < ccl; t++) {
        const int I = (int)(t % M->n[q + 1]), k = (int)((t / M->n[q + 1]) % l), J = (int)(t / ((int64_t)M->n[q + 1] * l));
        double rs4[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        for (int ch = 0; ch < 4; ch++) {
            const int i = 2 * I + (ch & 1), j = 2 * J + (ch >> 1);
            if (i >= Fn || j >= Fm) continue;
            const int64_t c = ((int64_t)j * l + k) * Fn + i;
            double at, as;
            mg_offmul(M, q, i, j, k, c, &at, &as);
            const double zt = M->z[q][c], zs = M->z[q][fcl + c];
            at += dg[c] * zt + dg[fcl + c] * zs;
            as += dg[2 * fcl + c] * zt + dg[3 * fcl + c] * zs;
            rs4[ch][0] = M->b[q][c] - at;
            rs4[ch][1] = M->b[q][fcl + c] - as;
        }
        M->b[q + 1][t] = (rs4[0][0] + rs4[1][0]) + (rs4[2][0] + rs4[3][0]);
        M->b[q + 1][ccl + t] = (rs4[0][1] + rs4[1][1]) + (rs4[2][1] + rs4[3][1]);
        M->z[q + 1][t] = M->z[q + 1][ccl + t] = 0.0;
    }
    mg_vcycle(g, mgp, q + 1);
    /* prolongation: fine iterate += its aggregate's correction (active unknowns) */
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < fcl; t++) {
        const int i = (int)(t % Fn), k = (int)((t / Fn) % l), j = (int)(t / ((int64_t)Fn * l));
        const int64_t p = ((int64_t)(j >> 1) * l + k) * M->n[q + 1] + (i >> 1);
        if (dg[t] != 0.0) M->z[q][t] += M->z[q + 1][p];
        if (dg[3 * fcl + t] != 0.0) M->z[q][fcl + t] += M->z[q + 1][ccl + p];
    }
    mg_smooth(M, q, 1);
}

/* level-0 right-hand side from bts, iterate 0 */
static void mg_begin(gs_t* g, void* mgp, double* z)
{
    (void)z;
    mg_t* M = (mg_t*)mgp;
    const int n = g->n, m = g->m, l = g->l;
    const int64_t nc0 = mg_ncl(M, 0);
    for (int j = 0; j < m; j++)
        for (int k = 0; k < l; k++)
            for (int i = 0; i < n; i++) {
                const int64_t c = ((int64_t)j * l + k) * n + i, rc = cel(g, i, j, k);
                M->b[0][c] = g->known[NUN * rc + TT] ? 0.0 : g->bts[NUN * rc + TT];
                M->b[0][nc0 + c] = g->known[NUN * rc + SS] ? 0.0 : g->bts[NUN * rc + SS];
                M->z[0][c] = M->z[0][nc0 + c] = 0.0;
            }
}
static void mg_end(gs_t* g, void* mgp, double* z)
{
    mg_t* M = (mg_t*)mgp;
    const int n = g->n, m = g->m, l = g->l;
    const int64_t nc0 = mg_ncl(M, 0);
    for (int j = 0; j < m; j++)
        for (int k = 0; k < l; k++)
            for (int i = 0; i < n; i++) {
                const int64_t c = ((int64_t)j * l + k) * n + i, rc = cel(g, i, j, k);
                if (!g->known[NUN * rc + TT]) z[NUN * rc + TT] = M->z[0][c];
                if (!g->known[NUN * rc + SS]) z[NUN * rc + SS] = M->z[0][nc0 + c];
            }
}

/* variant: dyn_iters defect-correction passes with step omega, ts_mg V-cycles (0: the
 * ts_sweeps plain sweeps); returns 0, or -1 if the T/S multigrid has no coarse level */
int orc_gs_config(void* h, int dyn_iters, double omega, int ts_mg)
{
    gs_t* g = (gs_t*)h;
    g->dyn_iters = dyn_iters > 1 ? dyn_iters : 1;
    g->dyn_omega = omega > 0.0 ? omega : 1.0;
    if (g->dyn_iters > 1 && !g->dres) {
        g->dres = (double*)calloc(g->N, sizeof(double));
        g->zc = (double*)calloc(g->N, sizeof(double));
    }
    g->ts_mg = ts_mg > 0 ? ts_mg : 0;
    if (g->ts_mg > 0 && !g->mg) {
        g->mg = mg_build(g);
        if (!g->mg) { g->ts_mg = 0; return -1; }
    }
    return 0;
}

/* 6. T/S right-hand side bts = rr_TS - A_TS,D z_D (z's T/S entries stay 0 until the T/S
 * solve) */
static void ts_rhs(gs_t* g, double* z)
{
    const int64_t N = g->N;
    const uint8_t* kn = g->known;
#pragma omp parallel for schedule(static)
    for (int64_t row = 0; row < N; row++) {
        int var = (int)(row % NUN);
        if (var < TT || kn[row]) continue;
        double acc = g->rr[row];
        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++) {
            int cv = g->col[p] % NUN;
            if (cv == TT || cv == SS || kn[g->col[p]]) continue;
            acc -= g->val[p] * z[g->col[p]];
        }
        g->bts[row] = acc;
        z[row] = 0.0;
    }
}

/* the T/S right-hand side after ts_at dynamics passes (0: after the last one) */
void orc_gs_ts_at(void* h, int ts_at)
{
    ((gs_t*)h)->ts_at = ts_at;
}

/* Study variant (CPU twin only, not on the GPU; DESIGN.md §4 "inner acceleration"):
 * dyn_krylov = 1 makes the dyn_iters applications of M_D a right-preconditioned GMRES on the
 * dynamics block A_DD z_D = rr_D (from z_D = 0; classical Gram-Schmidt twice) instead of the
 * damped defect-correction passes (the reference accelerates its sub-solves by GMRESR,
 * TRIOS_BlockPreconditioner.C:1479-1611) */
/* the exact Schur solve in schur_passes of the dynamics passes only: the first k - 1 and the
 * last (k = 1: the first; 0 or >= dyn_iters: all); the others take pbar = 0.  The GPU's
 * BlockGS::schur_passes (iemic_krylov.schur_passes, prec_gs.hip gs_pass_schur) */
void orc_gs_schur_passes(void* h, int k) { ((gs_t*)h)->schur_passes = k > 0 ? k : 0; }
void orc_gs_schur_mask(void* h, int mask) { ((gs_t*)h)->schur_mask = mask; }

void orc_gs_dyn_krylov(void* h, int on)
{
    gs_t* g = (gs_t*)h;
    g->dyn_krylov = on ? 1 : 0;
    if (on && !g->kv) {
        g->kv = (double*)calloc((size_t)(g->dyn_iters + 1) * g->N, sizeof(double));
        g->kz = (double*)calloc((size_t)g->dyn_iters * g->N, sizeof(double));
    }
}

static double dyn_dot(const gs_t* g, const double* a, const double* b)
{
    double s = 0.0;
    for (int64_t row = 0; row < g->N; row++)
        if (row % NUN <= PP && !g->known[row]) s += a[row] * b[row];
    return s;
}

/* z_D from GMRES(k) on the dynamics block, k = dyn_iters applications of dyn_solve */
static void dyn_gmres(gs_t* g, double* z)
{
    const int k = g->dyn_iters;
    const int64_t N = g->N;
    double H[17][16], cs[16], sn[16], e[17], y[16];
    memset(H, 0, sizeof(H));
    memset(e, 0, sizeof(e));
    double* V = g->kv;
    double* Z = g->kz;
    /* v0 = rr_D / beta (the rows the dynamics solve reads: U/V/W/P of the active rows) */
    for (int64_t row = 0; row < N; row++) V[row] = (row % NUN <= PP && !g->known[row]) ? g->rr[row] : 0.0;
    const double beta = sqrt(dyn_dot(g, V, V));
    if (!(beta > 0.0)) return;
    for (int64_t row = 0; row < N; row++) V[row] /= beta;
    e[0] = beta;
    int nk = 0;
    for (int j = 0; j < k; j++) {
        double* vj = V + (int64_t)j * N;
        double* zj = Z + (int64_t)j * N;
        double* w = V + (int64_t)(j + 1) * N;
        memset(zj, 0, sizeof(double) * N);
        {
            /* the Schur solve in the applications schur_passes selects (gs_pass_schur) */
            const int kk = g->schur_passes, last = j + 1 == k;
            const int solve = j == 0 || kk <= 0 || kk >= k || (kk >= 2 && (j < kk - 1 || last));
            g->skip_schur = !solve;
        }
        dyn_solve(g, vj, zj);
        g->skip_schur = 0;
        /* w = A_DD zj: the defect of zj against a zero right-hand side, negated */
        double* rrs = g->rr;
        static double* zero = NULL;
        static int64_t nz = 0;
        if (nz < N) { free(zero); zero = (double*)calloc(N, sizeof(double)); nz = N; }
        g->rr = zero;
        dyn_defect(g, zj, w);
        g->rr = rrs;
        for (int64_t row = 0; row < N; row++) w[row] = -w[row];
        for (int pass = 0; pass < 2; pass++)
            for (int i = 0; i <= j; i++) {
                const double hij = dyn_dot(g, V + (int64_t)i * N, w);
                H[i][j] += hij;
                for (int64_t row = 0; row < N; row++) w[row] -= hij * V[(int64_t)i * N + row];
            }
        const double hn = sqrt(dyn_dot(g, w, w));
        H[j + 1][j] = hn;
        if (hn > 0.0)
            for (int64_t row = 0; row < N; row++) w[row] /= hn;
        for (int i = 0; i < j; i++) {
            const double a = H[i][j], b = H[i + 1][j];
            H[i][j] = cs[i] * a + sn[i] * b;
            H[i + 1][j] = -sn[i] * a + cs[i] * b;
        }
        const double a = H[j][j], b = H[j + 1][j], d = sqrt(a * a + b * b);
        cs[j] = d > 0.0 ? a / d : 1.0;
        sn[j] = d > 0.0 ? b / d : 0.0;
        H[j][j] = d;
        H[j + 1][j] = 0.0;
        e[j + 1] = -sn[j] * e[j];
        e[j] = cs[j] * e[j];
        nk = j + 1;
        if (hn == 0.0) break;
    }
    for (int i = nk - 1; i >= 0; i--) {
        double s = e[i];
        for (int q = i + 1; q < nk; q++) s -= H[i][q] * y[q];
        y[i] = H[i][i] != 0.0 ? s / H[i][i] : 0.0;
    }
    for (int64_t row = 0; row < N; row++) {
        if (row % NUN > PP || g->known[row]) continue;
        double s = 0.0;
        for (int q = 0; q < nk; q++) s += y[q] * Z[(int64_t)q * N + row];
        z[row] = s;
    }
}

void orc_gs_apply(void* h, const double* r, double* z)
{
    gs_t* g = (gs_t*)h;
    const int n = g->n, m = g->m;
    const int64_t N = g->N, nc = g->ncell;
    const uint8_t* kn = g->known;
    memset(z, 0, sizeof(double) * N);
    /* known rows and rr */
#pragma omp parallel for schedule(static)
    for (int64_t row = 0; row < N; row++) {
        if (kn[row]) { z[row] = r[row]; g->rr[row] = 0.0; continue; }
        double acc = r[row];
        for (int64_t p = g->rowptr[row]; p < g->rowptr[row + 1]; p++)
            if (kn[g->col[p]]) acc -= g->val[p] * r[g->col[p]];
        g->rr[row] = acc;
    }
    double* rr = g->rr;
    const int ts_at = (g->ts_at >= 1 && g->ts_at < g->dyn_iters) ? g->ts_at : g->dyn_iters;
    if (g->dyn_krylov && g->dyn_iters > 1) {
        dyn_gmres(g, z);
        ts_rhs(g, z);
    } else {
        dyn_solve(g, rr, z);
    }
    /* defect correction: z_D += omega M_D^-1 (rr - A z)_D; the T/S right-hand side
     * rr_TS - A_TS,D z_D is formed after ts_at passes (default: all of them) */
    if (ts_at == 1 && !g->dyn_krylov) ts_rhs(g, z);
    for (int it = 1; !g->dyn_krylov && it < g->dyn_iters; it++) {
        dyn_defect(g, z, g->dres);
        memset(g->zc, 0, sizeof(double) * N);
        {
            /* schur_passes k: the first k - 1 passes and the last solve it (k = 1: the first
             * only; 0 or >= dyn_iters: every pass) -- the GPU's gs_pass_schur */
            const int k = g->schur_passes, last = it + 1 == g->dyn_iters;
            const int solve = k <= 0 || k >= g->dyn_iters || (k >= 2 && (it < k - 1 || last));
            g->skip_schur = g->schur_mask ? !((g->schur_mask >> it) & 1) : !solve;
        }
        dyn_solve(g, g->dres, g->zc);
        g->skip_schur = 0;
        for (int64_t row = 0; row < N; row++)
            if (row % NUN <= PP && !kn[row]) z[row] += g->dyn_omega * g->zc[row];
        if (it + 1 == ts_at) ts_rhs(g, z);
    }
    if (g->ts_mg > 0 && g->mg) {
        mg_begin(g, g->mg, z);
        for (int cyc = 0; cyc < g->ts_mg; cyc++) mg_vcycle(g, g->mg, 0);
        mg_end(g, g->mg, z);
        return;
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
