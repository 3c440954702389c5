/*
 * thcm_oracle.c -- TEST INFRASTRUCTURE ONLY (see thcm_oracle.h).
 *
 * Routine-by-routine CPU restatement of the reference THCM assembly.  Each function
 * cites the reference file:line it restates.  Floating-point expressions keep the
 * Fortran evaluation order (left-to-right, unary minus over the whole product) so the
 * restatement reproduces the reference to the last bit or within a few ulps; this file
 * must be compiled with -ffp-contract=off.
 *
 * Scope: ocean-only or coupled to an external atmosphere (coupled_T / coupled_S, no sea
 * ice: msi = gsi = mc = 0), idealized forcing (ite = its = 1, iza = 2), no internal
 * Levitus forcing; vertical mixing per the default vmix parameters.
 */
#include "thcm_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NUN 6
#define NP 27
#define UU 1
#define VV 2
#define WW 3
#define PP 4
#define TT 5
#define SS 6
#define OCEAN 0
#define LAND 1

/* par.F90:38-67 */
enum { AL_T = 1, RAYL, EK_V, EK_H, ROSB, MIXP, RESC, SPL1, HMTP, SUNP, PE_H, PE_V, P_VC,
       LAMB, SALT, WIND, TEMP, BIOT, COMB, ARCL, NLES, IFRICB, CONT, ENER, ALPC, CMPR,
       FPER, SPER, MKAP, SPL2 };

/* m_atm constants (atm.F90:5-19) */
static const double rhoa_atm = 1.25, ch_atm = 0.94 * 1.3e-03, cpa_atm = 1000., uw_atm = 8.5;
static const double sun0_atm = 1360., c0_atm = 0.43, lv_atm = 2.5e+06;

/* usr.F90:131-160 fixed parameters */
static const double pi_ = 3.14159265358979323846;
static const double omegadim = 7.292e-05, r0dim = 6.37e+06, udim = 0.1e+00, gdim = 9.8e+00;
static const double rhodim = 1.024e+03, deltas = 1.0, s0 = 35.0, cp0 = 4.2e+03;
static const double alpt1 = 2.93, alpt2 = 8.3e-02, alpt3 = 6.6e-04;
static const double ah = 2.5e+05, av = 1.0e-03, kappah = 1.0e+03, kappav = 1.0e-04;
static const double zmin = -1.0, zmax = 0.0;

struct orc {
    orc_cfg c;
    int n, m, l, ndim, ncell;
    double xmin, xmax, ymin, ymax;     /* radians */
    double dx, dy, dz;
    double *x, *y, *z, *xu, *yv, *zw, *ze, *zwe, *dfzT, *dfzW;   /* grid.F90 */
    int* landm;                        /* (0:n+1,0:m+1,0:l+1) */
    double par[31];
    double QTnd, QSnd;
    double *taux, *tauy, *tatm, *emip, *spert;
    /* coupled atmosphere (m_atm: atmos_coef usrc.F90:1183-1223, set_atmos_parameters
     * 237-293; inserted fields inserts.F90) */
    double *qatm, *albe, *patm, *suno;
    double Ooa, Os, lvsc, nus, eta_a, qdim_a, dqso, eo0, albe0, albed;
    double* Frc;                       /* forcing.F90 (before boundaries zeroing) */
    int rowintcon;                     /* 0-based, -1 if SRES != 0 */
    int vmix_temp, vmix_salt, vmix_fix; /* m_mix flags (mix_imp.f vmix_init/control)   */
    /* maximal graph */
    int64_t* gptr;
    int* gcol;
};

/* ------------------------------------------------------------------------------ */
#define LM(o, i, j, k) ((o)->landm[((size_t)(k) * ((o)->m + 2) + (j)) * ((o)->n + 2) + (i)])
#define Y(j) (o->y[(j)])          /* y(0:m+1) */
#define YV(j) (o->yv[(j)])        /* yv(0:m)  */
#define DFZT(k) (o->dfzT[(k)])    /* dfzT(1:l), index 0 unused */
#define DFZW(k) (o->dfzW[(k)])    /* dfzW(0:l) */

/* find_row2 (matetc.F90:123-144), returned 0-based */
static inline int frow(const orc_t* o, int i, int j, int k, int XX)
{
    return NUN * ((k - 1) * o->n * o->m + o->n * (j - 1) + i - 1) + XX - 1;
}

/* grid.F90:62-95 */
static double fz(double z, double qz)
{
    double th = tanh(qz * (z + 1));
    double tth = tanh(qz);
    if (qz > 1.0) return -1 + th / tth;
    return z + (1. - qz) * z * (1 - z);
}
static double dfdz(double z, double qz)
{
    double ch = cosh(qz * (z + 1));
    double tth = tanh(qz);
    if (qz > 1.0) return qz / (tth * ch * ch);
    return 1.0 + (1. - qz) * (1. - 2. * z);
}

/* spf.F90:792-854 */
static double amh(double y, int ih) { return ih == 0 ? 1.0 : 1. + 10.0 * exp(-5 * y * y); }
static double bmh(double y, int ih) { return ih == 0 ? 1.0 : 1.0 + 10.0 * exp(-5 * y * y); }
static double bmhy(double y, int ih) { return ih == 0 ? 0.0 : -10. * 10.0 * y * exp(-5 * y * y); }

/* grid.F90:2-60 */
static void grid(orc_t* o)
{
    int n = o->n, m = o->m, l = o->l;
    o->dx = (o->xmax - o->xmin) / n;
    o->dy = (o->ymax - o->ymin) / m;
    o->dz = (zmax - zmin) / l;
    for (int i = 1; i <= n; i++) {
        o->x[i] = ((double)i - 0.5) * o->dx + o->xmin;
        o->xu[i] = ((double)i) * o->dx + o->xmin;
    }
    o->xu[0] = o->xmin;
    for (int j = 1; j <= m; j++) {
        o->y[j] = ((double)j - 0.5) * o->dy + o->ymin;
        o->yv[j] = ((double)j) * o->dy + o->ymin;
    }
    o->y[0] = o->y[1] - o->dy;
    o->y[m + 1] = o->y[m] + o->dy;
    o->yv[0] = o->ymin;
    for (int k = 1; k <= l; k++) {
        o->ze[k] = ((double)k - 0.5) * o->dz + zmin;
        o->zwe[k] = ((double)k) * o->dz + zmin;
        o->z[k] = fz(o->ze[k], o->c.qz);
        o->zw[k] = fz(o->zwe[k], o->c.qz);
        o->dfzT[k] = dfdz(o->ze[k], o->c.qz);
        o->dfzW[k] = dfdz(o->zwe[k], o->c.qz);
    }
    o->zw[0] = zmin;
    o->dfzW[0] = dfdz(zmin, o->c.qz);
}

/* usrc.F90:1136-1180 (stpnt) + mix_imp.f vmix_par */
static void stpnt(orc_t* o)
{
    double* par = o->par;
    double hdim = o->c.hdim;
    par[AL_T] = 0.1 / (2 * omegadim * rhodim * hdim * udim * o->dz * DFZT(o->l));
    par[RAYL] = o->c.alphaT * gdim * hdim / (2 * omegadim * udim * r0dim);
    par[EK_V] = av / (2 * omegadim * hdim * hdim);
    par[EK_H] = ah / (2 * omegadim * r0dim * r0dim);
    par[ROSB] = udim / (2 * omegadim * r0dim);
    par[HMTP] = 0.0;
    par[SUNP] = 0.0;
    par[PE_H] = kappah / (udim * r0dim);
    par[PE_V] = kappav * r0dim / (udim * hdim * hdim);
    par[P_VC] = 2.5e+04 * par[PE_V];
    par[LAMB] = o->c.alphaS / o->c.alphaT;
    par[SALT] = 0.0;
    par[WIND] = 0.0;
    par[TEMP] = 0.0;
    par[BIOT] = r0dim / (75. * 3600. * 24. * udim);
    par[COMB] = 0.0;
    par[NLES] = 0.0;
    par[CMPR] = 0.0;
    par[ALPC] = 1.0;
    par[ENER] = 1.0e+02;
    par[MIXP] = 0.0;
    par[MKAP] = 0.0;
    par[SPL1] = 2.0e+03;
    par[SPL2] = 0.01;
    if (o->c.vmix == 0) { /* mix_imp.f vmix_par */
        par[MIXP] = 0.0;
        par[P_VC] = 0.0;
        par[ALPC] = 1.0;
        par[ENER] = 1.0e+2;
        par[MKAP] = 0.0;
    }
}

/* forcing.F90:489-533 */
static double wfun(double yy)
{
    return 0.2 - 0.8 * sin(6 * fabs(yy)) - 0.5 * (1 - tanh(10 * fabs(yy))) -
           0.5 * (1 - tanh(10 * (pi_ / 2 - fabs(yy))));
}
static double temfun(const orc_t* o, double yy)
{
    if (o->c.forcing_type == 2) return cos(pi_ * (yy - o->ymin) / (o->ymax - o->ymin));
    return cos(pi_ * yy / o->ymax) + o->par[CMPR] * sin(pi_ * yy / o->ymax);
}
static double salfun(const orc_t* o, double yy)
{
    if (o->c.forcing_type == 2) return cos(pi_ * (yy - o->ymin) / (o->ymax - o->ymin));
    if (o->c.forcing_type == 1) return (cos(pi_ * yy / o->ymax) + o->par[FPER] * yy / o->ymax) / cos(yy);
    return cos(pi_ * yy / o->ymax) + o->par[FPER] * yy / o->ymax;
}

/* forcing.F90:536-548 qint -> THCM.C:2704-2737 (serial) */
static double qint(const orc_t* o, const double* field)
{
    double lsint = 0.0, lfsint = 0.0;
    for (int j = 1; j <= o->m; j++)
        for (int i = 1; i <= o->n; i++) {
            int lm = LM(o, i, j, o->l);
            lfsint = field[(j - 1) * o->n + (i - 1)] * cos(Y(j)) * (1 - lm) + lfsint;
            lsint = cos(Y(j)) * (1 - lm) + lsint;
        }
    return lfsint / lsint;
}

/* forcing.F90:4-218, ocean-only idealized branch */
static void forcing(orc_t* o)
{
    int n = o->n, m = o->m, l = o->l;
    double* par = o->par;
    int TRES = o->c.tres, SRES = o->c.sres;
    memset(o->Frc, 0, sizeof(double) * o->ndim);
    double sigma = par[COMB] * par[WIND] * par[AL_T];
    for (int j = 1; j <= m; j++)
        for (int i = 1; i <= n; i++) {
            o->taux[(j - 1) * n + i - 1] = wfun(YV(j));
            o->tauy[(j - 1) * n + i - 1] = 0.0;
        }
    for (int j = 1; j <= m - 1; j++)
        for (int i = 1; i <= n; i++) {
            o->Frc[frow(o, i, j, l, UU)] = sigma * o->taux[(j - 1) * n + i - 1];
            o->Frc[frow(o, i, j, l, VV)] = sigma * o->tauy[(j - 1) * n + i - 1];
        }
    double etabi = par[COMB] * par[TEMP] * ((double)(1 - TRES) + TRES * par[BIOT]);
    double temcor = 0.0;
    if (!o->c.coupled_t) {
        for (int j = 1; j <= m; j++)
            for (int i = 1; i <= n; i++) o->tatm[(j - 1) * n + i - 1] = temfun(o, Y(j));
        if (TRES == 0) temcor = qint(o, o->tatm);
    }
    for (int j = 1; j <= m; j++)
        for (int i = 1; i <= n; i++) {
            const int q = (j - 1) * n + i - 1;
            if (o->c.coupled_t) {
                /* forcing.F90:75-94: QToa = QSW - QSH - QLH; no sea ice (msi = 0) */
                double QToa = par[COMB] * par[SUNP] * o->suno[j] * (1 - o->albe0 - o->albed * o->albe[q]) +
                              o->Ooa * o->tatm[q] + o->lvsc * o->eta_a * o->qdim_a * o->qatm[q] -
                              o->lvsc * o->eo0;
                o->Frc[frow(o, i, j, l, TT)] = QToa * (double)(1 - LM(o, i, j, l));
            } else {
                o->Frc[frow(o, i, j, l, TT)] = etabi * (o->tatm[q] - temcor);
            }
        }
    double gamma = par[COMB] * par[SALT] * ((double)(1 - SRES) + SRES * par[BIOT]);
    double salcor = 0.0, adapted_salcor = 0.0, spertcor = 0.0;
    for (int j = 1; j <= m; j++)
        for (int i = 1; i <= n; i++)
            o->emip[(j - 1) * n + i - 1] = salfun(o, Y(j)) * (1 - LM(o, i, j, l));
    if (SRES == 0) {
        salcor = qint(o, o->emip);
        double* zero = (double*)calloc((size_t)n * m, sizeof(double));
        adapted_salcor = qint(o, zero);
        free(zero);
        spertcor = qint(o, o->spert);
    }
    const double pQSnd = par[COMB] * par[SALT] * o->QSnd;
    for (int j = 1; j <= m; j++)
        for (int i = 1; i <= n; i++) {
            int q = (j - 1) * n + i - 1;
            if (o->c.coupled_s) {
                /* forcing.F90:162-182: E - P, patm dimensional; no sea ice (msi = gsi = 0) */
                double QSoa = pQSnd * (o->eo0 - o->eta_a * o->qdim_a * o->qatm[q] - o->patm[q]);
                o->Frc[frow(o, i, j, l, SS)] = QSoa * (double)(1 - LM(o, i, j, l));
                continue;
            }
            o->Frc[frow(o, i, j, l, SS)] =
                gamma * (1 - par[HMTP]) * (o->emip[q] - salcor) +
                gamma * par[HMTP] * (0.0 - adapted_salcor) +
                par[SPER] * ((double)(1 - SRES) + SRES * par[BIOT]) * (o->spert[q] - spertcor);
        }
    /* internal W forcing with zero internal T/S (forcing.F90:199-209) */
    for (int k = 1; k <= l - 1; k++)
        for (int j = 1; j <= m; j++)
            for (int i = 1; i <= n; i++)
                o->Frc[frow(o, i, j, k, WW)] =
                    -par[COMB] * (1 - LM(o, i, j, k)) * par[RAYL] *
                    (par[LAMB] * (0.0 + 0.0) / 2. - (0.0 + 0.0) / 2.);
}

/* ================================================================================
 * Per-cell atoms.  An atom is a 27-vector a[1..27] (index 0 unused) for one cell,
 * exactly the (loc) column of the Fortran atom(np,n,m,l) arrays of spf.F90.
 * ================================================================================ */
typedef double atom_t[NP + 1];
static inline void azero(atom_t a) { memset(a, 0, sizeof(atom_t)); }

/* spf.F90:13-74 uderiv */
static void uderiv(const orc_t* o, int type, int i, int j, int k, atom_t a)
{
    int m = o->m, ih = o->c.ih;
    double dx = o->dx, dy = o->dy, dz = o->dz;
    (void)i;
    azero(a);
    switch (type) {
    case 2:
        if (j <= m - 1) {
            double c = 1.0 / (cos(YV(j)) * dx);
            c = c * c;
            a[2] = amh(YV(j), ih) * c;
            a[8] = amh(YV(j), ih) * c;
            a[5] = -(a[2] + a[8]);
        }
        break;
    case 3:
        if (j <= m - 1) {
            double r = 1.0 / dy;
            r = r * r;
            a[4] = r * bmh(Y(j), ih) * cos(Y(j)) / cos(YV(j));
            a[6] = r * bmh(Y(j + 1), ih) * cos(Y(j + 1)) / cos(YV(j));
            a[5] = -(a[4] + a[6]);
        }
        break;
    case 4: {
        double r = 1.0 / dz;
        r = r * r;
        double h1 = 1. / (DFZT(k) * DFZW(k));
        double h2 = 1. / (DFZT(k) * DFZW(k - 1));
        a[14] = h2 * r;
        a[23] = h1 * r;
        a[5] = -(a[14] + a[23]);
    } break;
    case 5:
        if (j <= m - 1) {
            double t2 = 1 - tan(YV(j)) * tan(YV(j));
            a[5] = bmh(YV(j), ih) * t2 + tan(YV(j)) * bmhy(YV(j), ih);
        }
        break;
    case 6:
        if (j <= m - 1) {
            double t2 = tan(YV(j)), c2 = cos(YV(j));
            a[2] = (bmhy(YV(j), ih) - (amh(YV(j), ih) + bmh(YV(j), ih)) * t2) / (dx * c2);
            a[8] = -(bmhy(YV(j), ih) - (amh(YV(j), ih) + bmh(YV(j), ih)) * t2) / (dx * c2);
        }
        break;
    }
}

/* spf.F90:76-136 vderiv */
static void vderiv(const orc_t* o, int type, int i, int j, int k, atom_t a)
{
    int m = o->m, ih = o->c.ih;
    double dx = o->dx, dy = o->dy, dz = o->dz;
    (void)i;
    azero(a);
    switch (type) {
    case 2:
        if (j <= m - 1) {
            double c = 1.0 / (cos(YV(j)) * dx);
            c = c * c;
            a[2] = bmh(YV(j), ih) * c;
            a[5] = -2 * bmh(YV(j), ih) * c;
            a[8] = bmh(YV(j), ih) * c;
        }
        break;
    case 3:
        if (j <= m - 1) {
            double r = 1.0 / dy;
            r = r * r;
            a[4] = r * amh(Y(j), ih) * cos(Y(j)) / cos(YV(j));
            a[6] = r * amh(Y(j + 1), ih) * cos(Y(j + 1)) / cos(YV(j));
            a[5] = -(a[4] + a[6]);
        }
        break;
    case 4: {
        double r = 1.0 / dz;
        r = r * r;
        double h1 = 1. / (DFZT(k) * DFZW(k));
        double h2 = 1. / (DFZT(k) * DFZW(k - 1));
        a[14] = h2 * r;
        a[23] = h1 * r;
        a[5] = -(a[14] + a[23]);
    } break;
    case 5:
        if (j <= m - 1)
            a[5] = bmh(YV(j), ih) - amh(YV(j), ih) * tan(YV(j)) * tan(YV(j)) +
                   bmhy(YV(j), ih) * tan(YV(j));
        break;
    case 6:
        if (j <= m - 1) {
            double t2 = tan(YV(j)), c2 = cos(YV(j));
            a[2] = -((amh(YV(j), ih) + bmh(YV(j), ih)) * t2 - bmhy(YV(j), ih)) / (dx * c2);
            a[8] = ((amh(YV(j), ih) + bmh(YV(j), ih)) * t2 - bmhy(YV(j), ih)) / (dx * c2);
        }
        break;
    }
}

/* spf.F90:138-187 pderiv */
static void pderiv(const orc_t* o, int type, int i, int j, int k, atom_t a)
{
    (void)i;
    azero(a);
    switch (type) {
    case 1: {
        double c = 1.0 / (2 * cos(Y(j)) * o->dx);
        a[2] = -c;
        a[4] = c;
        a[1] = -c;
        a[5] = c;
    } break;
    case 2: {
        double c = 1. / (2 * cos(Y(j)) * o->dy);
        a[4] = -cos(YV(j - 1)) * c;
        a[2] = cos(YV(j)) * c;
        a[1] = -cos(YV(j - 1)) * c;
        a[5] = cos(YV(j)) * c;
    } break;
    case 3: {
        double dzi = 1.0 / o->dz;
        a[5] = dzi / DFZT(k);
        a[14] = -dzi / DFZT(k);
    } break;
    }
}

/* spf.F90:189-268 tderiv */
static void tderiv(const orc_t* o, int type, int i, int j, int k, atom_t a)
{
    int l = o->l;
    int wet = 1 - LM(o, i, j, l);
    azero(a);
    switch (type) {
    case 1:
    case 2:
        if (k == l) a[5] = 1.0;
        break;
    case 3: {
        double c = 1.0 / (cos(Y(j)) * o->dx);
        c = c * c;
        a[2] = c * wet;
        a[5] = -2 * c * wet;
        a[8] = c * wet;
    } break;
    case 4: {
        double r = 1.0 / o->dy;
        r = r * r;
        a[4] = (r * cos(YV(j - 1)) / cos(Y(j))) * wet;
        a[6] = (r * cos(YV(j)) / cos(Y(j))) * wet;
        a[5] = -(a[4] + a[6]);
    } break;
    case 5: {
        double r = 1.0 / o->dz;
        r = r * r;
        double h1 = 1. / (DFZT(k) * DFZW(k));
        double h2 = 1. / (DFZT(k) * DFZW(k - 1));
        if (k <= l - 1) {
            a[14] = h2 * r * wet;
            a[23] = h1 * r * wet;
            a[5] = -(a[14] + a[23]);
        } else {
            a[14] = h2 * r * wet;
            a[23] = 0.0;
            a[5] = -(a[14] + a[23]);
        }
    } break;
    case 6:
        a[23] = 1.0 * wet;
        a[5] = 1.0 * wet;
        break;
    case 7:
        if (k == 1) a[5] = 1.0;
        break;
    }
}

/* spf.F90:271-302 coriolis (both types identical) */
static void coriolis(const orc_t* o, int j, atom_t a)
{
    azero(a);
    if (j <= o->m - 1) a[5] = sin(YV(j)) * o->c.coriolis_on;
}

/* spf.F90:305-345 gradp */
static void gradp(const orc_t* o, int type, int j, int k, atom_t a)
{
    azero(a);
    switch (type) {
    case 1:
        if (j <= o->m - 1) {
            double c = 1. / (2 * cos(YV(j)) * o->dx);
            a[5] = -c;
            a[6] = -c;
            a[8] = c;
            a[9] = c;
        }
        break;
    case 2:
        if (j <= o->m - 1) {
            double d = 1. / (2 * o->dy);
            a[5] = -d;
            a[8] = -d;
            a[6] = d;
            a[9] = d;
        }
        break;
    case 3: {
        double dzi = 1. / o->dz;
        a[5] = -dzi / DFZW(k);
        a[23] = dzi / DFZW(k);
    } break;
    }
}

/* Local block An(27,6,6) of one cell: Aloc[kk][ii][jj], 1-based like the Fortran. */
typedef double aloc_t[NP + 1][NUN + 1][NUN + 1];

/* usrc.F90:588-772 lin, restricted to one cell (coupled terms without sea ice, mc = 0) */
static void lin_cell(const orc_t* o, int i, int j, int k, aloc_t A)
{
    const double* par = o->par;
    double EV = par[EK_V], EH = par[EK_H];
    double ph = (1 - par[MIXP]) * par[PE_H], pv = par[PE_V];
    double lambda = par[LAMB], xes = par[NLES], bi = par[BIOT], Ra = par[RAYL];
    int TRES = o->c.tres, SRES = o->c.sres;
    atom_t uxx, uyy, uzz, ucsi, vxs, fv, px, vxx, vyy, vzz, vcsi, uxs, fu, py, pz, tbc;
    atom_t uxc, vyc, wzc, tc, sc, txx, tyy, tzz;
    memset(A, 0, sizeof(aloc_t));

    uderiv(o, 2, i, j, k, uxx);
    uderiv(o, 3, i, j, k, uyy);
    uderiv(o, 4, i, j, k, uzz);
    uderiv(o, 5, i, j, k, ucsi);
    uderiv(o, 6, i, j, k, vxs);
    coriolis(o, j, fv);
    gradp(o, 1, j, k, px);
    for (int s = 1; s <= NP; s++) {
        A[s][UU][UU] = -EH * (uxx[s] + uyy[s] + ucsi[s]) - EV * uzz[s];
        A[s][UU][VV] = -fv[s] - EH * vxs[s];
        A[s][UU][PP] = px[s];
    }
    vderiv(o, 2, i, j, k, vxx);
    vderiv(o, 3, i, j, k, vyy);
    vderiv(o, 4, i, j, k, vzz);
    vderiv(o, 5, i, j, k, vcsi);
    vderiv(o, 6, i, j, k, uxs);
    coriolis(o, j, fu);
    gradp(o, 2, j, k, py);
    for (int s = 1; s <= NP; s++) {
        A[s][VV][UU] = fu[s] - EH * uxs[s];
        A[s][VV][VV] = -EH * (vxx[s] + vyy[s] + vcsi[s]) - EV * vzz[s];
        A[s][VV][PP] = py[s];
    }
    gradp(o, 3, j, k, pz);
    tderiv(o, 6, i, j, k, tbc);
    for (int s = 1; s <= NP; s++) {
        A[s][WW][PP] = pz[s];
        A[s][WW][TT] = -Ra * (1. + xes * alpt1) * tbc[s] / 2.;
        A[s][WW][SS] = lambda * Ra * tbc[s] / 2.;
    }
    pderiv(o, 1, i, j, k, uxc);
    pderiv(o, 2, i, j, k, vyc);
    pderiv(o, 3, i, j, k, wzc);
    for (int s = 1; s <= NP; s++) {
        A[s][PP][UU] = uxc[s];
        A[s][PP][VV] = vyc[s];
        A[s][PP][WW] = wzc[s];
    }
    tderiv(o, 1, i, j, k, tc);
    tderiv(o, 2, i, j, k, sc);
    tderiv(o, 3, i, j, k, txx);
    tderiv(o, 4, i, j, k, tyy);
    tderiv(o, 5, i, j, k, tzz);
    /* usrc.F90:724-766: the latent-heat dependence dedt = lvsc eta qdim (deltat/qdim) dqso
     * of T on T (coupled_T) and nus (deltat/qdim) dqso of S on T (coupled_S), deltat = 1 */
    const double deltat = 1.0;
    const double dedt_t = o->lvsc * o->eta_a * o->qdim_a * (deltat / o->qdim_a) * o->dqso;
    const double dedt_s = o->nus * (deltat / o->qdim_a) * o->dqso;
    for (int s = 1; s <= NP; s++) {
        if (o->c.coupled_t)
            A[s][TT][TT] = -ph * (txx[s] + tyy[s]) - pv * tzz[s] + o->Ooa * tc[s] + dedt_t * sc[s];
        else
            A[s][TT][TT] = -ph * (txx[s] + tyy[s]) - pv * tzz[s] + TRES * bi * tc[s];
        if (o->c.coupled_s) {
            A[s][SS][SS] = -ph * (txx[s] + tyy[s]) - pv * tzz[s];
            A[s][SS][TT] = -dedt_s * sc[s];
        } else {
            A[s][SS][SS] = -ph * (txx[s] + tyy[s]) - pv * tzz[s] + SRES * bi * sc[s];
        }
    }
}

/* ---- usol (usrc.F90:997-1104): state -> padded staggered arrays ---------------- */
typedef struct {
    int n, m, l;
    double *u, *v, *w, *p, *t, *s;
} fields_t;
/* u,v: (0:n,0:m,0:l+1); w: (0:n+1,0:m+1,0:l); p,t,s: (0:n+1,0:m+1,0:l+1) */
#define FU(f, i, j, k) ((f)->u[((size_t)(k) * ((f)->m + 1) + (j)) * ((f)->n + 1) + (i)])
#define FV(f, i, j, k) ((f)->v[((size_t)(k) * ((f)->m + 1) + (j)) * ((f)->n + 1) + (i)])
#define FW(f, i, j, k) ((f)->w[((size_t)(k) * ((f)->m + 2) + (j)) * ((f)->n + 2) + (i)])
#define FP(f, i, j, k) ((f)->p[((size_t)(k) * ((f)->m + 2) + (j)) * ((f)->n + 2) + (i)])
#define FT(f, i, j, k) ((f)->t[((size_t)(k) * ((f)->m + 2) + (j)) * ((f)->n + 2) + (i)])
#define FS(f, i, j, k) ((f)->s[((size_t)(k) * ((f)->m + 2) + (j)) * ((f)->n + 2) + (i)])

static void usol(const orc_t* o, const double* un, fields_t* f)
{
    int n = o->n, m = o->m, l = o->l;
    f->n = n; f->m = m; f->l = l;
    size_t nuv = (size_t)(n + 1) * (m + 1) * (l + 2);
    size_t nw = (size_t)(n + 2) * (m + 2) * (l + 1);
    size_t np_ = (size_t)(n + 2) * (m + 2) * (l + 2);
    f->u = (double*)calloc(nuv, sizeof(double));
    f->v = (double*)calloc(nuv, sizeof(double));
    f->w = (double*)calloc(nw, sizeof(double));
    f->p = (double*)calloc(np_, sizeof(double));
    f->t = (double*)calloc(np_, sizeof(double));
    f->s = (double*)calloc(np_, sizeof(double));
    for (int k = 1; k <= l; k++)
        for (int j = 1; j <= m; j++)
            for (int i = 1; i <= n; i++) {
                FU(f, i, j, k) = un[frow(o, i, j, k, UU)];
                FV(f, i, j, k) = un[frow(o, i, j, k, VV)];
                FW(f, i, j, k) = un[frow(o, i, j, k, WW)];
                FP(f, i, j, k) = un[frow(o, i, j, k, PP)];
                FT(f, i, j, k) = un[frow(o, i, j, k, TT)];
                FS(f, i, j, k) = un[frow(o, i, j, k, SS)];
            }
    for (int k = 1; k <= l; k++)
        for (int j = 1; j <= m; j++) {
            if (o->c.periodic) {
                FU(f, 0, j, k) = FU(f, n, j, k);
                FV(f, 0, j, k) = FV(f, n, j, k);
                FW(f, n + 1, j, k) = FW(f, 1, j, k);
                FW(f, 0, j, k) = FW(f, n, j, k);
                FP(f, n + 1, j, k) = FP(f, 1, j, k);
                FP(f, 0, j, k) = FP(f, n, j, k);
                FT(f, n + 1, j, k) = FT(f, 1, j, k);
                FT(f, 0, j, k) = FT(f, n, j, k);
                FS(f, n + 1, j, k) = FS(f, 1, j, k);
                FS(f, 0, j, k) = FS(f, n, j, k);
            } else {
                FU(f, 0, j, k) = 0.0;
                FU(f, n, j, k) = 0.0;
                FV(f, 0, j, k) = 0.0;
                FV(f, n, j, k) = 0.0;
                FP(f, 0, j, k) = 0.0;
                FP(f, n + 1, j, k) = 0.0;
                FT(f, 0, j, k) = FT(f, 1, j, k);
                FT(f, n + 1, j, k) = FT(f, n, j, k);
                FS(f, 0, j, k) = FS(f, 1, j, k);
                FS(f, n + 1, j, k) = FS(f, n, j, k);
            }
        }
    for (int k = 1; k <= l; k++)
        for (int i = 1; i <= n; i++) {
            FU(f, i, 0, k) = 0.0;
            FU(f, i, m, k) = 0.0;
            FV(f, i, 0, k) = 0.0;
            FV(f, i, m, k) = 0.0;
            FP(f, i, 0, k) = 0.0;
            FP(f, i, m + 1, k) = 0.0;
            FT(f, i, 0, k) = FT(f, i, 1, k);
            FT(f, i, m + 1, k) = FT(f, i, m, k);
            FS(f, i, 0, k) = FS(f, i, 1, k);
            FS(f, i, m + 1, k) = FS(f, i, m, k);
        }
    for (int j = 1; j <= m; j++)
        for (int i = 1; i <= n; i++) {
            FU(f, i, j, 0) = FU(f, i, j, 1);
            FU(f, i, j, l + 1) = FU(f, i, j, l);
            FV(f, i, j, 0) = FV(f, i, j, 1);
            FV(f, i, j, l + 1) = FV(f, i, j, l);
            FW(f, i, j, l) = 0.0;
            FW(f, i, j, 0) = 0.0;
            FP(f, i, j, l + 1) = 0.0;
            FP(f, i, j, 0) = 0.0;
            FT(f, i, j, l + 1) = FT(f, i, j, l);
            FT(f, i, j, 0) = FT(f, i, j, 1);
            FS(f, i, j, l + 1) = FS(f, i, j, l);
            FS(f, i, j, 0) = FS(f, i, j, 1);
        }
    for (int i = 1; i <= n; i++)
        for (int j = 1; j <= m; j++)
            for (int k = 1; k <= l; k++)
                if (LM(o, i, j, k) == 1) {
                    FU(f, i, j, k) = 0.0;
                    FV(f, i, j, k) = 0.0;
                    FU(f, i - 1, j, k) = 0.0;
                    FV(f, i - 1, j, k) = 0.0;
                    FU(f, i, j - 1, k) = 0.0;
                    FV(f, i, j - 1, k) = 0.0;
                    FU(f, i - 1, j - 1, k) = 0.0;
                    FV(f, i - 1, j - 1, k) = 0.0;
                }
}
static void fields_free(fields_t* f)
{
    free(f->u); free(f->v); free(f->w); free(f->p); free(f->t); free(f->s);
}

/* spf.F90:544-665 unlin (per cell) */
static void unlin(const orc_t* o, int type, const fields_t* f, int i, int j, int k, atom_t a)
{
    int n = o->n, m = o->m;
    double dx = o->dx, dy = o->dy;
    azero(a);
    switch (type) {
    case 1: {
        double c = 1.0 / (2 * cos(YV(j)) * dx);
        if (i <= n - 1) a[8] = FU(f, i + 1, j, k) * c;
        if (i >= 2) a[2] = -FU(f, i - 1, j, k) * c;
    } break;
    case 2: {
        double c = 1.0 / (2 * cos(YV(j)) * dx);
        if (i <= n - 1) a[8] = 2 * FU(f, i + 1, j, k) * c;
        if (i >= 2) a[2] = -2 * FU(f, i - 1, j, k) * c;
    } break;
    case 3: {
        double c = 1.0 / (2 * cos(YV(j)) * dy);
        if (j >= 2) a[4] = -FV(f, i, j - 1, k) * cos(YV(j - 1)) * c;
        if (j <= m - 1) a[6] = FV(f, i, j + 1, k) * cos(YV(j + 1)) * c;
    } break;
    case 4: {
        double c = 1.0 / (2 * cos(YV(j)) * dy);
        if (j >= 2) a[4] = -FU(f, i, j - 1, k) * cos(YV(j - 1)) * c;
        if (j <= m - 1) a[6] = FU(f, i, j + 1, k) * cos(YV(j + 1)) * c;
    } break;
    case 5: {
        double td = 1.0 / (8 * DFZT(k) * o->dz);
        a[23] = (FW(f, i, j, k) + FW(f, i, j + 1, k) + FW(f, i + 1, j, k) + FW(f, i + 1, j + 1, k)) * td;
        a[14] = -(FW(f, i, j, k - 1) + FW(f, i, j + 1, k - 1) + FW(f, i + 1, j, k - 1) +
                  FW(f, i + 1, j + 1, k - 1)) * td;
        a[5] = a[14] + a[23];
    } break;
    case 6: {
        double td = 1.0 / (8 * DFZT(k) * o->dz);
        double up = (FU(f, i, j, k) + FU(f, i, j, k + 1)) * td;
        double dn = -(FU(f, i, j, k) + FU(f, i, j, k - 1)) * td;
        a[5] = up; a[6] = up; a[8] = up; a[9] = up;
        a[14] = dn; a[15] = dn; a[17] = dn; a[18] = dn;
    } break;
    case 7:
        a[5] = FV(f, i, j, k) * tan(YV(j));
        break;
    case 8:
        a[5] = FU(f, i, j, k) * tan(YV(j));
        break;
    }
}

/* spf.F90:667-790 vnlin (per cell) */
static void vnlin(const orc_t* o, int type, const fields_t* f, int i, int j, int k, atom_t a)
{
    int n = o->n, m = o->m;
    double dx = o->dx, dy = o->dy;
    azero(a);
    switch (type) {
    case 1: {
        double c = 1.0 / (2 * cos(YV(j)) * dx);
        if (i <= n - 1) a[8] = FU(f, i + 1, j, k) * c;
        if (i >= 2) a[2] = -FU(f, i - 1, j, k) * c;
    } break;
    case 2: {
        double c = 1.0 / (2 * cos(YV(j)) * dx);
        if (i <= n - 1) a[8] = FV(f, i + 1, j, k) * c;
        if (i >= 2) a[2] = -FV(f, i - 1, j, k) * c;
    } break;
    case 3: {
        double c = 1.0 / (2 * cos(YV(j)) * dy);
        if (j <= m - 1) a[6] = FV(f, i, j + 1, k) * cos(YV(j + 1)) * c;
        if (j >= 2) a[4] = -FV(f, i, j - 1, k) * cos(YV(j - 1)) * c;
    } break;
    case 4: {
        double c = 1.0 / (2 * cos(YV(j)) * dy);
        if (j <= m - 1) a[6] = 2 * FV(f, i, j + 1, k) * cos(YV(j + 1)) * c;
        if (j >= 2) a[4] = -2 * FV(f, i, j - 1, k) * cos(YV(j - 1)) * c;
    } break;
    case 5: {
        double td = 1.0 / (8 * DFZT(k) * o->dz);
        a[23] = (FW(f, i, j, k) + FW(f, i, j + 1, k) + FW(f, i + 1, j, k) + FW(f, i + 1, j + 1, k)) * td;
        a[14] = -(FW(f, i, j, k - 1) + FW(f, i, j + 1, k - 1) + FW(f, i + 1, j, k - 1) +
                  FW(f, i + 1, j + 1, k - 1)) * td;
        a[5] = a[14] + a[23];
    } break;
    case 6: {
        double td = 1.0 / (8 * DFZT(k) * o->dz);
        double up = (FV(f, i, j, k) + FV(f, i, j, k + 1)) * td;
        double dn = -(FV(f, i, j, k) + FV(f, i, j, k - 1)) * td;
        a[5] = up; a[6] = up; a[8] = up; a[9] = up;
        a[14] = dn; a[15] = dn; a[17] = dn; a[18] = dn;
    } break;
    case 7:
        a[5] = FU(f, i, j, k) * tan(YV(j));
        break;
    case 8:
        a[5] = 2 * FU(f, i, j, k) * tan(YV(j));
        break;
    }
}

/* spf.F90:486-542 wnlin (t = FT or FS field pointer) */
static void wnlin(const orc_t* o, int type, const double* tf, const fields_t* f, int i, int j,
                  int k, atom_t a)
{
#define TF(ii, jj, kk) (tf[((size_t)(kk) * (f->m + 2) + (jj)) * (f->n + 2) + (ii)])
    azero(a);
    if (k > o->l - 1) return;
    double t0 = TF(i, j, k), t1 = TF(i, j, k + 1);
    switch (type) {
    case 1:
        a[23] = (t0 + t1) / 2.;
        a[5] = (t0 + t1) / 2.;
        break;
    case 2:
        a[23] = t1 / 4.;
        a[5] = (t0 + 2 * t1) / 4.;
        break;
    case 3: {
        double s = t0 + t1;
        a[5] = 0.375 * (s * s);
        a[23] = 0.375 * (s * s);
    } break;
    case 4:
        a[5] = 0.125 * (t0 * t0 + 3 * t1 * t0 + 3 * t1 * t1);
        a[23] = 0.125 * t1 * t1;
        break;
    }
}

/* spf.F90:362-484 tnlin (t = FT or FS field) */
static void tnlin(const orc_t* o, int type, const double* tf, const fields_t* f, int i, int j,
                  int k, atom_t a)
{
    int l = o->l;
    double wet = (double)(1 - LM(o, i, j, l));
    azero(a);
    switch (type) {
    case 2: {
        double c = 1.0 / (4 * cos(Y(j)) * o->dx);
        a[2] = -(TF(i, j, k) + TF(i - 1, j, k)) * c * wet;
        a[4] = (TF(i + 1, j, k) + TF(i, j, k)) * c * wet;
        a[1] = -(TF(i, j, k) + TF(i - 1, j, k)) * c * wet;
        a[5] = (TF(i + 1, j, k) + TF(i, j, k)) * c * wet;
    } break;
    case 3: {
        double c = 1.0 / (4 * cos(Y(j)) * o->dx);
        a[2] = -(FU(f, i - 1, j, k) + FU(f, i - 1, j - 1, k)) * c * wet;
        a[8] = (FU(f, i, j, k) + FU(f, i, j - 1, k)) * c * wet;
        a[5] = a[2] + a[8];
    } break;
    case 4: {
        double c = 1.0 / (4 * cos(Y(j)) * o->dy);
        a[4] = -c * (TF(i, j, k) + TF(i, j - 1, k)) * cos(YV(j - 1)) * wet;
        a[1] = -c * (TF(i, j, k) + TF(i, j - 1, k)) * cos(YV(j - 1)) * wet;
        a[5] = c * (TF(i, j + 1, k) + TF(i, j, k)) * cos(YV(j)) * wet;
        a[2] = c * (TF(i, j + 1, k) + TF(i, j, k)) * cos(YV(j)) * wet;
    } break;
    case 5: {
        double c = 1.0 / (4 * cos(Y(j)) * o->dy);
        a[4] = -(FV(f, i, j - 1, k) + FV(f, i - 1, j - 1, k)) * c * cos(YV(j - 1)) * wet;
        a[6] = (FV(f, i, j, k) + FV(f, i - 1, j, k)) * c * cos(YV(j)) * wet;
        a[5] = a[4] + a[6];
    } break;
    case 6: {
        double td = 1.0 / (2 * o->dz);
        a[14] = -td * wet * (TF(i, j, k) + TF(i, j, k - 1)) / DFZT(k);
        if (k <= l - 1)
            a[5] = td * wet * (TF(i, j, k + 1) + TF(i, j, k)) / DFZT(k);
        else
            a[5] = 0.0;
    } break;
    case 7: {
        double td = 1.0 / (2 * o->dz);
        a[14] = -FW(f, i, j, k - 1) * wet * td / DFZT(k);
        a[23] = FW(f, i, j, k) * wet * td / DFZT(k);
        a[5] = a[14] + a[23];
    } break;
    }
#undef TF
}

/* usrc.F90:873-995 nlin_jac restricted to one cell */
static void nlin_jac_cell(const orc_t* o, const fields_t* f, int i, int j, int k, aloc_t A)
{
    const double* par = o->par;
    double epsr = par[ROSB], Ra = par[RAYL], xes = par[NLES];
    atom_t Urux, uvy1, Urvy1, uwz, Urwz, uvy2, Urvy2;
    unlin(o, 2, f, i, j, k, Urux);
    unlin(o, 3, f, i, j, k, uvy1);
    unlin(o, 4, f, i, j, k, Urvy1);
    unlin(o, 5, f, i, j, k, uwz);
    unlin(o, 6, f, i, j, k, Urwz);
    unlin(o, 7, f, i, j, k, uvy2);
    unlin(o, 8, f, i, j, k, Urvy2);
    for (int s = 1; s <= NP; s++) {
        A[s][UU][UU] = A[s][UU][UU] + epsr * (Urux[s] + uvy1[s] + uwz[s] + uvy2[s]);
        A[s][UU][VV] = A[s][UU][VV] + epsr * (Urvy1[s] + Urvy2[s]);
        A[s][UU][WW] = A[s][UU][WW] + epsr * Urwz[s];
    }
    atom_t uvx, uVrx, Vrvy, vwz, Vrwz, Urt2;
    vnlin(o, 1, f, i, j, k, uvx);
    vnlin(o, 2, f, i, j, k, uVrx);
    vnlin(o, 4, f, i, j, k, Vrvy);
    vnlin(o, 5, f, i, j, k, vwz);
    vnlin(o, 6, f, i, j, k, Vrwz);
    vnlin(o, 8, f, i, j, k, Urt2);
    for (int s = 1; s <= NP; s++) {
        A[s][VV][UU] = A[s][VV][UU] + epsr * (Urt2[s] + uVrx[s]);
        A[s][VV][VV] = A[s][VV][VV] + epsr * (uvx[s] + Vrvy[s] + vwz[s]);
        A[s][VV][WW] = A[s][VV][WW] + epsr * Vrwz[s];
    }
    atom_t t2r, t3r;
    wnlin(o, 1, f->t, f, i, j, k, t2r);
    wnlin(o, 3, f->t, f, i, j, k, t3r);
    for (int s = 1; s <= NP; s++)
        A[s][WW][TT] = A[s][WW][TT] - Ra * xes * alpt2 * t2r[s] + Ra * xes * alpt3 * t3r[s];
    for (int q = 0; q < 2; q++) {
        const double* tf = q == 0 ? f->t : f->s;
        int X = q == 0 ? TT : SS;
        atom_t rx, tx, ry, ty, rz, tz;
        tnlin(o, 2, tf, f, i, j, k, rx);
        tnlin(o, 3, tf, f, i, j, k, tx);
        tnlin(o, 4, tf, f, i, j, k, ry);
        tnlin(o, 5, tf, f, i, j, k, ty);
        tnlin(o, 6, tf, f, i, j, k, rz);
        tnlin(o, 7, tf, f, i, j, k, tz);
        for (int s = 1; s <= NP; s++) {
            A[s][X][UU] = A[s][X][UU] + rx[s];
            A[s][X][VV] = A[s][X][VV] + ry[s];
            A[s][X][WW] = A[s][X][WW] + rz[s];
            A[s][X][X] = A[s][X][X] + tx[s] + ty[s] + tz[s];
        }
    }
}

/* usrc.F90:775-870 nlin_rhs restricted to one cell */
static void nlin_rhs_cell(const orc_t* o, const fields_t* f, int i, int j, int k, aloc_t A)
{
    const double* par = o->par;
    double epsr = par[ROSB], Ra = par[RAYL], xes = par[NLES];
    atom_t uux, uvy1, uwz, uvy2;
    unlin(o, 1, f, i, j, k, uux);
    unlin(o, 3, f, i, j, k, uvy1);
    unlin(o, 5, f, i, j, k, uwz);
    unlin(o, 7, f, i, j, k, uvy2);
    for (int s = 1; s <= NP; s++)
        A[s][UU][UU] = A[s][UU][UU] + epsr * (uux[s] + uvy1[s] + uwz[s] + uvy2[s]);
    atom_t uvx, vvy, vwz, ut2;
    vnlin(o, 1, f, i, j, k, uvx);
    vnlin(o, 3, f, i, j, k, vvy);
    vnlin(o, 5, f, i, j, k, vwz);
    vnlin(o, 7, f, i, j, k, ut2);
    for (int s = 1; s <= NP; s++) {
        A[s][VV][UU] = A[s][VV][UU] + epsr * ut2[s];
        A[s][VV][VV] = A[s][VV][VV] + epsr * (uvx[s] + vvy[s] + vwz[s]);
    }
    atom_t t2r, t3r;
    wnlin(o, 2, f->t, f, i, j, k, t2r);
    wnlin(o, 4, f->t, f, i, j, k, t3r);
    for (int s = 1; s <= NP; s++)
        A[s][WW][TT] = A[s][WW][TT] - Ra * xes * alpt2 * t2r[s] + Ra * xes * alpt3 * t3r[s];
    for (int q = 0; q < 2; q++) {
        const double* tf = q == 0 ? f->t : f->s;
        int X = q == 0 ? TT : SS;
        atom_t ux, vy, wz;
        tnlin(o, 3, tf, f, i, j, k, ux);
        tnlin(o, 5, tf, f, i, j, k, vy);
        tnlin(o, 7, tf, f, i, j, k, wz);
        for (int s = 1; s <= NP; s++) A[s][X][X] = A[s][X][X] + ux[s] + vy[s] + wz[s];
    }
}

/* boundary.F90:2-393 restricted to one cell.  frc_zero[ii] is set to 1 when the
 * Fortran zeroes Frc(find_row2(i,j,k,ii)). */
static void boundaries_cell(const orc_t* o, int i, int j, int k, aloc_t A, int frc_zero[NUN + 1])
{
    int n = o->n, m = o->m, l = o->l;
#define L_(a, b, c) LM(o, a, b, c)
    int southw = L_(i - 1, j - 1, k), west = L_(i - 1, j, k), nwest = L_(i - 1, j + 1, k);
    int south = L_(i, j - 1, k), center = L_(i, j, k), north = L_(i, j + 1, k);
    int southe = L_(i + 1, j - 1, k), east = L_(i + 1, j, k), neast = L_(i + 1, j + 1, k);
    int southwb = L_(i - 1, j - 1, k - 1), westb = L_(i - 1, j, k - 1), nwestb = L_(i - 1, j + 1, k - 1);
    int southb = L_(i, j - 1, k - 1), bottom = L_(i, j, k - 1), northb = L_(i, j + 1, k - 1);
    int southeb = L_(i + 1, j - 1, k - 1), eastb = L_(i + 1, j, k - 1), neastb = L_(i + 1, j + 1, k - 1);
    int southwt = L_(i - 1, j - 1, k + 1), westt = L_(i - 1, j, k + 1), nwestt = L_(i - 1, j + 1, k + 1);
    int southt = L_(i, j - 1, k + 1), top = L_(i, j, k + 1), northt = L_(i, j + 1, k + 1);
    int southet = L_(i + 1, j - 1, k + 1), eastt = L_(i + 1, j, k + 1), neastt = L_(i + 1, j + 1, k + 1);
    int southee = -1, easteast = -1, northee = -1, nnorthee = -1, nnwest = -1, nnorth = -1, nneast = -1;
    if (i < n) {
        southee = L_(i + 2, j - 1, k);
        easteast = L_(i + 2, j, k);
        northee = L_(i + 2, j + 1, k);
        if (j < m) nnorthee = L_(i + 2, j + 2, k);
    }
    if (j < m) {
        nnwest = L_(i, j + 2, k);
        nnorth = L_(i, j + 2, k);
        nneast = L_(i, j + 2, k);
    }
#undef L_
#define ADDC(dst, src, col)                                    \
    for (int r = 1; r <= NUN; r++) A[dst][r][col] = A[dst][r][col] + A[src][r][col];
#define ZEROC(pos, col) for (int r = 1; r <= NUN; r++) A[pos][r][col] = 0.0;
#define ZEROP(pos)                                              \
    for (int r = 1; r <= NUN; r++)                              \
        for (int c = 1; c <= NUN; c++) A[pos][r][c] = 0.0;
#define ZEROROW(row)                                            \
    for (int s = 1; s <= NP; s++)                               \
        for (int c = 1; c <= NUN; c++) A[s][row][c] = 0.0;

    if (center == OCEAN) {
        if (bottom == LAND) {
            if (westb == LAND && southwb == LAND && southb == LAND) { ADDC(1, 10, UU); ADDC(1, 10, VV); }
            ZEROC(10, UU); ZEROC(10, VV);
            if (westb == LAND && neastb == LAND && northb == LAND) { ADDC(2, 11, UU); ADDC(2, 11, VV); }
            ZEROC(11, UU); ZEROC(11, VV);
            if (eastb == LAND && southeb == LAND && southb == LAND) { ADDC(4, 13, UU); ADDC(4, 13, VV); }
            ZEROC(13, UU); ZEROC(13, VV);
            if (eastb == LAND && neastb == LAND && northb == LAND) { ADDC(5, 14, UU); ADDC(5, 14, VV); }
            ADDC(5, 14, TT); ADDC(5, 14, SS);
            ZEROP(14);
        }
        if (southwb == LAND) { ZEROP(10); }
        if (westb == LAND) { ZEROP(11); }
        if (nwestb == LAND) { ZEROP(12); }
        if (southb == LAND) { ZEROP(13); }
        if (northb == LAND) { ZEROP(15); }
        if (southeb == LAND) { ZEROP(16); }
        if (eastb == LAND) { ZEROP(17); }
        if (neastb == LAND) { ZEROP(18); }
        if (top == LAND) {
            if (westt == LAND && southwt == LAND && southt == LAND) { ADDC(1, 19, UU); ADDC(1, 19, VV); }
            ZEROC(19, UU); ZEROC(19, VV);
            if (westt == LAND && nwestt == LAND && northt == LAND) { ADDC(2, 20, UU); ADDC(2, 20, VV); }
            ZEROC(20, UU); ZEROC(20, VV);
            if (eastt == LAND && southet == LAND && southt == LAND) { ADDC(4, 22, UU); ADDC(4, 22, VV); }
            ZEROC(22, UU); ZEROC(22, VV);
            if (eastt == LAND && neastt == LAND && northt == LAND) { ADDC(5, 23, UU); ADDC(5, 23, VV); }
            ADDC(5, 23, TT); ADDC(5, 23, SS);
            ZEROP(23);
            frc_zero[WW] = 1;
            ZEROROW(WW);
            for (int r = 1; r <= NUN; r++) {
                A[5][r][WW] = 1.0e-10;
                A[6][r][WW] = 1.0e-10;
                A[8][r][WW] = 1.0e-10;
                A[9][r][WW] = 1.0e-10;
            }
            A[5][WW][WW] = 1.0;
        }
        if (southwt == LAND) { ZEROP(19); }
        if (westt == LAND) { ZEROP(20); }
        if (nwestt == LAND) { ZEROP(21); }
        if (southt == LAND) { ZEROP(22); }
        if (northt == LAND) { ZEROP(24); }
        if (southet == LAND) { ZEROP(25); }
        if (eastt == LAND) { ZEROP(26); }
        if (neastt == LAND) { ZEROP(27); }
        if (southw == LAND) { ZEROC(1, UU); ZEROC(1, VV); }
        if (west == LAND) {
            ADDC(5, 2, TT); ADDC(5, 2, SS);
            ZEROP(2);
            ZEROC(1, UU); ZEROC(1, VV);
        }
        if (nwest == LAND) {
            ZEROC(2, UU); ZEROC(2, VV); ZEROC(3, UU); ZEROC(3, VV);
        } else if (j < m) {
            if (nnwest == LAND) { ZEROC(3, UU); ZEROC(3, VV); }
        }
        if (south == LAND) {
            ADDC(5, 4, SS); ADDC(5, 4, TT);
            ZEROP(4);
            ZEROC(1, UU); ZEROC(1, VV);
        }
        if (north == LAND) {
            ZEROC(2, UU); ZEROC(2, VV);
            A[2][PP][UU] = 0.0; A[2][PP][VV] = 0.0;
            A[5][PP][UU] = 0.0; A[5][PP][VV] = 0.0;
            frc_zero[VV] = 1;
            ZEROROW(VV);
            ZEROC(5, VV);
            A[5][VV][VV] = 1.0;
            frc_zero[UU] = 1;
            ZEROROW(UU);
            ZEROC(5, UU);
            A[5][UU][UU] = 1.0;
            ADDC(5, 6, SS); ADDC(5, 6, TT);
            ZEROP(6);
        } else if (j < m) {
            if (nnorth == LAND) { ZEROC(3, UU); ZEROC(3, VV); ZEROC(6, UU); ZEROC(6, VV); }
        }
        if (southe == LAND) {
            ZEROC(4, UU); ZEROC(4, VV); ZEROC(7, UU); ZEROC(7, VV);
        } else if (i < n) {
            if (southee == LAND) { ZEROC(7, UU); ZEROC(7, VV); }
        }
        if (east == LAND) {
            ZEROC(4, UU); ZEROC(4, VV);
            A[4][PP][UU] = 0.0; A[4][PP][VV] = 0.0;
            A[5][PP][UU] = 0.0; A[5][PP][VV] = 0.0;
            frc_zero[UU] = 1;
            ZEROROW(UU);
            ZEROC(5, UU);
            A[5][UU][UU] = 1.0;
            frc_zero[VV] = 1;
            ZEROROW(VV);
            ZEROC(5, VV);
            A[5][VV][VV] = 1.0;
            ADDC(5, 8, SS); ADDC(5, 8, TT);
            ZEROP(8);
            ZEROC(7, UU); ZEROC(7, VV);
        } else if (i < n) {
            if (easteast == LAND) { ZEROC(7, UU); ZEROC(7, VV); ZEROC(8, UU); ZEROC(8, VV); }
        }
        if (neast == LAND) {
            frc_zero[UU] = 1;
            ZEROROW(UU);
            ZEROC(5, UU);
            A[5][UU][UU] = 1.0;
            frc_zero[VV] = 1;
            ZEROROW(VV);
            ZEROC(5, VV);
            A[5][VV][VV] = 1.0;
            ZEROC(7, UU); ZEROC(7, VV);
        } else if (i < n || j < m) {
            if (i < n) {
                if (northee == LAND) {
                    ZEROC(8, UU); ZEROC(8, VV); ZEROC(9, UU); ZEROC(9, VV);
                } else if (j < m) {
                    if (nnorthee == LAND) { ZEROC(9, UU); ZEROC(9, VV); }
                }
            }
            if (j < m) {
                if (nneast == LAND) { ZEROC(6, UU); ZEROC(6, VV); ZEROC(9, UU); ZEROC(9, VV); }
            }
        }
    } else {
        memset(A, 0, sizeof(aloc_t));
        for (int ii = 1; ii <= NUN; ii++) {
            frc_zero[ii] = 1;
            A[5][ii][ii] = 1.0;
        }
    }
    (void)l;
#undef ADDC
#undef ZEROC
#undef ZEROP
#undef ZEROROW
}

/* assemble.F90:142-179 shift */
static inline void shiftkk(const orc_t* o, int i, int j, int k, int kk, int* i2, int* j2, int* k2)
{
    if (kk < 10) {
        *k2 = k;
        *j2 = j - 1 + (kk + 2) % 3;
        *i2 = i - 1 + (kk - 1) / 3;
    } else if (kk < 19) {
        *k2 = k - 1;
        *j2 = j - 1 + (kk + 2) % 3;
        *i2 = i - 1 + (kk - 10) / 3;
    } else {
        *k2 = k + 1;
        *j2 = j - 1 + (kk + 2) % 3;
        *i2 = i - 1 + (kk - 19) / 3;
    }
    if (o->c.periodic) {
        if (*i2 == 0) *i2 = o->n;
        else if (*i2 == o->n + 1) *i2 = 1;
    }
}


/* ---- vertical mixing (mix_imp.f vmix_fun 231-562, vmix_jac 729-815) ---------------
 * Restricted to the default mixing parameters of stpnt (usrc.F90:1169-1176): MIXP =
 * MKAP = 0 (no neutral physics / Gent-McWilliams) and ALPC = 1 (no energetically
 * consistent mixing), which leaves the implicit convective vertical mixing of T and S:
 *   Ftimp(k) = -tprstb(-drhodzt(k), SPL1) * P_VC * dtdzt(k)   (top face of cell k)
 *   mix(T)   = (Ftimp(k) - Ftimp(k-1)) / (dz dfzT(k))          (rho_mixing off)      */
static int mix_supported(const orc_t* o)
{
    const double* par = o->par;
    return par[MIXP] == 0.0 && par[MKAP] == 0.0 && (1.0 - par[ALPC]) * par[ENER] * par[PE_V] == 0.0;
}
static inline double isoc_(const orc_t* o, int i, int j, int k)
{
    const int lm = LM(o, i, j, k);
    return (lm == OCEAN || lm == 3) ? 1.0 : 0.0;      /* OCEAN or PERIO (par.F90:78-81) */
}
/* tprstb (mix_imp.f:836-856) */
static inline double tprstb_(const orc_t* o, double grad, double spl)
{
    const double fac = o->c.alphaT * spl;
    const double x = -grad * fac;
    const double t = tanh(x * x * x);
    return t > 0.0 ? t : 0.0;
}
/* Ftimp, Fsimp on the top face of cell (i,j,k) from t, s at k and k+1 (dCdzt, drhodC) */
static void mix_face(const orc_t* o, int i, int j, int k, double t0, double t1, double s0,
                     double s1, double* ft, double* fs)
{
    const double* par = o->par;
    const double lambda = par[LAMB], xes = par[NLES], kvc = par[P_VC], sp1 = par[SPL1];
    if (kvc == 0.0) { *ft = *fs = 0.0; return; }
    const double r0 = lambda * s0 - t0 - xes * (alpt1 * t0 + alpt2 * t0 * t0 - alpt3 * t0 * t0 * t0);
    const double r1 = lambda * s1 - t1 - xes * (alpt1 * t1 + alpt2 * t1 * t1 - alpt3 * t1 * t1 * t1);
    const double iso = isoc_(o, i, j, k + 1) * isoc_(o, i, j, k);
    const double dzw = o->dz * DFZW(k);
    const double dtdz = iso * (t1 - t0) / dzw, dsdz = iso * (s1 - s0) / dzw;
    const double drdz = iso * (r1 - r0) / dzw;
    const double tpr = tprstb_(o, -drdz, sp1);
    *ft = -tpr * kvc * dtdz;
    *fs = -tpr * kvc * dsdz;
}
/* mix of row var (TT or SS) of cell (i,j,k) from t, s at k-1, k, k+1 (index 0..2) */
static double mix_row(const orc_t* o, int var, int i, int j, int k, const double* t3, const double* s3)
{
    const double* par = o->par;
    const double lambda = par[LAMB], xes = par[NLES];
    if ((var == TT && !o->vmix_temp) || (var == SS && !o->vmix_salt)) return 0.0;
    double ftk, fsk, ftm = 0.0, fsm = 0.0;
    mix_face(o, i, j, k, t3[1], t3[2], s3[1], s3[2], &ftk, &fsk);
    if (k >= 2) mix_face(o, i, j, k - 1, t3[0], t3[1], s3[0], s3[1], &ftm, &fsm);
    if (o->c.rho_mixing && xes == 0.0) {
        if (var == TT) return ((ftk - ftm) - (fsk - fsm) * lambda) / (2.0 * o->dz * DFZT(k)) + 0.0;
        return ((fsk - fsm) - (ftk - ftm) / lambda) / (2.0 * o->dz * DFZT(k)) + 0.0;
    }
    if (var == TT) return (ftk - ftm) / (o->dz * DFZT(k)) + 0.0;
    return (fsk - fsm) / (o->dz * DFZT(k)) + 0.0;
}
static void mix_col(const fields_t* f, int i, int j, int k, double* t3, double* s3)
{
    for (int d = 0; d < 3; d++) {
        t3[d] = FT(f, i, j, k - 1 + d);
        s3[d] = FS(f, i, j, k - 1 + d);
    }
}
static int mix_active(const orc_t* o) { return o->c.vmix != 0 && (o->vmix_temp || o->vmix_salt); }
/* vmix_control (mix_imp.f:131-166): flag 2 fixes T/S mixing at the first evaluation */
static void mix_control(orc_t* o, const double* x)
{
    if (o->c.vmix != 2 || o->vmix_fix) return;
    double st = 0.0, ss = 0.0;
    for (int r = 0; r < o->ndim; r += NUN) {
        st += x[r + TT - 1] * x[r + TT - 1];
        ss += x[r + SS - 1] * x[r + SS - 1];
    }
    o->vmix_temp = sqrt(st) > 1.0e-12;
    o->vmix_salt = sqrt(ss) > 1.0e-12;
    /* vmix_control partitions only when T mixes (mix_imp.f:158): salt-only mixing is off */
    if (!o->vmix_temp) o->vmix_salt = 0;
    o->vmix_fix = 1;
}
/* vmix_jac: forward differences (eps 1e-8) of mix w.r.t. the T/S unknowns of the
 * column neighbours k-1, k, k+1, added to An before boundaries */
static void mix_jac_cell(const orc_t* o, const fields_t* f, int i, int j, int k, aloc_t A)
{
    if (!mix_active(o) || LM(o, i, j, k) != OCEAN) return;
    const double eps = 1.0e-08;
    double t3[3], s3[3];
    mix_col(f, i, j, k, t3, s3);
    for (int var = TT; var <= SS; var++) {
        if ((var == TT && !o->vmix_temp) || (var == SS && !o->vmix_salt)) continue;
        const double m0 = mix_row(o, var, i, j, k, t3, s3);
        for (int d = 0; d < 3; d++) {
            const int kk = k - 1 + d;
            const int lm = LM(o, i, j, kk);
            if (lm != OCEAN && lm != 3) continue;
            const int pos = d == 0 ? 14 : (d == 1 ? 5 : 23);
            for (int cv = TT; cv <= SS; cv++) {
                if ((cv == TT && !o->vmix_temp) || (cv == SS && !o->vmix_salt)) continue;
                double tp[3] = {t3[0], t3[1], t3[2]}, sp[3] = {s3[0], s3[1], s3[2]};
                if (cv == TT) tp[d] = tp[d] + eps;
                else sp[d] = sp[d] + eps;
                const double m1 = mix_row(o, var, i, j, k, tp, sp);
                A[pos][var][cv] = A[pos][var][cv] + (m1 - m0) / eps;
            }
        }
    }
}

/* Build the final local block An(27,6,6) of cell (i,j,k) as matrix() (jac=1) or
 * rhs() (jac=0) would, before fillcolA. */
static void cell_block(const orc_t* o, const fields_t* f, int i, int j, int k, int jac, aloc_t A,
                       int frc_zero[NUN + 1])
{
    lin_cell(o, i, j, k, A);
    if (jac) {
        nlin_jac_cell(o, f, i, j, k, A);
        mix_jac_cell(o, f, i, j, k, A);
    } else {
        nlin_rhs_cell(o, f, i, j, k, A);
    }
    for (int q = 0; q <= NUN; q++) frc_zero[q] = 0;
    boundaries_cell(o, i, j, k, A, frc_zero);
}

/* fillcolB (assemble.F90:18-54) for one cell */
static void fillcolB_cell(const orc_t* o, int i, int j, int k, double* coB)
{
    for (int q = UU; q <= SS; q++) coB[frow(o, i, j, k, q)] = 0.0;
    if (LM(o, i, j, k) == OCEAN) {
        if (LM(o, i + 1, j, k) != LAND) coB[frow(o, i, j, k, UU)] = -o->par[ROSB];
        if (LM(o, i, j + 1, k) != LAND) coB[frow(o, i, j, k, VV)] = -o->par[ROSB];
        coB[frow(o, i, j, k, TT)] = -1.0;
        coB[frow(o, i, j, k, SS)] = -1.0;
    }
}

/* ================================================================================ */
orc_t* orc_create(const orc_cfg* cfg, const int* landm, const double* spert)
{
    if (cfg->ite != 1 || cfg->its != 1 || cfg->iza != 2 || cfg->vmix < 0 || cfg->vmix > 2) {
        fprintf(stderr, "orc_create: only idealized forcing, vmix 0..2 supported\n");
        return NULL;
    }
    orc_t* o = (orc_t*)calloc(1, sizeof(orc_t));
    o->c = *cfg;
    /* mix_imp.f vmix_init (58-109): flag 1 mixes T and S from the start, flag 2 decides
     * at the first matrix/rhs evaluation (vmix_control) */
    o->vmix_temp = o->vmix_salt = cfg->vmix == 1;
    o->vmix_fix = cfg->vmix != 2;
    int n = cfg->n, m = cfg->m, l = cfg->l;
    o->n = n; o->m = m; o->l = l;
    o->ncell = n * m * l;
    o->ndim = NUN * o->ncell;
    const double PI_ = 3.14159265358979323846; /* THCM.C PI_ */
    o->xmin = cfg->xmin_deg * PI_ / 180.0;
    o->xmax = cfg->xmax_deg * PI_ / 180.0;
    o->ymin = cfg->ymin_deg * PI_ / 180.0;
    o->ymax = cfg->ymax_deg * PI_ / 180.0;
    o->x = (double*)calloc(n + 2, sizeof(double));
    o->y = (double*)calloc(m + 2, sizeof(double));
    o->z = (double*)calloc(l + 2, sizeof(double));
    o->xu = (double*)calloc(n + 2, sizeof(double));
    o->yv = (double*)calloc(m + 2, sizeof(double));
    o->zw = (double*)calloc(l + 2, sizeof(double));
    o->ze = (double*)calloc(l + 2, sizeof(double));
    o->zwe = (double*)calloc(l + 2, sizeof(double));
    o->dfzT = (double*)calloc(l + 2, sizeof(double));
    o->dfzW = (double*)calloc(l + 2, sizeof(double));
    size_t nl = (size_t)(n + 2) * (m + 2) * (l + 2);
    o->landm = (int*)malloc(nl * sizeof(int));
    memcpy(o->landm, landm, nl * sizeof(int));
    /* usrc.F90:83-107 */
    for (int k = 0; k <= l + 1; k++)
        for (int j = 0; j <= m + 1; j++)
            for (int i = 0; i <= n + 1; i++) {
                if (!cfg->periodic && LM(o, i, j, k) == 3) LM(o, i, j, k) = OCEAN;
                if (!cfg->periodic && (i == 0 || i == n + 1)) LM(o, i, j, k) = LAND;
                if (j == 0 || j == m + 1 || k == 0 || k == l + 1) LM(o, i, j, k) = LAND;
            }
    o->taux = (double*)calloc((size_t)n * m, sizeof(double));
    o->tauy = (double*)calloc((size_t)n * m, sizeof(double));
    o->tatm = (double*)calloc((size_t)n * m, sizeof(double));
    o->emip = (double*)calloc((size_t)n * m, sizeof(double));
    o->spert = (double*)calloc((size_t)n * m, sizeof(double));
    o->qatm = (double*)calloc((size_t)n * m, sizeof(double));
    o->albe = (double*)calloc((size_t)n * m, sizeof(double));
    o->patm = (double*)calloc((size_t)n * m, sizeof(double));
    o->suno = (double*)calloc((size_t)m + 2, sizeof(double));
    if (spert) memcpy(o->spert, spert, sizeof(double) * n * m);
    o->Frc = (double*)calloc(o->ndim, sizeof(double));
    grid(o);
    double dzne = o->dz * DFZT(l);
    o->QTnd = r0dim / (udim * cp0 * rhodim * cfg->hdim * dzne);
    o->QSnd = s0 * r0dim / (deltas * udim * cfg->hdim * dzne);
    /* atmos_coef (usrc.F90:1183-1223) */
    {
        const double muoa = rhoa_atm * ch_atm * cpa_atm * uw_atm;
        o->Os = sun0_atm * c0_atm / 4 * o->QTnd;
        o->Ooa = muoa * o->QTnd;
        for (int j = 1; j <= m; j++) {
            const double sy = sin(Y(j));
            o->suno[j] = o->Os * (1 - .482 * (3 * (sy * sy) - 1.) / 2.);
        }
    }
    stpnt(o);
    forcing(o);
    /* integral condition row (THCM.C:661-711) */
    o->rowintcon = -1;
    if (cfg->sres == 0) {
        int Nic = cfg->nic == -1 ? n - 1 : cfg->nic;
        int Mic = cfg->mic == -1 ? m - 1 : cfg->mic;
        o->rowintcon = NUN * ((l - 1) * n * m + n * Mic + Nic) + SS - 1;
    }
    /* maximal graph (THCM.C:2241-2539) */
    o->gptr = (int64_t*)calloc(o->ndim + 1, sizeof(int64_t));
    int* tmp = (int*)malloc(sizeof(int) * 32);
    int cap = o->ndim * 24 + o->ncell + 16;
    o->gcol = (int*)malloc(sizeof(int) * (size_t)cap);
    int64_t pos = 0;
    for (int row = 0; row < o->ndim; row++) {
        o->gptr[row] = pos;
        int cell = row / NUN, var = row % NUN + 1;
        int i0 = cell % n, j0 = (cell / n) % m, k0 = cell / (n * m);
        int cnt = 0;
#define INS(di, dj, dk, X)                                                           \
    do {                                                                           \
        int ii = i0 + (di), jj = j0 + (dj), kk = k0 + (dk);                         \
        if (cfg->periodic) ii = ((ii % n) + n) % n;                                 \
        if (ii >= 0 && jj >= 0 && kk >= 0 && ii < n && jj < m && kk < l)             \
            tmp[cnt++] = NUN * (kk * n * m + n * jj + ii) + (X) - 1;                 \
    } while (0)
        if (row == o->rowintcon) {
            for (int ii = 0; ii < n; ii++)
                for (int jj = 0; jj < m; jj++)
                    for (int kk = 0; kk < l; kk++) o->gcol[pos++] = NUN * (kk * n * m + n * jj + ii) + SS - 1;
            /* sort */
            int64_t b = o->gptr[row];
            for (int64_t a = b + 1; a < pos; a++) {
                int v = o->gcol[a];
                int64_t c = a - 1;
                while (c >= b && o->gcol[c] > v) { o->gcol[c + 1] = o->gcol[c]; c--; }
                o->gcol[c + 1] = v;
            }
            continue;
        }
        switch (var) {
        case UU:
        case VV: {
            int A = var, B = var == UU ? VV : UU;
            INS(0, 0, 0, A); INS(-1, 0, 0, A); INS(1, 0, 0, A); INS(0, -1, 0, A); INS(0, 1, 0, A);
            INS(0, 0, -1, A); INS(0, 0, 1, A);
            INS(0, 0, 0, B); INS(-1, 0, 0, B); INS(1, 0, 0, B);
            if (var == UU) { INS(0, -1, 0, B); INS(0, 1, 0, B); }
            INS(0, 0, 0, WW); INS(1, 0, 0, WW); INS(1, 1, 0, WW); INS(0, 1, 0, WW);
            INS(0, 0, -1, WW); INS(1, 0, -1, WW); INS(1, 1, -1, WW); INS(0, 1, -1, WW);
            INS(0, 0, 0, PP); INS(1, 0, 0, PP); INS(0, 1, 0, PP); INS(1, 1, 0, PP);
        } break;
        case WW:
            INS(0, 0, 0, WW); INS(0, 0, 0, PP); INS(0, 0, 1, PP); INS(0, 0, 0, TT); INS(0, 0, 1, TT);
            INS(0, 0, 0, SS); INS(0, 0, 1, SS);
            break;
        case PP:
            INS(0, 0, 0, PP);
            INS(0, 0, 0, UU); INS(-1, 0, 0, UU); INS(0, -1, 0, UU); INS(-1, -1, 0, UU);
            INS(0, 0, 0, VV); INS(-1, 0, 0, VV); INS(0, -1, 0, VV); INS(-1, -1, 0, VV);
            INS(0, 0, 0, WW); INS(0, 0, -1, WW);
            break;
        case TT:
        case SS: {
            int A = var, B = var == TT ? SS : TT;
            INS(0, 0, 0, A); INS(-1, 0, 0, A); INS(1, 0, 0, A); INS(0, -1, 0, A); INS(0, 1, 0, A);
            INS(0, 0, -1, A); INS(0, 0, 1, A);
            INS(0, 0, 0, UU); INS(-1, 0, 0, UU); INS(-1, -1, 0, UU); INS(0, -1, 0, UU);
            INS(0, 0, 0, VV); INS(-1, 0, 0, VV); INS(-1, -1, 0, VV); INS(0, -1, 0, VV);
            INS(0, 0, 0, WW); INS(0, 0, -1, WW);
            INS(0, 0, 0, B); INS(0, 0, -1, B); INS(0, 0, 1, B);
        } break;
        }
#undef INS
        /* sort + dedupe (Epetra FillComplete) */
        for (int a = 1; a < cnt; a++) {
            int v = tmp[a], c = a - 1;
            while (c >= 0 && tmp[c] > v) { tmp[c + 1] = tmp[c]; c--; }
            tmp[c + 1] = v;
        }
        for (int a = 0; a < cnt; a++)
            if (a == 0 || tmp[a] != tmp[a - 1]) o->gcol[pos++] = tmp[a];
    }
    o->gptr[o->ndim] = pos;
    free(tmp);
    return o;
}

void orc_destroy(orc_t* o)
{
    if (!o) return;
    free(o->x); free(o->y); free(o->z); free(o->xu); free(o->yv); free(o->zw); free(o->ze);
    free(o->zwe); free(o->dfzT); free(o->dfzW); free(o->landm); free(o->taux); free(o->tauy);
    free(o->tatm); free(o->emip); free(o->spert);
    free(o->qatm); free(o->albe); free(o->patm); free(o->suno); free(o->Frc); free(o->gptr); free(o->gcol);
    free(o);
}

/* usrc.F90:163-181 setparcs: set, then forcing + lin (lin is evaluated lazily here) */
void orc_set_par(orc_t* o, int idx, double v)
{
    if (idx >= 1 && idx <= 30) o->par[idx] = v;
    forcing(o);
}
double orc_get_par(const orc_t* o, int idx) { return (idx >= 1 && idx <= 30) ? o->par[idx] : 0.0; }
int orc_nrows(const orc_t* o) { return o->ndim; }
int orc_rowintcon(const orc_t* o) { return o->rowintcon; }
const int* orc_landm(const orc_t* o) { return o->landm; }
int64_t orc_graph_nnz(const orc_t* o) { return o->gptr[o->ndim]; }
void orc_graph(const orc_t* o, int64_t* rowptr, int* col)
{
    memcpy(rowptr, o->gptr, sizeof(int64_t) * (o->ndim + 1));
    memcpy(col, o->gcol, sizeof(int) * (size_t)o->gptr[o->ndim]);
}

/* matrix() + assemble/fillcolA (assemble.F90:57-139): Fortran CSR, 1-based */
int64_t orc_fortran_matrix(orc_t* o, const double* x, int* beg, int* jco, double* co, double* coB)
{
    mix_control(o, x);
    if (mix_active(o) && !mix_supported(o)) {
        fprintf(stderr, "oracle: neutral physics / GM / consistent mixing not restated\n");
        abort();
    }
    fields_t f;
    usol(o, x, &f);
    int64_t v = 1;
    int row = 1;
    aloc_t* A = (aloc_t*)malloc(sizeof(aloc_t));
    int fz_[NUN + 1];
    for (int k = 1; k <= o->l; k++)
        for (int j = 1; j <= o->m; j++)
            for (int i = 1; i <= o->n; i++) {
                cell_block(o, &f, i, j, k, 1, *A, fz_);
                if (coB) fillcolB_cell(o, i, j, k, coB);
                for (int ii = 1; ii <= NUN; ii++) {
                    if (beg) beg[row - 1] = (int)v;
                    for (int kk = 1; kk <= NP; kk++)
                        for (int jj = 1; jj <= NUN; jj++) {
                            double a = (*A)[kk][ii][jj];
                            if (fabs(a) > 1.0e-10) {
                                int i2, j2, k2;
                                shiftkk(o, i, j, k, kk, &i2, &j2, &k2);
                                if (co) co[v - 1] = a;
                                if (jco) jco[v - 1] = frow(o, i2, j2, k2, jj) + 1;
                                v++;
                            }
                        }
                    row++;
                }
            }
    if (beg) beg[o->ndim] = (int)v;
    free(A);
    fields_free(&f);
    return v - 1;
}

/* rhs() (usrc.F90:506-586) with ires = 0: B = (-Au - mix + Frc_eff)*(1-landm) */
void orc_fortran_rhs(orc_t* o, const double* x, double* B)
{
    mix_control(o, x);
    if (mix_active(o) && !mix_supported(o)) {
        fprintf(stderr, "oracle: neutral physics / GM / consistent mixing not restated\n");
        abort();
    }
    fields_t f;
    usol(o, x, &f);
    int n = o->n, m = o->m, l = o->l;
#pragma omp parallel
    {
        aloc_t* A = (aloc_t*)malloc(sizeof(aloc_t));
        int fz_[NUN + 1];
#pragma omp for schedule(static)
        for (int c = 0; c < o->ncell; c++) {
            int i = c % n + 1, j = (c / n) % m + 1, k = c / (n * m) + 1;
            cell_block(o, &f, i, j, k, 0, *A, fz_);
            for (int ii = 1; ii <= NUN; ii++) {
                int row = frow(o, i, j, k, ii);
                double au = 0.0;
                for (int kk = 1; kk <= NP; kk++)
                    for (int jj = 1; jj <= NUN; jj++) {
                        double a = (*A)[kk][ii][jj];
                        if (fabs(a) > 1.0e-10) {
                            int i2, j2, k2;
                            shiftkk(o, i, j, k, kk, &i2, &j2, &k2);
                            au = a * x[frow(o, i2, j2, k2, jj)] + au;
                        }
                    }
                double frc = fz_[ii] ? 0.0 : o->Frc[row];
                double mx = 0.0;
                if ((ii == TT || ii == SS) && mix_active(o)) {
                    double t3[3], s3[3];
                    mix_col(&f, i, j, k, t3, s3);
                    mx = mix_row(o, ii, i, j, k, t3, s3);
                }
                double b = -au - mx + frc - 0.0 * (1 - o->par[RESC]) * 0.0;
                B[row] = b * (1 - LM(o, i, j, k));
            }
        }
        free(A);
    }
    (void)l;
    fields_free(&f);
}

void orc_intcond_coeff(const orc_t* o, double* coeff)
{
    memset(coeff, 0, sizeof(double) * o->ndim);
    for (int k = 1; k <= o->l; k++)
        for (int j = 1; j <= o->m; j++)
            for (int i = 1; i <= o->n; i++)
                if (LM(o, i, j, k) == OCEAN) coeff[frow(o, i, j, k, SS)] = cos(Y(j)) * DFZT(k);
}

/* THCM::evaluate(computeJac) (THCM.C:1035-1173): place the Fortran rows into the
 * maximal graph, intcond_S row (2121-2198), B = coB*Mass (Mass = 1). */
void orc_jacobian(orc_t* o, const double* x, double* val, double* diagB)
{
    mix_control(o, x);
    if (mix_active(o) && !mix_supported(o)) {
        fprintf(stderr, "oracle: neutral physics / GM / consistent mixing not restated\n");
        abort();
    }
    fields_t f;
    usol(o, x, &f);
    int n = o->n, m = o->m;
    memset(val, 0, sizeof(double) * (size_t)o->gptr[o->ndim]);
#pragma omp parallel
    {
        aloc_t* A = (aloc_t*)malloc(sizeof(aloc_t));
        int fz_[NUN + 1];
#pragma omp for schedule(static)
        for (int c = 0; c < o->ncell; c++) {
            int i = c % n + 1, j = (c / n) % m + 1, k = c / (n * m) + 1;
            cell_block(o, &f, i, j, k, 1, *A, fz_);
            if (diagB) fillcolB_cell(o, i, j, k, diagB);
            for (int ii = 1; ii <= NUN; ii++) {
                int row = frow(o, i, j, k, ii);
                if (row == o->rowintcon) continue;
                int64_t b = o->gptr[row], e = o->gptr[row + 1];
                for (int kk = 1; kk <= NP; kk++)
                    for (int jj = 1; jj <= NUN; jj++) {
                        double a = (*A)[kk][ii][jj];
                        if (fabs(a) > 1.0e-10) {
                            int i2, j2, k2;
                            shiftkk(o, i, j, k, kk, &i2, &j2, &k2);
                            int colx = frow(o, i2, j2, k2, jj);
                            int64_t lo = b, hi = e - 1, hit = -1;
                            while (lo <= hi) {
                                int64_t mid = (lo + hi) / 2;
                                if (o->gcol[mid] == colx) { hit = mid; break; }
                                if (o->gcol[mid] < colx) lo = mid + 1; else hi = mid - 1;
                            }
                            if (hit < 0) {
                                fprintf(stderr, "orc_jacobian: entry (%d,%d) outside maximal graph\n", row, colx);
                                abort();
                            }
                            val[hit] = a;
                        }
                    }
            }
        }
        free(A);
    }
    if (o->rowintcon >= 0) {
        double* coeff = (double*)malloc(sizeof(double) * o->ndim);
        orc_intcond_coeff(o, coeff);
        for (int64_t p = o->gptr[o->rowintcon]; p < o->gptr[o->rowintcon + 1]; p++)
            val[p] = o->c.int_sign * coeff[o->gcol[p]];
        if (diagB) diagB[o->rowintcon] = 0.0;
        free(coeff);
    }
    fields_free(&f);
}

/* THCM::evaluate(rhs) (THCM.C:985-1033): F = -B, intcond row, intCorrection = 0 */
void orc_rhs(orc_t* o, const double* x, double* F)
{
    orc_fortran_rhs(o, x, F);
    for (int r = 0; r < o->ndim; r++) F[r] = -F[r];
    if (o->rowintcon >= 0) {
        double* coeff = (double*)malloc(sizeof(double) * o->ndim);
        orc_intcond_coeff(o, coeff);
        double s = 0.0;
        for (int r = 0; r < o->ndim; r++) s += coeff[r] * x[r];
        F[o->rowintcon] = o->c.int_sign * (s - 0.0);
        free(coeff);
    }
}

void orc_csr_spmv(int nrows, const int64_t* rowptr, const int* col, const double* val,
                  const double* x, double* y)
{
#pragma omp parallel for schedule(static)
    for (int r = 0; r < nrows; r++) {
        double s = 0.0;
        for (int64_t p = rowptr[r]; p < rowptr[r + 1]; p++) s += val[p] * x[col[p]];
        y[r] = s;
    }
}

/* Ocean::synchronize(atmos): inserts.F90 setters and set_atmos_parameters (usrc.F90:237-293,
 * pars = AtmosLocal::CommPars: tdim, qdim, nuq, eta, dqso, dqsi, dqdt, Eo0, Ei0, Cs, t0o, t0i,
 * a0, da, tauf, tauc, comb, albf), then forcing */
void orc_set_atmos(orc_t* o, const double* t, const double* q, const double* a, const double* p,
                   const double* pars)
{
    const size_t nm = (size_t)o->n * o->m;
    memcpy(o->tatm, t, sizeof(double) * nm);
    memcpy(o->qatm, q, sizeof(double) * nm);
    memcpy(o->albe, a, sizeof(double) * nm);
    if (p) memcpy(o->patm, p, sizeof(double) * nm);
    else memset(o->patm, 0, sizeof(double) * nm);
    o->qdim_a = pars[1];
    o->eta_a = pars[3];
    o->dqso = pars[4];
    o->eo0 = pars[7];
    o->albe0 = pars[12];
    o->albed = pars[13];
    o->nus = o->par[COMB] * o->par[SALT] * o->eta_a * o->qdim_a * o->QSnd;
    o->lvsc = o->par[COMB] * o->par[TEMP] * rhodim * lv_atm * o->QTnd;
    forcing(o);
}

/* getdeps (usrc.F90:201-219) */
void orc_get_deps(const orc_t* o, double* out)
{
    out[0] = o->Ooa;
    out[1] = o->Os;
    out[2] = o->nus;
    out[3] = o->eta_a;
    out[4] = o->lvsc;
    out[5] = o->qdim_a;
    out[6] = o->par[COMB] * o->par[SALT] * o->QSnd;
}
