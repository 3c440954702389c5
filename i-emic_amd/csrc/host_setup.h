/*
 * host_setup.h -- one-time set-up of the 1-D metric tables, parameters and land mask.
 *
 * Restates the serial set-up path of the THCM constructor (src/ocean/THCM.C:178-798):
 *   init_ border handling of the land mask       usrc.F90:83-107
 *   grid                                         grid.F90:2-95
 *   QTnd / QSnd                                  usrc.F90:125-127
 *   stpnt + vmix_par                             usrc.F90:1136-1180, mix_imp.f vmix_par
 *   forcing profiles wfun/temfun/salfun          forcing.F90:489-533
 *   intcond coefficients                         thcm_utils.F90:285-312
 * Only 1-D tables (length m+2, l+2) and scalars are produced here; they are evaluated
 * with the same libm the reference uses so that the per-cell device arithmetic is
 * bit-identical.  Pure C++ (shared by the device library and its CPU unit test).
 */
#ifndef IEMIC_HOST_SETUP_H
#define IEMIC_HOST_SETUP_H

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "../../include/iemic.h"
#include "stencil.h"

namespace iemic {
namespace host {

constexpr double pi_ = 3.14159265358979323846;     /* par.F90:14, THCM.C PI_ */
constexpr double omegadim = 7.292e-05, r0dim = 6.37e+06, udim = 0.1e+00, gdim = 9.8e+00;
constexpr double rhodim = 1.024e+03, deltas = 1.0, s0 = 35.0, cp0 = 4.2e+03;
constexpr double ah = 2.5e+05, av = 1.0e-03, kappah = 1.0e+03, kappav = 1.0e-04;
constexpr double zmin = -1.0, zmax = 0.0;
/* m_atm constants (atm.F90:5-19) */
constexpr double rhoa_atm = 1.25, ch_atm = 0.94 * 1.3e-03, cpa_atm = 1000., uw_atm = 8.5;
constexpr double sun0_atm = 1360., c0_atm = 0.43, lv_atm = 2.5e+06;

inline double fz(double z, double qz)
{
    double th = std::tanh(qz * (z + 1));
    double tth = std::tanh(qz);
    if (qz > 1.0) return -1 + th / tth;
    return z + (1. - qz) * z * (1 - z);
}
inline double dfdz(double z, double qz)
{
    double ch = std::cosh(qz * (z + 1));
    double tth = std::tanh(qz);
    if (qz > 1.0) return qz / (tth * ch * ch);
    return 1.0 + (1. - qz) * (1. - 2. * z);
}
inline double amh(double y, int ih) { return ih == 0 ? 1.0 : 1. + 10.0 * std::exp(-5 * y * y); }
inline double bmh(double y, int ih) { return ih == 0 ? 1.0 : 1.0 + 10.0 * std::exp(-5 * y * y); }
inline double bmhy(double y, int ih) { return ih == 0 ? 0.0 : -10. * 10.0 * y * std::exp(-5 * y * y); }
inline double wfun(double yy)
{
    return 0.2 - 0.8 * std::sin(6 * std::fabs(yy)) - 0.5 * (1 - std::tanh(10 * std::fabs(yy))) -
           0.5 * (1 - std::tanh(10 * (pi_ / 2 - std::fabs(yy))));
}

struct Setup {
    iemic_grid cfg;
    /* m_mix flags (mix_imp.f vmix_init 58-109): Mixing 1 mixes T and S from the start;
     * Mixing 2 decides at the first evaluation (vmix_control, 131-166) */
    int vmix_t = 0, vmix_s = 0, vmix_fix = 1;
    void vmix_init()
    {
        vmix_t = vmix_s = cfg.vmix == 1;
        vmix_fix = cfg.vmix != 2;
    }
    /* MIXP = MKAP = 0 and ALPC = 1 (usrc.F90:1169-1176 defaults): only the implicit
     * vertical mixing term of vmix_fun is restated */
    bool vmix_supported() const
    {
        return par[P_MIXP] == 0.0 && par[P_MKAP] == 0.0 &&
               (1.0 - par[P_ALPC]) * par[P_ENER] * par[P_PE_V] == 0.0;
    }
    int n = 0, m = 0, l = 0;
    double xmin = 0, xmax = 0, ymin = 0, ymax = 0, dx = 0, dy = 0, dz = 0;
    std::vector<double> y, yv, dfzT, dfzW;
    std::vector<int> landm;          /* local mask after init_ border handling */
    std::vector<double> tab;         /* Geo table block (see geo())            */
    double par[31] = {0};
    double qtnd = 0, qsnd = 0;
    /* coupled atmosphere (m_atm): Ooa, Os from atmos_coef (usrc.F90:1183-1223); the
     * CommPars-derived values from set_atmos_parameters (usrc.F90:237-293), zero before */
    double Ooa = 0, Os = 0, lvsc = 0, eta_a = 0, qdim_a = 0, dqso = 0, eo0 = 0, albe0 = 0,
           albed = 0, nus = 0;
    /* set_atmos_parameters: pars = AtmosLocal::CommPars (tdim, qdim, nuq, eta, dqso, dqsi,
     * dqdt, Eo0, Ei0, Cs, t0o, t0i, a0, da, tauf, tauc, comb, albf) */
    void set_atmos(const double* pars)
    {
        qdim_a = pars[1];
        eta_a = pars[3];
        dqso = pars[4];
        eo0 = pars[7];
        albe0 = pars[12];
        albed = pars[13];
        nus = par[P_COMB] * par[P_SALT] * eta_a * qdim_a * qsnd;
        lvsc = par[P_COMB] * par[P_TEMP] * rhodim * lv_atm * qtnd;
    }
    /* lin's latent-heat coefficient dedt = lvsc eta qdim (deltat/qdim) dqso (usrc.F90:726) */
    double dedt() const { return lvsc * eta_a * qdim_a * (1.0 / qdim_a) * dqso; }
    int rowintcon_ref = -1;          /* reference (global) row of the integral condition */
    int64_t rowintcon = -1;          /* its ext row when this band owns it, else -1       */
    /* owned subdomain [ib0, ib1) x [jb0, jb1) of the Decomp2D process grid, full depth;
     * hx = HALO x-halo columns when the x direction is split (stencil.h ext layout) */
    int jb0 = 0, jb1 = 0, ib0 = 0, ib1 = 0, nx = 0, hx = 0;
    int64_t xb = 0;                  /* first x-halo cell                                 */
    int64_t nloc = 0, next = 0;      /* owned cells, cells of an ext vector               */

    /* ---- layout helpers (see the ext layout in stencil.h) ------------------------- */
    /* ext cell of 0-based global (i, j, k), j within the halo rows, i within the x halo
     * (after the global wrap) */
    int64_t ext_cell(int i, int j, int k) const
    {
        const int64_t r = ((int64_t)j - jb0 + HALO) * l + k;
        return xcell(r, xlocal(i, n, ib0, nx, hx, hx ? cfg.periodic : 0), nx, hx, xb);
    }
    int64_t ref_cell(int i, int j, int k) const { return ((int64_t)k * m + j) * n + i; }
    int64_t own0() const { return (int64_t)HALO * l * nx; }       /* first owned ext cell  */
    /* owned-local index lc -> 0-based (i, j, k) */
    void owned_ijk(int64_t lc, int& i, int& j, int& k) const
    {
        i = ib0 + (int)(lc % nx);
        k = (int)((lc / nx) % l);
        j = jb0 + (int)(lc / ((int64_t)nx * l));
    }
    /* ext cell -> 0-based global (i, j, k) (i wrapped into the grid) */
    void ext_ijk(int64_t ec, int& i, int& j, int& k) const
    {
        int64_t r;
        int il;
        if (ec < xb) {
            r = ec / nx;
            il = (int)(ec % nx);
        } else {
            r = (ec - xb) / (2 * hx);
            const int h = (int)((ec - xb) % (2 * hx));
            il = h < hx ? h - hx : nx + h - hx;
        }
        k = (int)(r % l);
        j = jb0 - HALO + (int)(r / l);
        i = ib0 + il;
        if (i < 0) i += n;
        if (i >= n) i -= n;
    }
    int64_t ext_to_ref_row(int64_t er) const
    {
        int i, j, k;
        ext_ijk(er / NUN, i, j, k);
        return NUN * ref_cell(i, j, k) + er % NUN;
    }
    bool owns(int i, int j) const { return j >= jb0 && j < jb1 && i >= ib0 && i < ib1; }

    /* sub0/sub1: owned columns [sub0[0], sub1[0]) and rows [sub0[1], sub1[1]); xsplit: the x
     * direction is split over several ranks (x halo in the layout) */
    void init(const iemic_grid& g, const int* landm_in, const int* sub0 = nullptr, const int* sub1 = nullptr,
              int xsplit = 0)
    {
        cfg = g;
        n = g.n; m = g.m; l = g.l;
        ib0 = sub0 ? sub0[0] : 0;
        ib1 = sub1 ? sub1[0] : n;
        jb0 = sub0 ? sub0[1] : 0;
        jb1 = sub1 ? sub1[1] : m;
        nx = ib1 - ib0;
        hx = xsplit ? HALO : 0;
        nloc = (int64_t)nx * l * (jb1 - jb0);
        xb = (int64_t)nx * l * (jb1 - jb0 + 2 * HALO);
        next = xb + (int64_t)2 * hx * l * (jb1 - jb0 + 2 * HALO);
        xmin = g.xmin * pi_ / 180.0;
        xmax = g.xmax * pi_ / 180.0;
        ymin = g.ymin * pi_ / 180.0;
        ymax = g.ymax * pi_ / 180.0;
        const size_t nl = (size_t)(n + 2) * (m + 2) * (l + 2);
        landm.assign(landm_in, landm_in + nl);
        for (int k = 0; k <= l + 1; k++)
            for (int j = 0; j <= m + 1; j++)
                for (int i = 0; i <= n + 1; i++) {
                    int& v = landm[((size_t)k * (m + 2) + j) * (n + 2) + i];
                    if (!g.periodic && v == 3) v = OCEAN;
                    if (!g.periodic && (i == 0 || i == n + 1)) v = LAND;
                    if (j == 0 || j == m + 1 || k == 0 || k == l + 1) v = LAND;
                }
        rowintcon = -1;
        rowintcon_ref = -1;
        if (g.sres == 0) {
            int Nic = g.int_i == -1 ? n - 1 : g.int_i;
            int Mic = g.int_j == -1 ? m - 1 : g.int_j;
            rowintcon_ref = (int)(NUN * ref_cell(Nic, Mic, l - 1) + SS);
            if (owns(Nic, Mic)) rowintcon = NUN * ext_cell(Nic, Mic, l - 1) + SS;
        }
        grid();
        stpnt();
    }

    void grid()
    {
        const int M2 = m + 2;
        dx = (xmax - xmin) / n;
        dy = (ymax - ymin) / m;
        dz = (zmax - zmin) / l;
        y.assign(M2, 0.0);
        yv.assign(M2, 0.0);
        for (int j = 1; j <= m; j++) {
            y[j] = ((double)j - 0.5) * dy + ymin;
            yv[j] = ((double)j) * dy + ymin;
        }
        y[0] = y[1] - dy;
        y[m + 1] = y[m] + dy;
        yv[0] = ymin;
        dfzT.assign(l + 2, 0.0);
        dfzW.assign(l + 2, 0.0);
        for (int k = 1; k <= l; k++) {
            double ze = ((double)k - 0.5) * dz + zmin;
            double zwe = ((double)k) * dz + zmin;
            dfzT[k] = dfdz(ze, cfg.qz);
            dfzW[k] = dfdz(zwe, cfg.qz);
        }
        dfzW[0] = dfdz(zmin, cfg.qz);
        const int ih = cfg.ih;
        tab.assign((size_t)10 * M2 + 2 * (l + 2), 0.0);
        for (int j = 0; j <= m + 1; j++) {
            tab[j] = std::cos(y[j]);
            tab[4 * M2 + j] = amh(y[j], ih);
            tab[5 * M2 + j] = bmh(y[j], ih);
        }
        for (int j = 0; j <= m; j++) {
            tab[M2 + j] = std::cos(yv[j]);
            tab[2 * M2 + j] = std::tan(yv[j]);
            tab[3 * M2 + j] = std::sin(yv[j]);
            tab[6 * M2 + j] = amh(yv[j], ih);
            tab[7 * M2 + j] = bmh(yv[j], ih);
            tab[8 * M2 + j] = bmhy(yv[j], ih);
        }
        for (int k = 0; k <= l + 1; k++) {
            tab[9 * M2 + k] = dfzT[k];
            tab[9 * M2 + (l + 2) + k] = dfzW[k];
        }
        double dzne = dz * dfzT[l];
        qtnd = r0dim / (udim * cp0 * rhodim * cfg.hdim * dzne);
        qsnd = s0 * r0dim / (deltas * udim * cfg.hdim * dzne);
        /* atmos_coef (usrc.F90:1183-1223) with the m_atm constants (atm.F90:5-19) */
        const double muoa = rhoa_atm * ch_atm * cpa_atm * uw_atm;
        Os = sun0_atm * c0_atm / 4 * qtnd;
        Ooa = muoa * qtnd;
        double* suno = tab.data() + 9 * M2 + 2 * (l + 2);
        for (int j = 1; j <= m; j++) {
            const double sy = std::sin(y[j]);
            suno[j] = Os * (1 - .482 * (3 * (sy * sy) - 1.) / 2.);
        }
    }

    void stpnt()
    {
        const double hdim = cfg.hdim;
        par[P_AL_T] = 0.1 / (2 * omegadim * rhodim * hdim * udim * dz * dfzT[l]);
        par[P_RAYL] = cfg.alpha_t * gdim * hdim / (2 * omegadim * udim * r0dim);
        par[P_EK_V] = av / (2 * omegadim * hdim * hdim);
        par[P_EK_H] = ah / (2 * omegadim * r0dim * r0dim);
        par[P_ROSB] = udim / (2 * omegadim * r0dim);
        par[P_HMTP] = 0.0;
        par[P_SUNP] = 0.0;
        par[P_PE_H] = kappah / (udim * r0dim);
        par[P_PE_V] = kappav * r0dim / (udim * hdim * hdim);
        par[P_P_VC] = 2.5e+04 * par[P_PE_V];
        par[P_LAMB] = cfg.alpha_s / cfg.alpha_t;
        par[P_SALT] = 0.0;
        par[P_WIND] = 0.0;
        par[P_TEMP] = 0.0;
        par[P_BIOT] = r0dim / (75. * 3600. * 24. * udim);
        par[P_COMB] = 0.0;
        par[P_NLES] = 0.0;
        par[P_CMPR] = 0.0;
        par[P_ALPC] = 1.0;
        par[P_ENER] = 1.0e+02;
        par[P_MIXP] = 0.0;
        par[P_MKAP] = 0.0;
        par[P_SPL1] = 2.0e+03;
        par[P_SPL2] = 0.01;
        if (cfg.vmix == 0) {
            par[P_MIXP] = 0.0;
            par[P_P_VC] = 0.0;
            par[P_ALPC] = 1.0;
            par[P_ENER] = 1.0e+2;
            par[P_MKAP] = 0.0;
        }
    }

    /* [wfun(yv) | temfun(y) | salfun(y) | spert(n*m)] for the current par (forcing.F90) */
    std::vector<double> forcing_tables() const
    {
        const int M2 = m + 2;
        std::vector<double> t((size_t)3 * M2 + (size_t)n * m, 0.0);
        for (int j = 0; j <= m; j++) t[j] = wfun(yv[j]);
        for (int j = 0; j <= m + 1; j++) {
            double yy = y[j];
            double tf, sf;
            if (cfg.forcing_type == 2) {
                tf = std::cos(pi_ * (yy - ymin) / (ymax - ymin));
                sf = tf;
            } else {
                tf = std::cos(pi_ * yy / ymax) + par[P_CMPR] * std::sin(pi_ * yy / ymax);
                if (cfg.forcing_type == 1)
                    sf = (std::cos(pi_ * yy / ymax) + par[P_FPER] * yy / ymax) / std::cos(yy);
                else
                    sf = std::cos(pi_ * yy / ymax) + par[P_FPER] * yy / ymax;
            }
            t[M2 + j] = tf;
            t[2 * M2 + j] = sf;
        }
        /* spert = real(SRES) (global.F90:590-611, no perturbation mask) */
        for (int q = 0; q < n * m; q++) t[3 * M2 + q] = (double)cfg.sres;
        return t;
    }

    /* integral-condition coefficient of the S unknown of (i,j,k), 0-based (thcm_utils.F90:285-312) */
    double intcond_at(int i, int j, int k) const
    {
        return landm[((size_t)(k + 1) * (m + 2) + (j + 1)) * (n + 2) + (i + 1)] == OCEAN
                   ? std::cos(y[j + 1]) * dfzT[k + 1] : 0.0;
    }
    /* coefficients in the ext layout (owned S rows), for the device */
    std::vector<double> intcond_coeff() const
    {
        std::vector<double> ic((size_t)NUN * next, 0.0);
        for (int64_t lc = 0; lc < nloc; lc++) {
            int i, j, k;
            owned_ijk(lc, i, j, k);
            ic[(size_t)NUN * ext_cell(i, j, k) + SS] = intcond_at(i, j, k);
        }
        return ic;
    }

    /* Owned rows of the maximal graph (THCM::CreateMaximalGraph, THCM.C:2288-2491) in the
     * reference's numbering: columns sorted as Epetra stores them, plus the stencil slot
     * feeding each (several slots can name one column on tiny periodic grids; `first` is
     * the column position they add into).  The intcond row (SRES = 0) is dense over all S
     * unknowns (THCM.C:2475-2486); its slots are -1. */
    void graph_row(int i, int j, int k, int var, std::vector<int64_t>& cols,
                   std::vector<std::pair<int, int>>& slot) const
    {
        cols.clear();
        slot.clear();
        if (NUN * ref_cell(i, j, k) + var == rowintcon_ref) {
            for (int64_t q = 0; q < (int64_t)n * m * l; q++) cols.push_back(NUN * q + SS);
            return;
        }
        Geo g = geo(nullptr, tab.data());
        std::vector<std::pair<int64_t, int>> e;
        for (int s = ROW_BEGIN[var]; s < ROW_BEGIN[var + 1]; s++) {
            int64_t col = slot_col(g, s, i + 1, j + 1, k + 1);
            if (col >= 0) e.push_back({ext_to_ref_row(col), s});
        }
        std::sort(e.begin(), e.end());
        for (size_t a = 0; a < e.size(); a++) {
            if (a == 0 || e[a].first != e[a - 1].first) cols.push_back(e[a].first);
            slot.push_back({(int)cols.size() - 1, e[a].second});
        }
    }

    /* Epetra-identical CSR of the owned rows (reference order: k-major) from slot-major
     * values v[s*nloc + lc]; the dense intcond row gets intSign*coefficient.  rowptr/col/val
     * may be null (count). */
    int64_t to_csr(const double* v, int64_t* rowptr, int* col, double* val) const
    {
        std::vector<int64_t> cols;
        std::vector<std::pair<int, int>> slot;
        int64_t pos = 0, r = 0;
        for (int k = 0; k < l; k++)
            for (int j = jb0; j < jb1; j++)
                for (int i = ib0; i < ib1; i++)
                    for (int var = 0; var < NUN; var++, r++) {
                        if (rowptr) rowptr[r] = pos;
                        graph_row(i, j, k, var, cols, slot);
                        if (col)
                            for (size_t a = 0; a < cols.size(); a++) col[pos + a] = (int)cols[a];
                        if (val) {
                            const int64_t lc = (((int64_t)j - jb0) * l + k) * nx + (i - ib0);
                            if (NUN * ref_cell(i, j, k) + var == rowintcon_ref)
                                for (size_t a = 0; a < cols.size(); a++) {
                                    const int64_t q = cols[a] / NUN;
                                    val[pos + a] = cfg.int_sign *
                                                   intcond_at((int)(q % n), (int)((q / n) % m), (int)(q / ((int64_t)n * m)));
                                }
                            else {
                                for (size_t a = 0; a < cols.size(); a++) val[pos + a] = 0.0;
                                for (auto& ps : slot) val[pos + ps.first] += v[(size_t)ps.second * nloc + lc];
                            }
                        }
                        pos += (int64_t)cols.size();
                    }
        if (rowptr) rowptr[r] = pos;
        return pos;
    }

    /* reference-ordered global vector <-> ext-layout local vector (owned rows only) */
    void ref_to_ext(const double* ref, double* ext) const
    {
        for (int64_t lc = 0; lc < nloc; lc++) {
            int i, j, k;
            owned_ijk(lc, i, j, k);
            const int64_t e = NUN * ext_cell(i, j, k), r = NUN * ref_cell(i, j, k);
            for (int v = 0; v < NUN; v++) ext[e + v] = ref[r + v];
        }
    }
    void ext_to_ref(const double* ext, double* ref) const
    {
        for (int64_t lc = 0; lc < nloc; lc++) {
            int i, j, k;
            owned_ijk(lc, i, j, k);
            const int64_t e = NUN * ext_cell(i, j, k), r = NUN * ref_cell(i, j, k);
            for (int v = 0; v < NUN; v++) ref[r + v] = ext[e + v];
        }
    }

    /* Geo over externally owned copies of landm / tab */
    Geo geo(const int* landm_p, const double* tab_p, const double* atm_p = nullptr) const
    {
        Geo g{};
        g.n = n; g.m = m; g.l = l;
        g.jb0 = jb0;
        g.ib0 = ib0;
        g.nx = nx;
        g.hx = hx;
        g.xb = xb;
        g.periodic = cfg.periodic;
        g.tres = cfg.tres; g.sres = cfg.sres; g.coriolis_on = cfg.coriolis_on;
        g.dx = dx; g.dy = dy; g.dz = dz;
        g.landm = landm_p;
        const int M2 = m + 2;
        g.cos_y = tab_p;
        g.cos_yv = tab_p + M2;
        g.tan_yv = tab_p + 2 * M2;
        g.sin_yv = tab_p + 3 * M2;
        g.amh_y = tab_p + 4 * M2;
        g.bmh_y = tab_p + 5 * M2;
        g.amh_yv = tab_p + 6 * M2;
        g.bmh_yv = tab_p + 7 * M2;
        g.bmhy_yv = tab_p + 8 * M2;
        g.dfzT = tab_p + 9 * M2;
        g.dfzW = tab_p + 9 * M2 + (l + 2);
        for (int i = 0; i < 31; i++) g.par[i] = par[i];
        g.vmix_t = cfg.vmix != 0 && vmix_t;
        g.vmix_s = cfg.vmix != 0 && vmix_s;
        g.rho_mixing = cfg.rho_mixing;
        g.alphaT = cfg.alpha_t;
        g.coupled_t = cfg.coupled_t;
        g.coupled_s = cfg.coupled_s;
        g.dedt_s = qdim_a != 0.0 ? nus * (1.0 / qdim_a) * dqso : 0.0;
        g.qsnd = qsnd;
        g.Ooa = Ooa;
        g.dedt = qdim_a != 0.0 ? dedt() : 0.0;
        g.lvsc = lvsc;
        g.eta_a = eta_a;
        g.qdim_a = qdim_a;
        g.eo0 = eo0;
        g.albe0 = albe0;
        g.albed = albed;
        g.suno = tab_p + 9 * M2 + 2 * (l + 2);
        g.atm = atm_p;
        return g;
    }
};

}  // namespace host
}  // namespace iemic
#endif
