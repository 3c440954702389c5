// ocean_driver.cpp -- C++ host check of i-emic_amd/csrc/ocean.hpp (the Ocean-shaped class
// a C++ i-emic build links).  Reads a problem file written by tests/test_cpp_host.py:
//   int32 n,m,l,periodic,tres,sres,forcing_type,ih,coriolis,int_sign,npar
//   float64 xmin,xmax,ymin,ymax,hdim,qz,alpha_t,alpha_s
//   npar x (int32 idx, float64 value); int32 landm[(n+2)(m+2)(l+2)]; float64 x[N]
// and writes F, the solution of J s = -F and a line of norms to <out>.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../i-emic_amd/csrc/ocean.hpp"

template <typename T> static void rd(FILE* f, T* p, size_t n)
{
    if (fread(p, sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
}

int main(int argc, char** argv)
{
    if (argc < 3) { fprintf(stderr, "usage: ocean_driver <in> <out>\n"); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int hdr[11];
    rd(f, hdr, 11);
    double dv[8];
    rd(f, dv, 8);
    iemic_grid g{};
    g.n = hdr[0]; g.m = hdr[1]; g.l = hdr[2]; g.periodic = hdr[3]; g.tres = hdr[4];
    g.sres = hdr[5]; g.forcing_type = hdr[6]; g.ih = hdr[7]; g.coriolis_on = hdr[8];
    g.int_sign = hdr[9];
    g.xmin = dv[0]; g.xmax = dv[1]; g.ymin = dv[2]; g.ymax = dv[3]; g.hdim = dv[4]; g.qz = dv[5];
    g.alpha_t = dv[6]; g.alpha_s = dv[7];
    g.vmix = 0; g.int_i = -1; g.int_j = -1; g.analyze_jacobian = 1; g.max_mask_fixes = 5;
    g.device = 0;
    const int npar = hdr[10];
    std::vector<std::pair<int, double>> pars(npar);
    for (int q = 0; q < npar; q++) {
        rd(f, &pars[q].first, 1);
        rd(f, &pars[q].second, 1);
    }
    const size_t nl = (size_t)(g.n + 2) * (g.m + 2) * (g.l + 2);
    std::vector<int> landm(nl);
    rd(f, landm.data(), nl);
    const size_t N = (size_t)6 * g.n * g.m * g.l;
    iemic::Vector x(N);
    rd(f, x.data(), N);
    fclose(f);
    try {
        iemic::Ocean ocean(g, landm);
        for (auto& p : pars) iemic::check(iemic_set_par(ocean.handle(), p.first, p.second), "set_par");
        ocean.setState(x);
        ocean.computeRHS();
        ocean.computeJacobian();
        iemic::Vector b(*ocean.getRHS('C'));
        b.Scale(-1.0);
        ocean.solve(b);
        auto s = ocean.getSolution('V');
        iemic::Vector r(N);
        ocean.applyMatrix(*s, r);
        r.Update(1.0, b, -1.0);   // r = b - J s
        FILE* o = fopen(argv[2], "wb");
        fwrite(ocean.getRHS('V')->data(), sizeof(double), N, o);
        fwrite(s->data(), sizeof(double), N, o);
        fclose(o);
        printf("normF %.17g iters %d relres %.3e combined %.17g\n", ocean.getRHS('V')->Norm2(),
               ocean.lastSolve().iters, r.Norm2() / b.Norm2(), ocean.getPar("Combined Forcing"));
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
