/*
 * decomp.h -- the TRIOS Decomp2D domain decomposition (TRIOS_Domain.C:81-195) and the halo
 * exchange plans of the ext layout (stencil.h).  Pure C++: shared by the device library
 * (capi.hip, comm.hip) and its CPU test harness (tests/emul), so the multi-process CPU
 * tests run the library's own partition, neighbour and message-pairing rules.
 */
#ifndef IEMIC_DECOMP_H
#define IEMIC_DECOMP_H

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "stencil.h"

namespace iemic {

/* TRIOS::Domain::Decomp2D (TRIOS_Domain.C:88-109), the same integer arithmetic: npy = the
 * largest t1 dividing P with the smallest |m/t1 - n/(P/t1)| (ties to the smaller t1) */
inline void decomp2d(int n, int m, int P, int& npx, int& npy)
{
    int npM = P, npN = 1;
    double r_min = 100;
    for (int t1 = P; t1 > 0; t1--) {
        const int t2 = P / t1;
        const double r = std::abs(m / t1 - n / t2);
        if (t1 * t2 == P && r <= r_min) {
            r_min = r;
            npM = t1;
            npN = t2;
        }
    }
    npx = npN;
    npy = npM;
}

/* the reference's split of N points over np parts: the first N % np parts take one more
 * (TRIOS_Domain.C:151-162) */
inline void part_of(int N, int np, int p, int& off, int& cnt)
{
    off = p * (N / np) + std::min(p, N % np);
    cnt = N / np + (p < N % np ? 1 : 0);
}

/* one rank's subdomain: process grid npx x npy, rank = py * npx + px, owned columns
 * [ib0, ib1) and rows [jb0, jb1), x-halo width hx (HALO when npx > 1), neighbours
 * nb[W, E, S, N] (-1: none; W/E wrap on a periodic grid) */
struct Sub {
    int rank = 0, nranks = 1, npx = 1, npy = 1, px = 0, py = 0;
    int ib0 = 0, ib1 = 0, jb0 = 0, jb1 = 0, nx = 0, mb = 0, hx = 0, l = 0;
    int64_t xb = 0;                   /* first x-halo cell of an ext vector           */
    int nb[4] = {-1, -1, -1, -1};
};

/* 0, or a message for a decomposition the layout cannot hold */
inline const char* sub_init(Sub& d, int n, int m, int l, int periodic, int rank, int nranks, int npx)
{
    if (nranks < 1 || rank < 0 || rank >= nranks) return "bad rank / nranks";
    if (npx < 0 || npx > nranks) return "npx must be 0 (Decomp2D rule) or a divisor of nranks";
    int npy = 1;
    if (npx <= 0) decomp2d(n, m, nranks, npx, npy);
    if (npx < 1 || nranks % npx) return "npx must divide nranks";
    npy = nranks / npx;
    /* every subdomain covers the halo depth; a periodic x halo never wraps onto itself */
    if (m / npy < HALO || (npx > 1 && n / npx < HALO) ||
        (npx > 1 && periodic && n < (n + npx - 1) / npx + 2 * HALO))
        return "too many ranks for the grid (subdomains need >= 2 rows and columns)";
    d.rank = rank;
    d.nranks = nranks;
    d.npx = npx;
    d.npy = npy;
    d.px = rank % npx;
    d.py = rank / npx;
    part_of(n, npx, d.px, d.ib0, d.nx);
    part_of(m, npy, d.py, d.jb0, d.mb);
    d.ib1 = d.ib0 + d.nx;
    d.jb1 = d.jb0 + d.mb;
    d.l = l;
    d.hx = npx > 1 ? HALO : 0;
    d.xb = (int64_t)d.nx * l * (d.mb + 2 * HALO);
    const bool wrap = periodic && npx > 1;
    d.nb[0] = d.px > 0 ? rank - 1 : (wrap ? rank + npx - 1 : -1);
    d.nb[1] = d.px < npx - 1 ? rank + 1 : (wrap ? rank - (npx - 1) : -1);
    d.nb[2] = d.py > 0 ? rank - npx : -1;
    d.nb[3] = d.py < npy - 1 ? rank + npx : -1;
    return nullptr;
}

/* one message: nblk blocks of len doubles, stride doubles apart, from offset off */
struct SegD {
    int64_t off, nblk, len, stride;
};
struct MsgD {
    int send;
    int peer;
    SegD s;
};

/* Exchange plan of arrays in the ext layout (width doubles per cell), depth rows / columns.
 * Phase x over the owned rows (main-block runs of the edge columns <-> x-halo runs), phase
 * y over whole latitude rows (a slab of the main block and one of the x halo, so the y
 * messages carry the x halo and the diagonal neighbours arrive too).  Pairing rule: the
 * k-th message rank a sends to rank b is the k-th message b receives from a; every
 * direction is posted as "send my edge to nb[d], receive my opposite halo from
 * nb[opposite d]" in the order W, E, S, N, so with npx = 2 on a periodic grid, where W and
 * E are the same rank, the two messages still pair up. */
inline void plan_ext(const Sub& d, int width, int depth, std::vector<MsgD>& x, std::vector<MsgD>& y)
{
    const int64_t w = width, l = d.l, nx = d.nx, hx = d.hx, mb = d.mb;
    const int64_t dx = std::min<int64_t>(depth, hx), dy = std::min<int64_t>(depth, HALO);
    const int W = d.nb[0], E = d.nb[1], S = d.nb[2], N = d.nb[3];
    if (hx > 0 && dx > 0) {
        const int64_t r0 = (int64_t)HALO * l, nr = mb * l;        /* owned rows of the main block */
        const int64_t xr = d.xb + r0 * 2 * hx;                      /* their x-halo runs            */
        auto main = [&](int64_t col) { return SegD{(r0 * nx + col) * w, nr, dx * w, nx * w}; };
        auto halo = [&](int64_t h) { return SegD{(xr + h) * w, nr, dx * w, 2 * hx * w}; };
        if (W >= 0) x.push_back({1, W, main(0)});                    /* to W: my first columns   */
        if (E >= 0) x.push_back({0, E, halo(hx)});                   /* from E: right halo       */
        if (E >= 0) x.push_back({1, E, main(nx - dx)});              /* to E: my last columns    */
        if (W >= 0) x.push_back({0, W, halo(hx - dx)});              /* from W: left halo        */
    }
    if (dy > 0) {
        const int64_t rows = dy * l;
        auto slab = [&](int64_t jl, bool xh) {                       /* rows of latitudes jl..   */
            const int64_t r = (jl + HALO) * l;
            return xh ? SegD{(d.xb + r * 2 * hx) * w, 1, rows * 2 * hx * w, rows * 2 * hx * w}
                      : SegD{r * nx * w, 1, rows * nx * w, rows * nx * w};
        };
        for (int xh = 0; xh < (hx > 0 ? 2 : 1); xh++) {
            if (S >= 0) y.push_back({1, S, slab(0, xh)});
            if (N >= 0) y.push_back({0, N, slab(mb, xh)});
            if (N >= 0) y.push_back({1, N, slab(mb - dy, xh)});
            if (S >= 0) y.push_back({0, S, slab(-dy, xh)});
        }
    }
}

}  // namespace iemic
#endif
