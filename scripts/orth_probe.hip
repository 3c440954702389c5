/* DCGS2 basis-pass probe at the 2-degree vector length: the library's dot / update passes
 * (krylov.hip k_dcgs_dot, k_dcgs_update) against variants with 16-byte loads (two
 * elements per lane), the vector group fastest in the block order (u, w re-read from L2)
 * and deeper unrolling of the update.  Prints the achieved GB/s of the algorithmic bytes:
 * (nv + 2) vectors read for the dot, nv + 2 read + 2 written for the update. */
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int NV>
__device__ __forceinline__ void bsum(double* v, double* sm)
{
#pragma unroll
    for (int q = 0; q < NV; q++)
        for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_down(v[q], o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) sm[q * nw + wid] = v[q];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int q = 0; q < NV; q++) {
            double t = 0.0;
            for (int w = 0; w < nw; w++) t += sm[q * nw + w];
            v[q] = t;
        }
}

/* the library's dot pass (2-D grid, 8-byte loads) */
__global__ void __launch_bounds__(256) k_dot_ref(const double* __restrict__ V, long ldv, int nvec,
                                                 const double* __restrict__ u, const double* __restrict__ w,
                                                 long N, double* __restrict__ partial)
{
    constexpr int DG = 8;
    __shared__ double sm[8 * 2 * DG];
    const int nq = (nvec + DG - 1) / DG;
    const int by = blockIdx.y;
    const long stride = (long)gridDim.x * blockDim.x;
    const long e0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (by < nq) {
        const int i0 = DG * by;
        const int nv = min(DG, nvec - i0);
        double acc[2 * DG];
#pragma unroll
        for (int t = 0; t < 2 * DG; t++) acc[t] = 0.0;
        const double* q0 = V + (long)i0 * ldv;
        for (long e = e0; e < N; e += stride) {
            const double ue = u[e], we = w[e];
#pragma unroll
            for (int t = 0; t < DG; t++) {
                if (t < nv) {
                    const double qe = q0[(long)t * ldv + e];
                    acc[2 * t] += qe * ue;
                    acc[2 * t + 1] += qe * we;
                }
            }
        }
        bsum<2 * DG>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 2 * nv; t++) partial[(long)(2 * i0 + t) * gridDim.x + blockIdx.x] = acc[t];
    } else {
        double acc[3] = {0, 0, 0};
        for (long e = e0; e < N; e += stride) {
            const double ue = u[e], we = w[e];
            acc[0] += ue * ue;
            acc[1] += ue * we;
            acc[2] += we * we;
        }
        bsum<3>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 3; t++) partial[(long)(2 * nvec + t) * gridDim.x + blockIdx.x] = acc[t];
    }
}

/* 16-byte loads; YF: 1-D grid with the group index fastest */
template <int DG, bool YF>
__global__ void __launch_bounds__(256) k_dot2(const double* __restrict__ V, long ldv, int nvec,
                                              const double* __restrict__ u, const double* __restrict__ w,
                                              long N, double* __restrict__ partial, int nbx)
{
    __shared__ double sm[4 * 2 * DG];
    const int nq = (nvec + DG - 1) / DG;
    int by, bx;
    if (YF) { by = blockIdx.x % (nq + 1); bx = blockIdx.x / (nq + 1); }
    else { by = blockIdx.y; bx = blockIdx.x; }
    const long N2 = N / 2;
    const long stride = (long)nbx * blockDim.x;
    const long e0 = (long)bx * blockDim.x + threadIdx.x;
    const double2* u2 = reinterpret_cast<const double2*>(u);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    if (by < nq) {
        const int i0 = DG * by;
        const int nv = min(DG, nvec - i0);
        double acc[2 * DG];
#pragma unroll
        for (int t = 0; t < 2 * DG; t++) acc[t] = 0.0;
        const double* q0 = V + (long)i0 * ldv;
        for (long e = e0; e < N2; e += stride) {
            const double2 ue = u2[e], we = w2[e];
#pragma unroll
            for (int t = 0; t < DG; t++) {
                if (t < nv) {
                    const double2 qe = reinterpret_cast<const double2*>(q0 + (long)t * ldv)[e];
                    acc[2 * t] += qe.x * ue.x + qe.y * ue.y;
                    acc[2 * t + 1] += qe.x * we.x + qe.y * we.y;
                }
            }
        }
        bsum<2 * DG>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 2 * nv; t++) partial[(long)(2 * i0 + t) * nbx + bx] = acc[t];
    } else {
        double acc[3] = {0, 0, 0};
        for (long e = e0; e < N2; e += stride) {
            const double2 ue = u2[e], we = w2[e];
            acc[0] += ue.x * ue.x + ue.y * ue.y;
            acc[1] += ue.x * we.x + ue.y * we.y;
            acc[2] += we.x * we.x + we.y * we.y;
        }
        bsum<3>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 3; t++) partial[(long)(2 * nvec + t) * nbx + bx] = acc[t];
    }
}

/* the library's update pass */
__global__ void __launch_bounds__(256) k_upd_ref(const double* __restrict__ V, long ldv, int nvec,
                                                 const double* __restrict__ coef, double ib, double gamma,
                                                 double* __restrict__ u, double* __restrict__ w, long N)
{
    __shared__ double cs[2 * 1024];
    for (int i = threadIdx.x; i < 2 * nvec; i += blockDim.x) cs[i] = coef[i];
    __syncthreads();
    const double* a = cs;
    const double* cc = cs + nvec;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (long)gridDim.x * blockDim.x) {
        double su = 0.0, sw = 0.0;
        int i = 0;
        for (; i + 2 <= nvec; i += 2) {
            const double q0 = V[(long)i * ldv + e], q1 = V[(long)(i + 1) * ldv + e];
            su += a[i] * q0 + a[i + 1] * q1;
            sw += cc[i] * q0 + cc[i + 1] * q1;
        }
        for (; i < nvec; i++) {
            const double q0 = V[(long)i * ldv + e];
            su += a[i] * q0;
            sw += cc[i] * q0;
        }
        const double ue = u[e];
        u[e] = (ue - su) * ib;
        w[e] = (w[e] - sw - gamma * ue) * ib;
    }
}

/* 16-byte loads, UN basis vectors per inner step */
template <int UN>
__global__ void __launch_bounds__(256) k_upd2(const double* __restrict__ V, long ldv, int nvec,
                                              const double* __restrict__ coef, double ib, double gamma,
                                              double* __restrict__ u, double* __restrict__ w, long N)
{
    __shared__ double cs[2 * 1024];
    for (int i = threadIdx.x; i < 2 * nvec; i += blockDim.x) cs[i] = coef[i];
    __syncthreads();
    const double* a = cs;
    const double* cc = cs + nvec;
    const long N2 = N / 2;
    double2* u2 = reinterpret_cast<double2*>(u);
    double2* w2 = reinterpret_cast<double2*>(w);
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < N2; e += (long)gridDim.x * blockDim.x) {
        double sux = 0.0, suy = 0.0, swx = 0.0, swy = 0.0;
        int i = 0;
        for (; i + UN <= nvec; i += UN) {
            double2 q[UN];
#pragma unroll
            for (int k = 0; k < UN; k++) q[k] = reinterpret_cast<const double2*>(V + (long)(i + k) * ldv)[e];
#pragma unroll
            for (int k = 0; k < UN; k++) {
                sux += a[i + k] * q[k].x;
                suy += a[i + k] * q[k].y;
                swx += cc[i + k] * q[k].x;
                swy += cc[i + k] * q[k].y;
            }
        }
        for (; i < nvec; i++) {
            const double2 q = reinterpret_cast<const double2*>(V + (long)i * ldv)[e];
            sux += a[i] * q.x;
            suy += a[i] * q.y;
            swx += cc[i] * q.x;
            swy += cc[i] * q.y;
        }
        const double2 ue = u2[e], we = w2[e];
        u2[e] = make_double2((ue.x - sux) * ib, (ue.y - suy) * ib);
        w2[e] = make_double2((we.x - swx - gamma * ue.x) * ib, (we.y - swy - gamma * ue.y) * ib);
    }
}

int main(int argc, char** argv)
{
    const long N = argc > 1 ? atol(argv[1]) : 1400832;   /* even */
    const int MAXV = 92, REPS = 40;
    double *V, *u, *w, *part, *coef;
    CK(hipMalloc(&V, sizeof(double) * (N + 8448) * MAXV));
    CK(hipMalloc(&u, sizeof(double) * N));
    CK(hipMalloc(&w, sizeof(double) * N));
    CK(hipMalloc(&part, sizeof(double) * 4096 * (2 * MAXV + 4)));
    CK(hipMalloc(&coef, sizeof(double) * 2 * MAXV));
    std::vector<double> h(N);
    for (long i = 0; i < N; i++) h[i] = 1e-3 * (double)((i * 7919) % 1000);
    for (int v = 0; v < MAXV; v++) CK(hipMemcpy(V + (long)v * (N + 8448), h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(u, h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
    CK(hipMemset(coef, 0, sizeof(double) * 2 * MAXV));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, int nv, double vecs, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < REPS; r++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / REPS;
        printf("%-24s nv=%2d  %8.2f us  %7.1f GB/s\n", name, nv, us, vecs * 8.0 * N / (us * 1e3));
    };
    /* basis stride: the library's (N rounded by the ext layout) and padded variants, which
     * stagger the vectors' streams over the memory channels */
    for (long pad : {0L, 256L, 1280L, 8448L}) {
        const long ldv = N + pad;
        for (int nv : {45, 89}) {
            const double vd = nv + 2, vu = nv + 4;
            const int nq8 = (nv + 7) / 8, nq4 = (nv + 3) / 4;
            char nm[64];
            snprintf(nm, sizeof nm, "dot ref pad%ld", pad);
            run(nm, nv, vd, [&] { k_dot_ref<<<dim3(1024, nq8 + 1), 256>>>(V, ldv, nv, u, w, N, part); });
            snprintf(nm, sizeof nm, "dot2 DG4 yf pad%ld", pad);
            run(nm, nv, vd, [&] { k_dot2<4, true><<<dim3(1024 * (nq4 + 1)), 256>>>(V, ldv, nv, u, w, N, part, 1024); });
            snprintf(nm, sizeof nm, "dot2 DG8 2D pad%ld", pad);
            run(nm, nv, vd, [&] { k_dot2<8, false><<<dim3(1024, nq8 + 1), 256>>>(V, ldv, nv, u, w, N, part, 1024); });
            const unsigned G = (unsigned)std::min<long>((N + 255) / 256, 4096);
            snprintf(nm, sizeof nm, "upd ref pad%ld", pad);
            run(nm, nv, vu, [&] { k_upd_ref<<<G, 256>>>(V, ldv, nv, coef, 1.0, 0.0, u, w, N); });
            snprintf(nm, sizeof nm, "upd2 UN4 g1024 pad%ld", pad);
            run(nm, nv, vu, [&] { k_upd2<4><<<1024, 256>>>(V, ldv, nv, coef, 1.0, 0.0, u, w, N); });
        }
    }
    return 0;
}
