/* Microbenchmark of the DCGS2 basis passes (dot: Q^T[u w] + self products; update:
 * u -= Q a, w -= Q c) at the 2-degree global ocean's vector length, for block-order and
 * group-size variants of the dot pass.  Prints achieved GB/s of the algorithmic bytes
 * ((nv + 2) vectors read for the dot, nv + 2 read + 2 written for the update).
 * build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_orth tools/mb_orth.hip */
#include <hip/hip_runtime.h>
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

/* YFAST: 1-D grid, the group index varies fastest (the groups of one chunk run together, so
 * u and w are re-read from L2) */
template <int DG, bool YFAST>
__global__ void __launch_bounds__(256) k_dot(const double* __restrict__ V, long ldv, int nvec,
                                             const double* __restrict__ u, const double* __restrict__ w,
                                             long N, double* __restrict__ partial, int nbx)
{
    __shared__ double sm[4 * 2 * DG];
    const int nq = (nvec + DG - 1) / DG;
    int by, bx;
    if (YFAST) { by = blockIdx.x % (nq + 1); bx = blockIdx.x / (nq + 1); }
    else { by = blockIdx.y; bx = blockIdx.x; }
    const long stride = (long)nbx * blockDim.x;
    const long e0 = (long)bx * blockDim.x + threadIdx.x;
    if (by < nq) {
        const int i0 = DG * by;
        const int nv = min(DG, nvec - i0);
        double acc[2 * DG];
#pragma unroll
        for (int t = 0; t < 2 * DG; t++) acc[t] = 0.0;
        const double* q0 = V + (long)i0 * ldv;
        if (nv == DG) {
            for (long e = e0; e < N; e += stride) {
                const double ue = u[e], we = w[e];
#pragma unroll
                for (int t = 0; t < DG; t++) {
                    const double qe = q0[(long)t * ldv + e];
                    acc[2 * t] += qe * ue;
                    acc[2 * t + 1] += qe * we;
                }
            }
        } else {
            for (long e = e0; e < N; e += stride) {
                const double ue = u[e], we = w[e];
                for (int t = 0; t < nv; t++) {
                    const double qe = q0[(long)t * ldv + e];
                    acc[2 * t] += qe * ue;
                    acc[2 * t + 1] += qe * we;
                }
            }
        }
        bsum<2 * DG>(acc, sm);
        if (threadIdx.x == 0)
            for (int t = 0; t < 2 * nv; t++) partial[(long)(2 * i0 + t) * nbx + bx] = acc[t];
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
            for (int t = 0; t < 3; t++) partial[(long)(2 * nvec + t) * nbx + bx] = acc[t];
    }
}

/* the update pass, UN basis vectors per inner step */
template <int UN>
__global__ void __launch_bounds__(256) k_upd(const double* __restrict__ V, long ldv, int nvec,
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
        for (; i + UN <= nvec; i += UN) {
            double q[UN];
#pragma unroll
            for (int k = 0; k < UN; k++) q[k] = V[(long)(i + k) * ldv + e];
#pragma unroll
            for (int k = 0; k < UN; k++) {
                su += a[i + k] * q[k];
                sw += cc[i + k] * q[k];
            }
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

int main(int argc, char** argv)
{
    const long N = argc > 1 ? atol(argv[1]) : 1400832;
    const int MAXV = 92, NB = 1024, REPS = 40;
    double *V, *u, *w, *part, *coef;
    CK(hipMalloc(&V, sizeof(double) * N * MAXV));
    CK(hipMalloc(&u, sizeof(double) * N));
    CK(hipMalloc(&w, sizeof(double) * N));
    CK(hipMalloc(&part, sizeof(double) * NB * (2 * MAXV + 4)));
    CK(hipMalloc(&coef, sizeof(double) * 2 * MAXV));
    std::vector<double> h(N);
    for (long i = 0; i < N; i++) h[i] = 1e-3 * (double)((i * 7919) % 1000);
    for (int v = 0; v < MAXV; v++) CK(hipMemcpy(V + (long)v * N, h.data(), sizeof(double) * N, hipMemcpyHostToDevice));
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
        printf("%-22s nv=%2d  %8.2f us  %7.1f GB/s\n", name, nv, us, vecs * 8.0 * N / (us * 1e3));
    };
    for (int nv : {8, 24, 45, 68, 89}) {
        const double vd = nv + 2, vu = nv + 4;
        int nq8 = (nv + 7) / 8, nq16 = (nv + 15) / 16, nq4 = (nv + 3) / 4;
        run("dot DG8 2D", nv, vd, [&] { k_dot<8, false><<<dim3(NB, nq8 + 1), 256>>>(V, N, nv, u, w, N, part, NB); });
        run("dot DG8 yfast", nv, vd, [&] { k_dot<8, true><<<dim3(NB * (nq8 + 1)), 256>>>(V, N, nv, u, w, N, part, NB); });
        run("dot DG16 yfast", nv, vd, [&] { k_dot<16, true><<<dim3(NB * (nq16 + 1)), 256>>>(V, N, nv, u, w, N, part, NB); });
        run("dot DG4 yfast", nv, vd, [&] { k_dot<4, true><<<dim3(NB * (nq4 + 1)), 256>>>(V, N, nv, u, w, N, part, NB); });
        run("dot DG8 yfast nb512", nv, vd, [&] { k_dot<8, true><<<dim3(512 * (nq8 + 1)), 256>>>(V, N, nv, u, w, N, part, 512); });
        run("dot DG8 yfast nb2048", nv, vd, [&] { k_dot<8, true><<<dim3(2048 * (nq8 + 1)), 256>>>(V, N, nv, u, w, N, part, 2048); });
        const unsigned G = (unsigned)std::min<long>((N + 255) / 256, 2048);
        const unsigned G2 = (unsigned)((N + 255) / 256);
        run("upd UN2", nv, vu, [&] { k_upd<2><<<G, 256>>>(V, N, nv, coef, 1.0, 0.0, u, w, N); });
        run("upd UN4", nv, vu, [&] { k_upd<4><<<G, 256>>>(V, N, nv, coef, 1.0, 0.0, u, w, N); });
        run("upd UN8", nv, vu, [&] { k_upd<8><<<G, 256>>>(V, N, nv, coef, 1.0, 0.0, u, w, N); });
        run("upd UN4 full grid", nv, vu, [&] { k_upd<4><<<G2, 256>>>(V, N, nv, coef, 1.0, 0.0, u, w, N); });
        run("upd UN8 full grid", nv, vu, [&] { k_upd<8><<<G2, 256>>>(V, N, nv, coef, 1.0, 0.0, u, w, N); });
    }
    return 0;
}
