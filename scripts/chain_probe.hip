// Cost of a chain of dependent small launches on one stream (untraced, HIP events): what a
// latency-bound phase of the block GS apply pays per launch, by the number of dependent
// memory rounds inside the kernel.  Prints us per launch for each variant.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_nop(double* p) {}
__global__ void k_store(double* p, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = 1.0;
}
__global__ void k_ld1(const double* __restrict__ a, double* __restrict__ p, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = a[t] * 2.0 + 1.0;
}
/* two dependent rounds: an index, then the value it points to */
__global__ void k_ld2(const int* __restrict__ idx, const double* __restrict__ a, double* __restrict__ p, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = a[idx[t]] * 2.0 + 1.0;
}
/* one round of 16 independent loads per thread (a line solve's factors + neighbours) */
__global__ void k_ld16(const double* __restrict__ a, double* __restrict__ p, int n, int stride)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) s += a[t + q * stride];
    p[t] = s;
}

int main()
{
    const int NMAX = 1 << 22;
    double *a, *p;
    int* idx;
    hipMalloc(&a, sizeof(double) * NMAX * 17);
    hipMalloc(&p, sizeof(double) * NMAX);
    hipMalloc(&idx, sizeof(int) * NMAX);
    hipMemset(a, 0, sizeof(double) * NMAX * 17);
    hipMemset(idx, 0, sizeof(int) * NMAX);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int sizes[5] = {256, 1920, 29184, 233472, 1 << 20};
    const int R = 200;
    for (int v = 0; v < 5; v++) {
        for (int si = 0; si < 5; si++) {
            const int n = sizes[si];
            const dim3 g((n + 255) / 256), b(256);
            auto launch = [&]() {
                switch (v) {
                case 0: hipLaunchKernelGGL(k_nop, g, b, 0, s, p); break;
                case 1: hipLaunchKernelGGL(k_store, g, b, 0, s, p, n); break;
                case 2: hipLaunchKernelGGL(k_ld1, g, b, 0, s, a, p, n); break;
                case 3: hipLaunchKernelGGL(k_ld2, g, b, 0, s, idx, a, p, n); break;
                default: hipLaunchKernelGGL(k_ld16, g, b, 0, s, a, p, n, n); break;
                }
            };
            for (int r = 0; r < 20; r++) launch();
            hipEventRecord(e0, s);
            for (int r = 0; r < R; r++) launch();
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            static const char* nm[5] = {"nop", "store", "load1", "load2dep", "load16"};
            printf("%-9s threads %8d: %.2f us/launch\n", nm[v], n, ms * 1e3 / R);
        }
    }
    return 0;
}
