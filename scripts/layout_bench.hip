// Layout micro-benchmark for the stencil-ELL values (development tool): one wavefront
// reads NS slot values for 64 cells, either slot-major SoA (val[s*ncell + c], the slot
// arrays 1.9 MB apart at 2 degrees) or tiled (val[(tile*NS + s)*64 + lane]: one
// contiguous 53 KB chunk per 64 cells).  Prints GB/s of each after an L3 flush.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NS = 104;

__global__ void __launch_bounds__(256) k_soa(const double* __restrict__ v, int64_t nc, double* out)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    double s = 0.0;
#pragma unroll 8
    for (int q = 0; q < NS; q++) s += v[(int64_t)q * nc + c];
    out[c] = s;
}
__global__ void __launch_bounds__(256) k_tiled(const double* __restrict__ v, int64_t nc, double* out)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    const double* b = v + (c >> 6) * (int64_t)NS * 64 + (c & 63);
    double s = 0.0;
#pragma unroll 8
    for (int q = 0; q < NS; q++) s += b[q * 64];
    out[c] = s;
}
__global__ void k_flush(const double2* __restrict__ a, int64_t n2, double* sink)
{
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        s += a[i].x + a[i].y;
    if (s == 1.2345e300) sink[0] = s;
}

int main()
{
    const int64_t nc = 233472;                       // 2-degree cells
    const int64_t nv = nc * NS;
    double *v, *out, *fl;
    const int64_t fb = (int64_t)1 << 30;
    if (hipMalloc(&v, nv * 8) || hipMalloc(&out, nc * 8) || hipMalloc(&fl, fb)) return 1;
    hipMemset(v, 0, nv * 8);
    hipMemset(fl, 0, fb);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 2; kind++) {
        float tot = 0;
        for (int r = 0; r < 21; r++) {
            hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (const double2*)fl, fb / 16, out);
            hipEventRecord(e0, 0);
            if (kind == 0) hipLaunchKernelGGL(k_soa, dim3((nc + 255) / 256), dim3(256), 0, 0, v, nc, out);
            else hipLaunchKernelGGL(k_tiled, dim3((nc + 255) / 256), dim3(256), 0, 0, v, nc, out);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r) tot += ms;
        }
        const double us = tot / 20 * 1e3;
        printf("%s: %.1f us  %.0f GB/s\n", kind ? "tiled64" : "soa", us, (nv * 8 + nc * 8) / (us * 1e-6) / 1e9);
    }
    return 0;
}
