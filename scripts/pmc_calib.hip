// PMC calibration: streaming reads of a known byte count with 8-B and 16-B lanes and a
// streaming 8-B write, so rocprofv3 FETCH_SIZE / WRITE_SIZE can be converted to bytes for
// the access widths the library's kernels use (MI355X_MICROARCH.md: FETCH_SIZE reports
// 1/2 of a 16-B/lane stream on gfx950; other widths uncalibrated).  Development tool.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) k_read8(const double* __restrict__ a, int64_t n, double* out)
{
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 1.2345) out[0] = s;   // keeps the loads, never stores in practice
}
__global__ void __launch_bounds__(256) k_read16(const double2* __restrict__ a, int64_t n2, double* out)
{
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;
}
__global__ void __launch_bounds__(256) k_write8(double* __restrict__ a, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}

int main()
{
    const int64_t bytes = (int64_t)1 << 30, n = bytes / 8;   // 1 GiB: 4x the Infinity Cache
    double *a = nullptr, *out = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
    const dim3 G(4096), B(256);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k_read8, G, B, 0, 0, a, n, out);
        hipLaunchKernelGGL(k_read16, G, B, 0, 0, (const double2*)a, n / 2, out);
        hipLaunchKernelGGL(k_write8, G, B, 0, 0, a, n);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("calib bytes per launch: %lld\n", (long long)bytes);
    (void)hipFree(a);
    (void)hipFree(out);
    return 0;
}
