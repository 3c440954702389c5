// Coefficient-layout probe: the defect's read pattern (a workgroup of 4 waves per 64 cells,
// each wave reading 16 of the 64 slots of its cells) on the slot-major layout val[s][cell]
// (one 512-B chunk per slot and wave, chunks nloc * 8 B apart) against a tile-blocked layout
// val[cell / 64][s][cell % 64] (a workgroup's 64 slots x 64 cells contiguous, 32 KB), same
// bytes, same arithmetic.  Prints GB/s for both at the 2- and 1-degree cell counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool BLOCKED>
__global__ void __launch_bounds__(256) k_read(const double* __restrict__ val, double* __restrict__ out, int64_t n,
                                              int nblk)
{
    __shared__ double red[4][64];
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t cell = (int64_t)tile * 64 + c;
    double v[16];
    if (cell < n) {
#pragma unroll
        for (int s = 0; s < 16; s++) {
            const int slot = 16 * g + s;
            v[s] = BLOCKED ? val[((int64_t)tile * 64 + slot) * 64 + c] : val[(int64_t)slot * n + cell];
        }
    } else {
#pragma unroll
        for (int s = 0; s < 16; s++) v[s] = 0.0;
    }
    double a = 0.0;
#pragma unroll
    for (int s = 0; s < 16; s++) a += v[s] * (s + 1);
    red[g][c] = a;
    __syncthreads();
    if (g == 0 && cell < n) out[cell] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

int main()
{
    for (int64_t n : {233472LL, 1867776LL}) {
        const int nblk = (int)((n + 63) / 64);
        const size_t nv = (size_t)64 * nblk * 64;
        double *val, *out;
        CK(hipMalloc(&val, nv * sizeof(double)));
        CK(hipMalloc(&out, n * sizeof(double)));
        CK(hipMemset(val, 0, nv * sizeof(double)));
        // flush buffer, larger than the last-level caches
        double* fl;
        const size_t nf = (size_t)64 << 20;
        CK(hipMalloc(&fl, nf * sizeof(double)));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const unsigned grid = 8u * (unsigned)((nblk + 7) / 8);
        for (int b = 0; b < 2; b++) {
            float best = 1e30f, sum = 0.f;
            const int reps = 20;
            for (int r = 0; r < reps + 2; r++) {
                CK(hipMemsetAsync(fl, r, nf * sizeof(double)));
                CK(hipEventRecord(e0));
                if (b) hipLaunchKernelGGL(k_read<true>, dim3(grid), dim3(256), 0, 0, val, out, n, nblk);
                else hipLaunchKernelGGL(k_read<false>, dim3(grid), dim3(256), 0, 0, val, out, n, nblk);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) { best = ms < best ? ms : best; sum += ms; }
            }
            const double bytes = 64.0 * 8 * n + 8.0 * n;
            printf("n %lld %s: best %.2f us avg %.2f us  %.0f GB/s (avg)\n", (long long)n, b ? "blocked   " : "slot-major",
                   best * 1e3, sum / 20 * 1e3, bytes / (sum / 20 * 1e-3) / 1e9);
        }
        CK(hipFree(val));
        CK(hipFree(out));
        CK(hipFree(fl));
    }
    return 0;
}
