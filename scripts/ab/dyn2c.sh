# dynamics defect with two cells per lane (128-cell workgroups): twice the independent loads
# in flight per wave, half the waves
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('__global__ void __launch_bounds__(256) k_spmv_dyn(')
b=s.index('int spmv_dyn_defect(', a)
new='''__global__ void __launch_bounds__(256) k_spmv_dyn(SubLay X, const double* __restrict__ val,
                                                  const double* __restrict__ z,
                                                  const double* __restrict__ r,
                                                  const uint8_t* __restrict__ knP,
                                                  double* __restrict__ d, int64_t nloc, int nblk, int64_t ps)
{
    __shared__ double red[4][2][128];
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t lc0 = (int64_t)tile * 128;
    const int64_t e0 = (int64_t)HALO * X.l * X.nx;
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int64_t lc = lc0 + 64 * h + c;
        if (lc >= nloc) continue;
        const int il = (int)(lc % X.nx), k = (int)((lc / X.nx) % X.l), j = X.jb0 + (int)(lc / ((int64_t)X.nx * X.l));
        int nc[3][9];
        nb_cells(X, il, j, k, nc);
        const int64_t cell = e0 + lc;
        const int v0 = g == 0 ? 0 : g - 1;
        const bool on[2] = {!knP[cell + ps * v0], g > 0 && !knP[cell + ps * (v0 + 1)]};
        if (g == 0) dyn_partial<0, 16>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else if (g == 1) dyn_partial<16, 32>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else if (g == 2) dyn_partial<32, 48>(val, z, lc, nloc, nc, on, ps, acc[h]);
        else dyn_partial<48, 64>(val, z, lc, nloc, nc, on, ps, acc[h]);
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
        red[g][0][64 * h + c] = acc[h][0];
        red[g][1][64 * h + c] = acc[h][1];
    }
    __syncthreads();
    const int R = threadIdx.x >> 6;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int cc = 64 * h + (threadIdx.x & 63);
        if (lc0 + cc >= nloc) break;
        const double sum = R == 0 ? red[0][0][cc] + red[1][0][cc]
                         : R == 1 ? red[1][1][cc] + red[2][0][cc]
                         : R == 2 ? red[2][1][cc] + red[3][0][cc]
                                  : red[3][1][cc];
        const int64_t cell = e0 + lc0 + cc, e = cell + ps * R;
        d[e] = knP[e] ? 0.0 : r[NUN * cell + R] - sum;
    }
}

'''
s=s[:a]+new+s[b:]
old="""    const int nblk = (int)((c->nloc + 63) / 64);
    const unsigned grid = 8u * (unsigned)((nblk + 7) / 8);
    hipLaunchKernelGGL(k_spmv_dyn,"""
new2="""    const int nblk = (int)((c->nloc + 127) / 128);
    const unsigned grid = 8u * (unsigned)((nblk + 7) / 8);
    hipLaunchKernelGGL(k_spmv_dyn,"""
assert old in s
s=s.replace(old,new2)
open(p,'w').write(s)
PY
