# dynamics defect with eight waves of 8 slots per 64 cells (512 threads): half the loads per
# lane, twice the waves
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('__global__ void __launch_bounds__(256) k_spmv_dyn(')
b=s.index('int spmv_dyn_defect(', a)
new='''__global__ void __launch_bounds__(512) k_spmv_dyn(SubLay X, const double* __restrict__ val,
                                                  const double* __restrict__ z,
                                                  const double* __restrict__ r,
                                                  const uint8_t* __restrict__ knP,
                                                  double* __restrict__ d, int64_t nloc, int nblk, int64_t ps)
{
    __shared__ double red[8][2][64];
    const int per = (nblk + 7) >> 3;
    const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (tile >= nblk) return;
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t lc0 = (int64_t)tile * 64, lc = lc0 + c;
    const bool act = lc < nloc;
    const int64_t e0 = (int64_t)HALO * X.l * X.nx;
    double acc[2] = {0.0, 0.0};
    if (act) {
        const int il = (int)(lc % X.nx), k = (int)((lc / X.nx) % X.l), j = X.jb0 + (int)(lc / ((int64_t)X.nx * X.l));
        int nc[3][9];
        nb_cells(X, il, j, k, nc);
        const int64_t cell = e0 + lc;
        /* rows of the groups: g0-2 {U} g3-4 {V} g5 {V, W} g6 {W, P} g7 {P} */
        const int v0 = g < 3 ? 0 : g < 5 ? 1 : g == 5 ? 1 : g == 6 ? 2 : 3;
        const bool on[2] = {!knP[cell + ps * v0], (g == 5 || g == 6) && !knP[cell + ps * (v0 + 1)]};
        switch (g) {
        case 0: dyn_partial<0, 8>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 1: dyn_partial<8, 16>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 2: dyn_partial<16, 24>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 3: dyn_partial<24, 32>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 4: dyn_partial<32, 40>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 5: dyn_partial<40, 48>(val, z, lc, nloc, nc, on, ps, acc); break;
        case 6: dyn_partial<48, 56>(val, z, lc, nloc, nc, on, ps, acc); break;
        default: dyn_partial<56, 64>(val, z, lc, nloc, nc, on, ps, acc); break;
        }
    }
    red[g][0][c] = acc[0];
    red[g][1][c] = acc[1];
    __syncthreads();
    if (threadIdx.x >= 256) return;
    const int R = threadIdx.x >> 6, cc = threadIdx.x & 63;
    if (lc0 + cc >= nloc) return;
    const double sum = R == 0 ? (red[0][0][cc] + red[1][0][cc]) + red[2][0][cc]
                     : R == 1 ? (red[3][0][cc] + red[4][0][cc]) + red[5][0][cc]
                     : R == 2 ? red[5][1][cc] + red[6][0][cc]
                              : red[6][1][cc] + red[7][0][cc];
    const int64_t cell = e0 + lc0 + cc, e = cell + ps * R;
    d[e] = knP[e] ? 0.0 : r[NUN * cell + R] - sum;
}

'''
s=s[:a]+new+s[b:]
old="""    hipLaunchKernelGGL(k_spmv_dyn, dim3(grid), dim3(256),"""
assert old in s
s=s.replace(old,"""    hipLaunchKernelGGL(k_spmv_dyn, dim3(grid), dim3(512),""")
open(p,'w').write(s)
PY
