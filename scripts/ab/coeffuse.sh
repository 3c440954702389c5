# one rank: the DCGS2 dot rows summed over the workgroup partials inside the coefficient
# kernel (one 1024-thread launch instead of k_mdot_final + k_dcgs_coef)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
anchor='/* DCGS2 update pass, one read of Q:'
new='''/* rows t < nrow of hb = sum over the nb partials (partial[t * nb + b]), one wave per row in
 * turn, then the coefficients as k_dcgs_coef (one rank: no sum over ranks in between) */
__global__ void __launch_bounds__(1024) k_dcgs_final_coef(const double* __restrict__ partial, int nb,
                                                          double* __restrict__ hb, int nv,
                                                          double* __restrict__ coef)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int nrow = 2 * nv + 3;
    for (int t = wv; t < nrow; t += nw) {
        double a = 0.0;
        for (int b = lane; b < nb; b += 64) a += partial[(int64_t)t * nb + b];
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) hb[t] = a;
    }
    __syncthreads();
    __shared__ double sm[2 * 16];
    __shared__ double tot[2];
    double v[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
        const double a = hb[2 * i], b = hb[2 * i + 1];
        v[0] += a * a;
        v[1] += a * b;
    }
    block_sum_n<2>(v, sm);
    if (threadIdx.x == 0) {
        tot[0] = v[0];
        tot[1] = v[1];
    }
    __syncthreads();
    const double beta2 = hb[2 * nv] - tot[0];
    const double bt = beta2 > 0.0 ? sqrt(beta2) : 0.0;
    const bool ok = bt > 0.0 && bt <= 1.79e308;
    const double hjj = ok ? (hb[2 * nv + 1] - tot[1]) / bt : 0.0;
    const double gamma = ok ? hjj / bt : 0.0;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
        const double a = hb[2 * i], b = hb[2 * i + 1];
        coef[i] = a;
        coef[nv + i] = b - a * gamma;
    }
    if (threadIdx.x == 0) {
        coef[DCGS_SCAL] = ok ? 1.0 / bt : 0.0;
        coef[DCGS_SCAL + 1] = gamma;
        hb[2 * nv + 3] = bt;
        hb[2 * nv + 4] = hjj;
    }
}

'''
s=s.replace(anchor,new+anchor,1)
old='''                hipLaunchKernelGGL(k_mdot_final, dim3(2 * nv + 3), dim3(256), 0, c->stream, c->d_part.p,
                                   nbx1, 2 * nv + 3, c->d_hbuf.p);
                if ((rc2 = allreduce_sum(c, c->d_hbuf.p, 2 * nv + 3))) return rc2;
                hipLaunchKernelGGL(k_dcgs_coef, dim3(1), dim3(256), 0, c->stream, c->d_hbuf.p, nv,
                                   c->d_hbuf.p + RED_ROWS);'''
new2='''                if (c->nranks <= 1) {
                    hipLaunchKernelGGL(k_dcgs_final_coef, dim3(1), dim3(1024), 0, c->stream, c->d_part.p, nbx1,
                                       c->d_hbuf.p, nv, c->d_hbuf.p + RED_ROWS);
                } else {
                    hipLaunchKernelGGL(k_mdot_final, dim3(2 * nv + 3), dim3(256), 0, c->stream, c->d_part.p,
                                       nbx1, 2 * nv + 3, c->d_hbuf.p);
                    if ((rc2 = allreduce_sum(c, c->d_hbuf.p, 2 * nv + 3))) return rc2;
                    hipLaunchKernelGGL(k_dcgs_coef, dim3(1), dim3(256), 0, c->stream, c->d_hbuf.p, nv,
                                       c->d_hbuf.p + RED_ROWS);
                }'''
assert old in s
s=s.replace(old,new2)
open(p,'w').write(s)
PY
