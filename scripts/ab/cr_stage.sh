# Schur apply step: the nv vectors staged in one flat pass (every lane's loads issued together)
python3 - <<'PY'
p='csrc/schur_cr.hip'
s=open(p).read()
old='''    const CrWg& d = wgs[w];
    const int nv = d.nv;
    const double* base[4] = {b, x, bv, xv};
    for (int q = 0; q < nv; q++) {
        const int ref = d.vref[q];
        const double* src = base[ref >> 28] + (ref & 0x0fffffff);
        for (int c = t; c < m; c += 256) vs[q][c] = src[c];
    }
    __syncthreads();'''
new='''    const CrWg& d = wgs[w];
    const int nv = d.nv;
    const double* base[4] = {b, x, bv, xv};
    {
        /* (vector, element) pairs dealt over the lanes, all loads before the first store */
        constexpr int SPT = ((CR_MT + 1) * 192 + 255) / 256;
        const int tot = nv * m;
        double v[SPT];
        int qv[SPT], cv[SPT], refs[CR_MT];
#pragma unroll
        for (int q = 0; q < CR_MT; q++) refs[q] = d.vref[q];
#pragma unroll
        for (int i = 0; i < SPT; i++) {
            const int e = t + 256 * i;
            qv[i] = e < tot ? e / m : 0;
            cv[i] = e < tot ? e - qv[i] * m : -1;
            int ref = refs[0];
#pragma unroll
            for (int q = 1; q < CR_MT; q++)
                if (qv[i] == q) ref = refs[q];
            v[i] = cv[i] >= 0 ? base[ref >> 28][(ref & 0x0fffffff) + cv[i]] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < SPT; i++)
            if (cv[i] >= 0) vs[qv[i]][cv[i]] = v[i];
    }
    __syncthreads();'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
