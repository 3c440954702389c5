# tail and coarsest GEMVs: the right-hand side staged with all of a lane's loads issued first
python3 - <<'PY'
for p, old, nmax in (('csrc/schur_cr.hip', '    for (int c = threadIdx.x; c < M; c += 256) vb[c] = b[c];', 'CR_TAIL_MAX'),
                     ('csrc/prec_gs.hip', '    for (int c = threadIdx.x; c < N; c += 256) vb[c] = b[c];', '64 * NL')):
    s=open(p).read()
    assert old in s, p
    lim = 'M' if 'M;' in old else 'N'
    new=f"""    {{
        constexpr int SV = ({nmax} + 255) / 256;
        double t_[SV];
#pragma unroll
        for (int u = 0; u < SV; u++) {{
            const int c = threadIdx.x + 256 * u;
            t_[u] = c < {lim} ? b[c] : 0.0;
        }}
#pragma unroll
        for (int u = 0; u < SV; u++) {{
            const int c = threadIdx.x + 256 * u;
            if (c < {lim}) vb[c] = t_[u];
        }}
    }}"""
    s=s.replace(old,new)
    open(p,'w').write(s)
PY
