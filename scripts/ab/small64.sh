# the dense tail GEMV of the Schur solve and the coarsest T/S GEMV in 64-thread workgroups
# (one row each: 4x the workgroups)
python3 - <<'PY'
for p, kern in (('csrc/schur_cr.hip', 'k_cr_tail('), ('csrc/prec_gs.hip', 'k_gemv_w(')):
    s=open(p).read()
    a=s.index(kern); b=s.index('\n}\n', a)
    k=s[a:b]
    k=k.replace('r = blockIdx.x * 4 + (threadIdx.x >> 6);','r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);')
    k=k.replace('c += 256) vb[c] = b[c];','c += blockDim.x) vb[c] = b[c];')
    s=s[:a]+k+s[b:]
    if kern == 'k_cr_tail(':
        old='hipLaunchKernelGGL(k_cr_tail, dim3((cr.tM + 3) / 4), dim3(256),'
        assert old in s
        s=s.replace(old,'hipLaunchKernelGGL(k_cr_tail, dim3(cr.tM), dim3(64),')
    else:
        for NLv in ('16','32'):
            old=f'hipLaunchKernelGGL(k_gemv_w<{NLv}>, dim3((unsigned)((N + 3) / 4)), dim3(256),'
            assert old in s
            s=s.replace(old,f'hipLaunchKernelGGL(k_gemv_w<{NLv}>, dim3((unsigned)N), dim3(64),')
    open(p,'w').write(s)
PY
