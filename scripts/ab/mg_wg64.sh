# z-line and restriction launches in 64-thread workgroups (4 columns each): a coarse level's
# few columns spread over 4x the CUs
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
s=s.replace('''#define MG_LAUNCH_P(P, KERNEL, GRID, ...)''','''#define MG_LAUNCH_P64(P, KERNEL, GRID, ...)                                                \\
    do {                                                                                   \\
        if ((P) == 16) hipLaunchKernelGGL(KERNEL<16>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \\
        else if ((P) == 32) hipLaunchKernelGGL(KERNEL<32>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__); \\
        else hipLaunchKernelGGL(KERNEL<64>, dim3(GRID), dim3(64), 0, s, __VA_ARGS__);     \\
    } while (0)
#define MG_LAUNCH_P(P, KERNEL, GRID, ...)''')
old='''    const unsigned g = blocks_for(mg_columns_of(V, colour) * P);
    if (!g) return 0;'''
new='''    const unsigned g = (unsigned)((mg_columns_of(V, colour) * P + 63) / 64);
    if (!g) return 0;'''
assert old in s
s=s.replace(old,new)
s=s.replace("MG_LAUNCH_P(P, k_mg_zl, g,","MG_LAUNCH_P64(P, k_mg_zl, g,")
s=s.replace("MG_LAUNCH_P(P, k_mg_rc, blocks_for((int64_t)C.n * C.mb * P),","MG_LAUNCH_P64(P, k_mg_rc, (unsigned)(((int64_t)C.n * C.mb * P + 63) / 64),")
open(p,'w').write(s)
PY
grep -q "MG_LAUNCH_P64(P, k_mg_rc" csrc/prec_gs.hip
