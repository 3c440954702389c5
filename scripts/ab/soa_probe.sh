# timing probe only (wrong values): the AoS accesses of the dynamics-pass kernels (ptil + rcol,
# U/V, p/w with duv_uv, the entry k_gs_rr) made stride-1, as a component-planar layout would
# read them (upper bound of a planar-layout rewrite); set-up kernels untouched
python3 - <<'PY'
import re
p='csrc/prec_gs.hip'
s=open(p).read()
for name in ['k_gs_ptil_rcol(', 'k_gs_uvp(', 'k_gs_pw_t(', 'double duv_uv(', 'k_gs_rr(']:
    a=s.rindex(name) if name == 'double duv_uv(' else s.index(name)
    a=s.index('{', a)
    depth=0; b=a
    while True:
        if s[b]=='{': depth+=1
        elif s[b]=='}':
            depth-=1
            if depth==0: break
        b+=1
    s=s[:a]+s[a:b].replace('NUN * ','1 * ')+s[b:]
open(p,'w').write(s)
PY
