# k_gs_pw_t: the P-row loads issued on every cell (no branch on the P flag before them)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='''    if (pa) {
        /* an inactive P row (land) reads nothing: its (A, B) = (0, 0) */
        const double a = val[(int64_t)S_PW0 * ncell + (cell - L.own0)];
        const double b = val[(int64_t)S_PWM * ncell + (cell - L.own0)];
        const double rhs = rr[NUN * cell + PP] - duv_uv(val, known, z, i, j, k, cell - L.own0, L);
        pb = pbar[(int64_t)i * L.m + j];
        zp = z[NUN * cell + PP];
        if (wa && a != 0.0) {
            A = rhs / a;
            B = -b / a;
        }
    }'''
new='''    if (on) {
        const double a = val[(int64_t)S_PW0 * ncell + (cell - L.own0)];
        const double b = val[(int64_t)S_PWM * ncell + (cell - L.own0)];
        const double rhs = rr[NUN * cell + PP] - duv_uv(val, known, z, i, j, k, cell - L.own0, L);
        pb = pa ? pbar[(int64_t)i * L.m + j] : 0.0;
        zp = pa ? z[NUN * cell + PP] : 0.0;
        if (pa && wa && a != 0.0) {
            A = rhs / a;
            B = -b / a;
        }
    }'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
