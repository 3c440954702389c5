# k_gs_ptil_rcol: corner and own-P loads issued on every cell (no branch on the P flag)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='''        if (pa) {
            /* the corner and own-P coefficients vanish on an inactive P row (land): not read */
#pragma unroll'''
new='''        {
#pragma unroll'''
assert old in s
s=s.replace(old,new)
old='''            if (k < l - 1 && !kw) {
                const double g0 = val[(int64_t)S_WP0 * ncell + (cell - L.own0)];
                const double g1 = val[(int64_t)S_WP1 * ncell + (cell - L.own0)];
                if (g0 != 0.0) {'''
new='''            if (k < l - 1) {
                const double g0 = val[(int64_t)S_WP0 * ncell + (cell - L.own0)];
                const double g1 = val[(int64_t)S_WP1 * ncell + (cell - L.own0)];
                if (pa && !kw && g0 != 0.0) {'''
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
