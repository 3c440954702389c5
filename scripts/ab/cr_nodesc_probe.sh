# timing probe only (wrong values): the Schur step vectors staged from fixed offsets of b, so
# no vector load waits for the workgroup's descriptor (upper bound of pushing the vectors
# into consumer order)
python3 - <<'PY'
p='csrc/schur_cr.hip'
s=open(p).read()
old='''            int ref = refs[0];
#pragma unroll
            for (int q = 1; q < CR_MT; q++)
                if (qv[i] == q) ref = refs[q];
            v[i] = cv[i] >= 0 ? base[ref >> 28][(ref & 0x0fffffff) + cv[i]] : 0.0;'''
new='''            (void)refs;
            v[i] = cv[i] >= 0 ? b[(w % 64) * m + qv[i] * m + cv[i]] : 0.0;'''
assert old in s
s=s.replace(old,new)
s=s.replace('const int tot = nv * m;','const int tot = 6 * m;')
open(p,'w').write(s)
PY
