# DCGS2 dot pass in the plain block order (group index fastest, no XCD dealing)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
a=s.index('    const int G = nq + 1, sb = blockIdx.x / (8 * G), rem = blockIdx.x % (8 * G);')
b=s.index('\n', s.index('const int by = rem / 8, bx = sb * 8 + rem % 8;'))
s=s[:a]+'    const int by = blockIdx.x % (nq + 1), bx = blockIdx.x / (nq + 1);'+s[b:]
open(p,'w').write(s)
PY
