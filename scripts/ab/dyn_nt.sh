# dynamics defect coefficients loaded non-temporally (re-test with the Krylov basis streamed
# non-temporally)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
old='acc[q] += val[(int64_t)s * nloc + lc] * z[(int64_t)cidx + ps * sl.var];'
assert old in s
s=s.replace(old,'acc[q] += __builtin_nontemporal_load(val + (int64_t)s * nloc + lc) * z[(int64_t)cidx + ps * sl.var];')
open(p,'w').write(s)
PY
