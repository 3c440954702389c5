# ptil + Schur right-hand side: the rcol coefficients loaded non-temporally
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
reps=[('for (int e = 0; e < 9; e++) a0 += R[e * es] * rr[PL(nc9[e], WW)];','for (int e = 0; e < 9; e++) a0 += __builtin_nontemporal_load(R + e * es) * rr[PL(nc9[e], WW)];'),
      ('a1 += R[(9 + q4) * es] * rr[PL(qc, UU)];','a1 += __builtin_nontemporal_load(R + (9 + q4) * es) * rr[PL(qc, UU)];'),
      ('a2 += R[(13 + q4) * es] * rr[PL(qc, VV)];','a2 += __builtin_nontemporal_load(R + (13 + q4) * es) * rr[PL(qc, VV)];'),
      ('a2 += R[17 * es] * rr[PL(cell, PP)];','a2 += __builtin_nontemporal_load(R + 17 * es) * rr[PL(cell, PP)];')]
for o,n in reps:
    assert o in s, o
    s=s.replace(o,n)
open(p,'w').write(s)
PY
