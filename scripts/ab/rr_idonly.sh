# entry kernel: the output's identity rows only (the active rows are all written later: U/V/W/P
# by the last pass, T/S by the multigrid's final launches)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old="""        const double zv = kn[R] ? acc[R] : 0.0;
        z[row] = zv;
        zP[PL(cell, R)] = zv;"""
new="""        const double zv = kn[R] ? acc[R] : 0.0;
        if (kn[R] || rr) z[row] = zv;
        zP[PL(cell, R)] = zv;"""
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
