# k_gs_rr with 16-byte loads and stores of the AoS cell records and the planar flags
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old="""    double acc[NUN];
    bool kn[NUN];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        const int64_t row = NUN * cell + R;
        acc[R] = r[row];
        kn[R] = known[row] != 0;
        const double zv = kn[R] ? acc[R] : 0.0;
        z[row] = zv;
        zP[PL(cell, R)] = zv;
    }"""
new="""    double acc[NUN];
    bool kn[NUN];
    {
        const double2* r2 = reinterpret_cast<const double2*>(r + NUN * cell);
        const double2 a0 = r2[0], a1 = r2[1], a2 = r2[2];
        acc[0] = a0.x; acc[1] = a0.y; acc[2] = a1.x; acc[3] = a1.y; acc[4] = a2.x; acc[5] = a2.y;
    }
    double zv[NUN];
#pragma unroll
    for (int R = 0; R < NUN; R++) {
        kn[R] = known[NUN * cell + R] != 0;
        zv[R] = kn[R] ? acc[R] : 0.0;
        zP[PL(cell, R)] = zv[R];
    }
    {
        double2* z2 = reinterpret_cast<double2*>(z + NUN * cell);
        z2[0] = make_double2(zv[0], zv[1]);
        z2[1] = make_double2(zv[2], zv[3]);
        z2[2] = make_double2(zv[4], zv[5]);
    }"""
assert old in s
s=s.replace(old,new)
open(p,'w').write(s)
PY
