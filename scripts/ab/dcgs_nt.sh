# DCGS2 passes with non-temporal loads of the basis (streamed once per pass, 1 GB > the
# Infinity Cache)
python3 - <<'PY'
p='csrc/krylov.hip'
s=open(p).read()
helper='''__device__ __forceinline__ double2 ldnt2(const double2* p)
{
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
'''
a=s.index('constexpr int DOT1_E')
s=s[:a]+helper+s[a:]
reps=[('qn[k] = reinterpret_cast<const double2*>(V)[ex[k]];','qn[k] = ldnt2(reinterpret_cast<const double2*>(V) + ex[k]);'),
      ('qn[k] = qv[ex[k]];','qn[k] = ldnt2(qv + ex[k]);'),
      ('q[k] = reinterpret_cast<const double2*>(V + (int64_t)(i + k) * ldv)[e];','q[k] = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)(i + k) * ldv) + e);'),
      ('const double2 q = reinterpret_cast<const double2*>(V + (int64_t)i * ldv)[e];','const double2 q = ldnt2(reinterpret_cast<const double2*>(V + (int64_t)i * ldv) + e);')]
for o,n in reps:
    assert o in s, o
    s=s.replace(o,n)
open(p,'w').write(s)
PY
