# SpMV coefficients with the default (temporal) load policy
sed -i 's/v\[s - S0\] = !act ? 0.0 : __builtin_nontemporal_load(val + (int64_t)s \* nloc + lc);/v[s - S0] = !act ? 0.0 : val[(int64_t)s * nloc + lc];/' csrc/krylov.hip
