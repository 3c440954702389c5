# T/S right-hand side coefficients with the default (temporal) load policy
sed -i 's/? 0.0 : __builtin_nontemporal_load(val + (int64_t)(B + s) \* nloc + lc);/? 0.0 : val[(int64_t)(B + s) * nloc + lc];/' csrc/prec_gs.hip
