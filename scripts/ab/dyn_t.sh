# dynamics defect coefficients with the default (temporal) load policy
sed -i 's/acc\[q\] += __builtin_nontemporal_load(val + (int64_t)s \* nloc + lc) \* z/acc[q] += val[(int64_t)s * nloc + lc] * z/' csrc/krylov.hip
