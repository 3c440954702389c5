# coarse T/S inverse GEMV with the default (temporal) load policy
sed -i 's/a\[u\] = c < N ? __builtin_nontemporal_load(A + c) : 0.0;/a[u] = c < N ? A[c] : 0.0;/' csrc/prec_gs.hip
