# packed Schur operators with the default (temporal) load policy
sed -i 's/__builtin_nontemporal_load(Pw + ((int64_t)q \* m + c) \* RC + rr)/Pw[((int64_t)q * m + c) * RC + rr]/' csrc/schur_cr.hip
