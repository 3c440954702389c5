# A/B: the dynamics defect reading the W row's T/S slots again (z(T, S) = 0: same values)
sed -i '/if (sl.var == TT || sl.var == SS) continue;      \/\* z(T, S) = 0 in every pass \*\//d' csrc/krylov.hip
! grep -q "z(T, S) = 0 in every pass" csrc/krylov.hip
