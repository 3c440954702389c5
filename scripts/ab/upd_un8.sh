# DCGS2 update pass with eight basis vectors per step
sed -i 's/^    constexpr int UN = 4;/    constexpr int UN = 8;/' csrc/krylov.hip
grep -q "constexpr int UN = 8;" csrc/krylov.hip
