# DCGS2 one-read dot pass with 8 16-byte elements of u, w per lane
sed -i 's/^constexpr int DOT1_E = 4;/constexpr int DOT1_E = 8;/' csrc/krylov.hip
grep -q "DOT1_E = 8;" csrc/krylov.hip
