# DCGS2 one-read dot pass with 2 16-byte elements of u, w per lane
sed -i 's/^constexpr int DOT1_E = 4;/constexpr int DOT1_E = 2;/' csrc/krylov.hip
grep -q "DOT1_E = 2;" csrc/krylov.hip
