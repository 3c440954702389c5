# column kernels (ptil + rcol, p/w) in 512-thread workgroups: 32 columns x 16 levels, twice
# the workgroups (228 -> 456 at 2 degrees: every CU busy)
sed -i 's|^constexpr int col_ti() { return 1024 / LP; }|constexpr int col_ti() { return 512 / LP; }|' csrc/prec_gs.hip
sed -i 's|^    const int cti = 1024 / Pl;|    const int cti = 512 / Pl;|' csrc/prec_gs.hip
sed -i 's|^    const dim3 bct(1024u);|    const dim3 bct(512u);|' csrc/prec_gs.hip
grep -q "return 512 / LP" csrc/prec_gs.hip && grep -q "bct(512u)" csrc/prec_gs.hip && grep -q "cti = 512 / Pl" csrc/prec_gs.hip
