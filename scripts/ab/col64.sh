# transposed column kernels in 64-column tiles (1024 threads at 16 levels)
sed -i 's/^constexpr int COL_TI = 16;/constexpr int COL_TI = 64;/' csrc/prec_gs.hip
