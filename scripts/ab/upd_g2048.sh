# DCGS2 update pass on 2048 workgroups
sed -i 's/hipLaunchKernelGGL(k_dcgs_update, dim3(1024)/hipLaunchKernelGGL(k_dcgs_update, dim3(2048)/' csrc/krylov.hip
grep -q "k_dcgs_update, dim3(2048)" csrc/krylov.hip
