# A/B: the dynamics defect capped at 4 waves per SIMD
sed -i 's/__global__ void __launch_bounds__(256) k_spmv_dyn(/__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) k_spmv_dyn(/' csrc/krylov.hip
grep -q "amdgpu_waves_per_eu(1, 4))) k_spmv_dyn" csrc/krylov.hip
