# x halos on the first 1 intermediate T/S levels only
sed -i "s/^constexpr int MG_XHALO_LEVELS = 99;/constexpr int MG_XHALO_LEVELS = 1;/" csrc/prec_gs.hip
