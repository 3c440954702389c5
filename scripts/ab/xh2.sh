# x halos on the first 2 intermediate T/S levels only
sed -i "s/^constexpr int MG_XHALO_LEVELS = 99;/constexpr int MG_XHALO_LEVELS = 2;/" csrc/prec_gs.hip
