# A/B: the coarse T/S levels by the unfused launches (k_mg_zl + k_mg_rc) instead of k_mg_dn / k_mg_up
sed -i 's/if (q < 1 || q + 1 >= gs.mg_nlev/if (true || q < 1 || q + 1 >= gs.mg_nlev/' csrc/prec_gs.hip
grep -q "if (true || q < 1" csrc/prec_gs.hip
