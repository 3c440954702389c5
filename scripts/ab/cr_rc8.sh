# Schur apply steps in 8-row chunks (twice the workgroups of the 16-row default)
sed -i 's/^    int rcw = 16;$/    int rcw = 8;/' csrc/schur_cr.hip
grep -q "^    int rcw = 8;$" csrc/schur_cr.hip
