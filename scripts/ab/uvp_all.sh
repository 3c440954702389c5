# k_gs_uvp: every cell issues its loads at once (no early return on land; stores predicated)
python3 - <<'PY'
p='csrc/prec_gs.hip'
s=open(p).read()
old='    if (!ua && !va) return;                 /* land: none of the point\'s operands is read */\n'
assert old in s
s=s.replace(old,'')
open(p,'w').write(s)
PY
