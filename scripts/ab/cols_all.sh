bash "$ROOT/scripts/ab/uvp_all.sh" && bash "$ROOT/scripts/ab/pw_all.sh" && bash "$ROOT/scripts/ab/ptil_all.sh"
