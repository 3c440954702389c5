/* krylov_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU FGMRES + preconditioner (filled in below). */
#include "thcm_oracle.h"
