/* prec_gs.hip -- block Gauss-Seidel preconditioner (placeholder, filled in next). */
#include "common.h"
namespace iemic {
int gs_compute(iemic_ctx*, const iemic_krylov*) { set_error("block GS not built yet"); return IEMIC_EINVAL; }
int gs_apply(iemic_ctx*, const double*, double*) { return IEMIC_EINVAL; }
}
