/*
 * comm.hip -- RCCL over xGMI for the latitude-band decomposition.
 *
 * Replaces the Epetra/MPI communication of the reference path: the Import of ghost rows
 * before matrix_/rhs_ and Apply (TRIOS_Domain.C Solve2Assembly, Epetra_CrsMatrix::Apply)
 * and the MPI_Allreduce inside Belos' dots and norms and THCM's intcond/forcing sums.
 * In the j-major ext layout every halo is a contiguous slab of whole latitude rows, so an
 * exchange is one ncclSend/ncclRecv pair per neighbour straight from the vector, grouped
 * and enqueued on the context stream.  One rank: all calls are no-ops.
 */
#include <rccl/rccl.h>

#include <cstring>

#include "common.h"

namespace iemic {

#define NCCL_OK(expr)                                                                    \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess) {                                                         \
            set_error(std::string(#expr) + ": " + ncclGetErrorString(r_));               \
            return IEMIC_EDEVICE;                                                        \
        }                                                                                \
    } while (0)

int comm_unique_id(unsigned char* id128)
{
    ncclUniqueId uid;
    NCCL_OK(ncclGetUniqueId(&uid));
    memcpy(id128, &uid, sizeof(uid));
    return 0;
}

int comm_init(iemic_ctx* c, const unsigned char* id, int rank, int nranks)
{
    if (nranks <= 1) return 0;
    ncclUniqueId uid;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm;
    NCCL_OK(ncclCommInitRank(&comm, nranks, uid, rank));
    c->comm = (void*)comm;
    return 0;
}

void comm_destroy(iemic_ctx* c)
{
    if (c->comm) (void)ncclCommDestroy((ncclComm_t)c->comm);
    c->comm = nullptr;
}

int allreduce_sum(iemic_ctx* c, double* dev, int count)
{
    if (c->nranks <= 1 || count <= 0) return 0;
    NCCL_OK(ncclAllReduce(dev, dev, (size_t)count, ncclDouble, ncclSum, (ncclComm_t)c->comm,
                          c->stream));
    return 0;
}

/* exchange rows_j (<= HALO) latitude rows with the neighbouring bands */
int halo_exchange(iemic_ctx* c, double* v, int rows_j)
{
    if (c->nranks <= 1) return 0;
    const int64_t slab = (int64_t)NUN * c->l * c->n;          /* doubles per latitude row */
    const int64_t cnt = slab * rows_j;
    const int64_t own_first = (int64_t)NUN * c->own0;          /* first owned row          */
    const int64_t own_end = own_first + c->nlrows;             /* one past the last owned  */
    ncclComm_t comm = (ncclComm_t)c->comm;
    NCCL_OK(ncclGroupStart());
    if (c->rank > 0) {
        NCCL_OK(ncclSend(v + own_first, (size_t)cnt, ncclDouble, c->rank - 1, comm, c->stream));
        NCCL_OK(ncclRecv(v + own_first - cnt, (size_t)cnt, ncclDouble, c->rank - 1, comm, c->stream));
    }
    if (c->rank < c->nranks - 1) {
        NCCL_OK(ncclSend(v + own_end - cnt, (size_t)cnt, ncclDouble, c->rank + 1, comm, c->stream));
        NCCL_OK(ncclRecv(v + own_end, (size_t)cnt, ncclDouble, c->rank + 1, comm, c->stream));
    }
    NCCL_OK(ncclGroupEnd());
    return 0;
}

}  // namespace iemic
