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

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

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

/* ---- in-process group (test facility) ------------------------------------------------
 * Several band contexts of one problem in one process (one host thread each, e.g. on one
 * GPU, where RCCL refuses duplicate devices): collectives are host-staged through a shared
 * object with a reusable barrier.  Sums are taken in rank order, so results do not depend
 * on thread timing. */
struct LocalGroup {
    int P;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, generation = 0;
    std::vector<std::vector<double>> slot;
    std::vector<double*> vec;
    std::vector<iemic_ctx*> ctxs;
    explicit LocalGroup(int p) : P(p), slot(p), vec(p, nullptr), ctxs(p, nullptr) {}
    void barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        const int gen = generation;
        if (++arrived == P) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

static int local_allreduce(iemic_ctx* c, double* dev, int count)
{
    LocalGroup* g = (LocalGroup*)c->group;
    auto& mine = g->slot[c->rank];
    mine.resize(count);
    int rc = d2h(c, mine.data(), dev, sizeof(double) * count);
    if (rc) return rc;
    g->barrier();
    std::vector<double> sum(count, 0.0);
    for (int r = 0; r < g->P; r++)
        for (int q = 0; q < count; q++) sum[q] += g->slot[r][q];
    g->barrier();
    return h2d(c, dev, sum.data(), sizeof(double) * count);
}

static int local_halo(iemic_ctx* c, double* v, int width, int rows_j)
{
    LocalGroup* g = (LocalGroup*)c->group;
    const int64_t slab = (int64_t)width * c->l * c->n, cnt = slab * rows_j;
    const int64_t own_first = (int64_t)width * c->own0, own_end = own_first + (int64_t)width * c->nloc;
    HIP_OK(hipStreamSynchronize(c->stream));
    g->vec[c->rank] = v;
    g->barrier();
    /* neighbours' ext vectors have the same halo depth; their owned rows start at HALO */
    if (c->rank > 0) {
        /* lower halo <- last rows of rank-1's band; rank-1 owns the band below: its owned end */
        iemic_ctx* nb = g->ctxs[c->rank - 1];
        const double* src = g->vec[c->rank - 1] + (int64_t)width * (nb->own0 + nb->nloc) - cnt;
        HIP_OK(hipMemcpyAsync(v + own_first - cnt, src, sizeof(double) * cnt, hipMemcpyDeviceToDevice, c->stream));
    }
    if (c->rank < g->P - 1) {
        iemic_ctx* nb = g->ctxs[c->rank + 1];
        const double* src = g->vec[c->rank + 1] + (int64_t)width * nb->own0;
        HIP_OK(hipMemcpyAsync(v + own_end, src, sizeof(double) * cnt, hipMemcpyDeviceToDevice, c->stream));
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    g->barrier();
    return 0;
}

void* local_group_new(int nranks) { return nranks > 0 ? new LocalGroup(nranks) : nullptr; }
void local_group_free(void* g) { delete (LocalGroup*)g; }
void local_group_join(iemic_ctx* c, void* g)
{
    c->group = g;
    ((LocalGroup*)g)->ctxs[c->rank] = c;
}

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
    if (c->group) return local_allreduce(c, dev, count);
    NCCL_OK(ncclAllReduce(dev, dev, (size_t)count, ncclDouble, ncclSum, (ncclComm_t)c->comm,
                          c->stream));
    return 0;
}

/* exchange rows_j (<= HALO) latitude rows of a per-cell array (width doubles per ext
 * cell) with the neighbouring bands */
int halo_exchange_w(iemic_ctx* c, double* v, int width, int rows_j)
{
    if (c->nranks <= 1) return 0;
    if (c->group) return local_halo(c, v, width, rows_j);
    const int64_t slab = (int64_t)width * c->l * c->n;        /* doubles per latitude row */
    const int64_t cnt = slab * rows_j;
    const int64_t own_first = (int64_t)width * c->own0;        /* first owned cell         */
    const int64_t own_end = own_first + (int64_t)width * c->nloc; /* one past the last     */
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

int halo_exchange_pair(iemic_ctx* c, double* a, double* b)
{
    if (c->nranks <= 1) return 0;
    if (c->group) {
        int rc = local_halo(c, a, 1, 1);
        return rc ? rc : local_halo(c, b, 1, 1);
    }
    const int64_t cnt = (int64_t)c->l * c->n;                   /* one latitude row */
    const int64_t own_first = c->own0, own_end = own_first + c->nloc;
    ncclComm_t comm = (ncclComm_t)c->comm;
    NCCL_OK(ncclGroupStart());
    for (double* v : {a, b}) {
        if (c->rank > 0) {
            NCCL_OK(ncclSend(v + own_first, (size_t)cnt, ncclDouble, c->rank - 1, comm, c->stream));
            NCCL_OK(ncclRecv(v + own_first - cnt, (size_t)cnt, ncclDouble, c->rank - 1, comm, c->stream));
        }
        if (c->rank < c->nranks - 1) {
            NCCL_OK(ncclSend(v + own_end - cnt, (size_t)cnt, ncclDouble, c->rank + 1, comm, c->stream));
            NCCL_OK(ncclRecv(v + own_end, (size_t)cnt, ncclDouble, c->rank + 1, comm, c->stream));
        }
    }
    NCCL_OK(ncclGroupEnd());
    return 0;
}

/* state-vector halo (NUN doubles per cell) */
int halo_exchange(iemic_ctx* c, double* v, int rows_j) { return halo_exchange_w(c, v, NUN, rows_j); }

}  // namespace iemic
