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
#include <map>
#include <mutex>
#include <tuple>
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
    /* point-to-point mailbox: (src, dst, k) -> the k-th message src sent to dst in a batch */
    std::map<std::tuple<int, int, int>, std::vector<double>> box;
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

/* One batch of point-to-point messages.  The halo exchanges build their batch once
 * (halo_ops) and hand it to the transport: RCCL (one ncclGroupStart/End, messages to the
 * same peer matched in order, as NCCL requires) or, for in-process band groups, the host
 * mailbox below, which pairs the k-th send of rank a to b with the k-th receive of b from
 * a -- the same pairing rule, so the batches the tests run are the ones RCCL runs. */
struct P2P {
    bool send;
    double* buf;
    int64_t cnt;
    int peer;
};

/* rows_j (<= HALO) latitude rows of a per-cell array (width doubles per ext cell) to and
 * from the neighbouring bands */
static void halo_ops(const iemic_ctx* c, double* v, int width, int rows_j, std::vector<P2P>& ops)
{
    const int64_t slab = (int64_t)width * c->l * c->n;        /* doubles per latitude row */
    const int64_t cnt = slab * rows_j;
    const int64_t own_first = (int64_t)width * c->own0;        /* first owned cell         */
    const int64_t own_end = own_first + (int64_t)width * c->nloc; /* one past the last     */
    if (c->rank > 0) {
        ops.push_back({true, v + own_first, cnt, c->rank - 1});
        ops.push_back({false, v + own_first - cnt, cnt, c->rank - 1});
    }
    if (c->rank < c->nranks - 1) {
        ops.push_back({true, v + own_end - cnt, cnt, c->rank + 1});
        ops.push_back({false, v + own_end, cnt, c->rank + 1});
    }
}

static int run_local(iemic_ctx* c, const std::vector<P2P>& ops)
{
    LocalGroup* g = (LocalGroup*)c->group;
    std::map<int, int> ksend, krecv;
    for (const P2P& op : ops) {
        if (!op.send) continue;
        std::vector<double> h((size_t)op.cnt);
        int rc = d2h(c, h.data(), op.buf, sizeof(double) * h.size());
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(g->mu);
        g->box[std::make_tuple(c->rank, op.peer, ksend[op.peer]++)] = std::move(h);
    }
    g->barrier();
    for (const P2P& op : ops) {
        if (op.send) continue;
        std::vector<double> h;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            auto it = g->box.find(std::make_tuple(op.peer, c->rank, krecv[op.peer]++));
            if (it == g->box.end() || (int64_t)it->second.size() != op.cnt) {
                set_error("band group: unmatched receive");
                return IEMIC_EINVAL;
            }
            h = std::move(it->second);
            g->box.erase(it);
        }
        int rc = h2d(c, op.buf, h.data(), sizeof(double) * h.size());
        if (rc) return rc;
    }
    g->barrier();
    return 0;
}

static int run_ops(iemic_ctx* c, const std::vector<P2P>& ops)
{
    if (c->group) return run_local(c, ops);
    ncclComm_t comm = (ncclComm_t)c->comm;
    ncclResult_t first = ncclSuccess;
    std::string what;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) {
        set_error(std::string("ncclGroupStart: ") + ncclGetErrorString(r));
        return IEMIC_EDEVICE;
    }
    for (const P2P& op : ops) {
        r = op.send ? ncclSend(op.buf, (size_t)op.cnt, ncclDouble, op.peer, comm, c->stream)
                    : ncclRecv(op.buf, (size_t)op.cnt, ncclDouble, op.peer, comm, c->stream);
        if (r != ncclSuccess && first == ncclSuccess) {
            first = r;
            what = op.send ? "ncclSend" : "ncclRecv";
        }
    }
    /* the group is always closed, also after a failed enqueue, so the communicator stays
     * usable for the peers' matching calls and later collectives */
    r = ncclGroupEnd();
    if (first == ncclSuccess && r != ncclSuccess) {
        first = r;
        what = "ncclGroupEnd";
    }
    if (first != ncclSuccess) {
        set_error(what + ": " + ncclGetErrorString(first));
        return IEMIC_EDEVICE;
    }
    return 0;
}

int halo_exchange_w(iemic_ctx* c, double* v, int width, int rows_j)
{
    if (c->nranks <= 1) return 0;
    std::vector<P2P> ops;
    halo_ops(c, v, width, rows_j, ops);
    return run_ops(c, ops);
}

/* one row of two arrays of whole rows (slab doubles each; owned rows [first, first + count)),
 * e.g. the level-0 T/S multigrid iterate, in one communication group */
int halo_exchange_slab2(iemic_ctx* c, double* a, double* b, int64_t first, int64_t count, int64_t slab)
{
    if (c->nranks <= 1) return 0;
    std::vector<P2P> ops;
    for (double* v : {a, b}) {
        if (c->rank > 0) {
            ops.push_back({true, v + first, slab, c->rank - 1});
            ops.push_back({false, v + first - slab, slab, c->rank - 1});
        }
        if (c->rank < c->nranks - 1) {
            ops.push_back({true, v + first + count - slab, slab, c->rank + 1});
            ops.push_back({false, v + first + count, slab, c->rank + 1});
        }
    }
    return run_ops(c, ops);
}

/* state-vector halo (NUN doubles per cell) */
int halo_exchange(iemic_ctx* c, double* v, int rows_j) { return halo_exchange_w(c, v, NUN, rows_j); }

}  // namespace iemic
