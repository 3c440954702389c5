/*
 * comm.hip -- halo exchanges and sums of the Decomp2D subdomains over
 * RCCL (xGMI), an in-process group (tests on one GPU) or a caller's host transport.
 *
 * Replaces the Epetra/MPI communication of the reference path: the Import of ghost cells
 * before matrix_/rhs_ and Apply (TRIOS_Domain.C Solve2Assembly, Epetra_CrsMatrix::Apply)
 * and the MPI_Allreduce inside Belos' dots and norms and THCM's intcond/forcing sums.
 * In the ext layout (stencil.h) a latitude halo is a contiguous slab of the main block
 * plus one of the x-halo block, so a y exchange goes straight from the vector; an x halo
 * is one short run per (j, k) row, packed by a 2-D copy on the stream.  An exchange runs
 * in two phases, x then y, and the y messages carry the x halo of the rows they send, so
 * the diagonal neighbours arrive too.  One rank: all calls are no-ops.
 */
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "common.h"
#include "local_group.h"

namespace iemic {

#define NCCL_OK(expr)                                                                    \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess) {                                                         \
            set_error(std::string(#expr) + ": " + ncclGetErrorString(r_));               \
            return IEMIC_EDEVICE;                                                        \
        }                                                                                \
    } while (0)

/* ---- in-process group (test facility; local_group.h) ------------------------------- */
static int host_allreduce(iemic_ctx* c, double* dev, int count)
{
    std::vector<double> h(count);
    int rc = d2h(c, h.data(), dev, sizeof(double) * count);
    if (rc) return rc;
    if (c->tp.allreduce_sum(c->tp.user, h.data(), count)) {
        set_error("host transport: allreduce failed");
        return IEMIC_EDEVICE;
    }
    return h2d(c, dev, h.data(), sizeof(double) * count);
}

static int local_allreduce(iemic_ctx* c, double* dev, int count)
{
    LocalGroup* g = (LocalGroup*)c->group;
    std::vector<double> h(count);
    int rc = d2h(c, h.data(), dev, sizeof(double) * count);
    if (rc) return rc;
    std::string err;
    if (g->sum(c->rank, h.data(), h.data(), count, c->comm_timeout_s, err)) {
        set_error(err);
        return err.find("did not arrive") != std::string::npos ? IEMIC_EDEVICE : IEMIC_EINVAL;
    }
    return h2d(c, dev, h.data(), sizeof(double) * count);
}

static int group_barrier(iemic_ctx* c, LocalGroup* g, const char* what)
{
    if (g->barrier(c->comm_timeout_s)) return 0;
    std::string err;
    LocalGroup::timed_out(err, what, c->rank, c->comm_timeout_s);
    set_error(err);
    return IEMIC_EDEVICE;
}

void* local_group_new(int nranks) { return nranks > 0 ? new LocalGroup(nranks) : nullptr; }
/* the owner gives the group up; it is deleted now, or by the last context still attached */
void local_group_free(void* g)
{
    if (g && ((LocalGroup*)g)->release()) delete (LocalGroup*)g;
}
void local_group_join(iemic_ctx* c, void* g)
{
    c->group = g;
    ((LocalGroup*)g)->attach(c->rank);
}
void local_group_leave(iemic_ctx* c)
{
    LocalGroup* g = (LocalGroup*)c->group;
    c->group = nullptr;
    if (g && g->detach(c->rank)) delete g;
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

/* the ranks the transport itself reports (RCCL: ncclCommCount) and its kind: 0 none (one
 * rank), 1 RCCL, 2 in-process group, 3 host transport (the caller's, which reports none:
 * its nranks) */
int comm_size(const iemic_ctx* c, int* size, int* kind)
{
    if (c->nranks <= 1) {
        *size = 1;
        *kind = 0;
    } else if (c->group) {
        *size = ((LocalGroup*)c->group)->P;
        *kind = 2;
    } else if (c->tp.send) {
        *size = c->nranks;
        *kind = 3;
    } else {
        int n = 0;
        NCCL_OK(ncclCommCount((ncclComm_t)c->comm, &n));
        *size = n;
        *kind = 1;
    }
    return 0;
}

/* Bounded wait for the RCCL work enqueued on the stream (or up to event e): polls the
 * stream / event and the communicator's asynchronous error; on an error or after
 * comm_timeout_s the communicator is aborted (its kernels see the abort flag and return) and
 * the call fails naming `what`.  Every host wait of an RCCL context goes through here
 * (dev_wait), so a peer that never posts a matching call -- at the first collective or at one
 * of a plan first used in the middle of a solve -- ends the call instead of hanging the
 * process.  The first 200 polls spin (the FGMRES loop waits on every iteration: no sleep
 * latency), then the poll backs off to 20 us and later 1 ms. */
static int rccl_wait(iemic_ctx* c, const std::string& what, hipEvent_t e = nullptr)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    ncclComm_t comm = (ncclComm_t)c->comm;
    for (int it = 0;; it++) {
        const hipError_t q = e ? hipEventQuery(e) : hipStreamQuery(c->stream);
        if (q == hipSuccess) return 0;
        if (q != hipErrorNotReady) {
            set_error(what + ": " + hipGetErrorString(q));
            return IEMIC_EDEVICE;
        }
        if (it < 200) {
            std::this_thread::yield();
            continue;
        }
        ncclResult_t ae = ncclSuccess;
        const bool failed = ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess &&
                            ae != ncclInProgress;
        const double dt = std::chrono::duration<double>(clk::now() - t0).count();
        if (failed || dt > c->comm_timeout_s) {
            (void)ncclCommAbort(comm);
            c->comm = nullptr;
            set_error(what + " on rank " + std::to_string(c->rank) + ": " +
                      (failed ? std::string("RCCL error ") + ncclGetErrorString(ae)
                              : "not complete after " + std::to_string(c->comm_timeout_s) +
                                    " s (a peer never posted the matching call)") +
                      "; communicator aborted");
            return IEMIC_EDEVICE;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(it < 5000 ? 20 : 1000));
    }
}

/* the host waits of the library: for the stream (e null) or an event; bounded under RCCL */
int dev_wait(iemic_ctx* c, hipEvent_t e, const char* what)
{
    if (!c->comm) {
        HIP_OK(e ? hipEventSynchronize(e) : hipStreamSynchronize(c->stream));
        return 0;
    }
    return rccl_wait(c, std::string("wait in ") + what, e);
}

static int rccl_live(iemic_ctx* c)
{
    if (c->comm) return 0;
    set_error("RCCL communicator was aborted by an earlier failure");
    return IEMIC_EDEVICE;
}

int allreduce_sum(iemic_ctx* c, double* dev, int count)
{
    if (c->nranks <= 1 || count <= 0) return 0;
    c->stat[3]++;
    if (c->group) return local_allreduce(c, dev, count);
    if (c->tp.send) return host_allreduce(c, dev, count);
    int rc = rccl_live(c);
    if (rc) return rc;
    NCCL_OK(ncclAllReduce(dev, dev, (size_t)count, ncclDouble, ncclSum, (ncclComm_t)c->comm,
                          c->stream));
    if (!(c->comm_checked & 1)) {
        c->comm_checked |= 1;
        return rccl_wait(c, "first all-reduce (" + std::to_string(count) + " doubles)");
    }
    return 0;
}

/* ---- messages ----------------------------------------------------------------------
 * Pairing rule (RCCL's, and that of the in-process mailbox and the host transport): the
 * k-th message rank a sends to rank b is the k-th message b receives from a (the plans of
 * decomp.h are built for it). */

static size_t seg_count(const Seg& g) { return (size_t)(g.nblk * g.len); }

/* strided message <-> contiguous buffer (device or host), stream-ordered */
static int seg_copy(iemic_ctx* c, const Seg& g, double* buf, bool to_buf, hipMemcpyKind kind)
{
    if (!g.nblk || !g.len) return 0;
    double* p = g.base + g.off;
    const size_t w = sizeof(double) * g.len, sp = sizeof(double) * g.stride;
    if (to_buf) HIP_OK(hipMemcpy2DAsync(buf, w, p, sp, w, g.nblk, kind, c->stream));
    else HIP_OK(hipMemcpy2DAsync(p, sp, buf, w, w, g.nblk, kind, c->stream));
    return 0;
}
static bool seg_contig(const Seg& g) { return g.nblk == 1 || g.len == g.stride; }

/* device buffers of a batch: contiguous messages straight from / into the vector, strided
 * ones in the device staging buffer, the sends packed there (stream-ordered).  Shared by
 * RCCL and the in-process group, so the packing offsets of the RCCL path run on one GPU. */
static int stage_sends(iemic_ctx* c, const std::vector<Msg>& ops, std::vector<double*>& buf)
{
    size_t tot = 0;
    for (const Msg& op : ops)
        if (!seg_contig(op.s)) tot += seg_count(op.s);
    if (c->d_stage.n < tot && c->d_stage.alloc(tot)) {
        set_error("halo exchange: out of device memory");
        return IEMIC_ENOMEM;
    }
    buf.assign(ops.size(), nullptr);
    size_t o = 0;
    int rc;
    for (size_t q = 0; q < ops.size(); q++) {
        const Msg& op = ops[q];
        if (seg_contig(op.s)) {
            buf[q] = op.s.base + op.s.off;
            continue;
        }
        buf[q] = c->d_stage.p + o;
        o += seg_count(op.s);
        if (op.send && (rc = seg_copy(c, op.s, buf[q], true, hipMemcpyDeviceToDevice))) return rc;
    }
    return 0;
}

/* the strided receives of a batch, from the staging buffer into the vector */
static int unstage_recvs(iemic_ctx* c, const std::vector<Msg>& ops, const std::vector<double*>& buf)
{
    int rc;
    for (size_t q = 0; q < ops.size(); q++) {
        const Msg& op = ops[q];
        if (!op.send && !seg_contig(op.s) && (rc = seg_copy(c, op.s, buf[q], false, hipMemcpyDeviceToDevice)))
            return rc;
    }
    return 0;
}

static int run_local(iemic_ctx* c, const std::vector<Msg>& ops)
{
    LocalGroup* g = (LocalGroup*)c->group;
    std::vector<double*> buf;
    int rc = stage_sends(c, ops, buf);
    if (rc) return rc;
    std::map<int, int> ksend, krecv;
    for (size_t q = 0; q < ops.size(); q++) {
        const Msg& op = ops[q];
        if (!op.send) continue;
        std::vector<double> h(seg_count(op.s));
        HIP_OK(hipMemcpyAsync(h.data(), buf[q], sizeof(double) * h.size(), hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        g->post(c->rank, op.peer, ksend[op.peer]++, std::move(h));
    }
    if ((rc = group_barrier(c, g, "halo batch"))) return rc;
    bool ok = true;
    for (size_t q = 0; q < ops.size() && ok; q++) {
        const Msg& op = ops[q];
        if (op.send) continue;
        std::vector<double> h;
        if (!(ok = g->take(op.peer, c->rank, krecv[op.peer]++, seg_count(op.s), h))) break;
        HIP_OK(hipMemcpyAsync(buf[q], h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
    }
    if (ok && (rc = unstage_recvs(c, ops, buf))) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    /* the second meeting also after an unmatched receive, so the peers are not left waiting */
    if ((rc = group_barrier(c, g, "halo batch"))) return rc;
    if (!ok) {
        set_error("rank group: unmatched receive on rank " + std::to_string(c->rank));
        return IEMIC_EINVAL;
    }
    return 0;
}

/* the caller's host transport: all sends (staged), all receives, wait, unpack */
static int run_host(iemic_ctx* c, const std::vector<Msg>& ops)
{
    size_t tot = 0;
    for (const Msg& op : ops) tot += seg_count(op.s);
    if (c->h_stage.size() < tot) c->h_stage.resize(tot);
    double* h = c->h_stage.data();
    size_t o = 0;
    int rc;
    for (const Msg& op : ops) {
        if (op.send && (rc = seg_copy(c, op.s, h + o, true, hipMemcpyDeviceToHost))) return rc;
        o += seg_count(op.s);
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    o = 0;
    for (const Msg& op : ops) {
        if (op.send && c->tp.send(c->tp.user, op.peer, h + o, (int64_t)seg_count(op.s))) {
            set_error("host transport: send failed");
            return IEMIC_EDEVICE;
        }
        o += seg_count(op.s);
    }
    o = 0;
    for (const Msg& op : ops) {
        if (!op.send && c->tp.recv(c->tp.user, op.peer, h + o, (int64_t)seg_count(op.s))) {
            set_error("host transport: recv failed");
            return IEMIC_EDEVICE;
        }
        o += seg_count(op.s);
    }
    if (c->tp.wait && c->tp.wait(c->tp.user)) {
        set_error("host transport: wait failed");
        return IEMIC_EDEVICE;
    }
    o = 0;
    for (const Msg& op : ops) {
        if (!op.send && (rc = seg_copy(c, op.s, h + o, false, hipMemcpyHostToDevice))) return rc;
        o += seg_count(op.s);
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

/* RCCL: one group of sends and receives on the stream between the packing and the
 * unpacking of the strided messages */
static int run_rccl(iemic_ctx* c, const std::vector<Msg>& ops)
{
    std::vector<double*> buf;
    int rc = rccl_live(c);
    if (rc) return rc;
    if ((rc = stage_sends(c, ops, buf))) return rc;
    ncclComm_t comm = (ncclComm_t)c->comm;
    ncclResult_t first = ncclSuccess;
    std::string what;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) {
        set_error(std::string("ncclGroupStart: ") + ncclGetErrorString(r));
        return IEMIC_EDEVICE;
    }
    for (size_t q = 0; q < ops.size(); q++) {
        const Msg& op = ops[q];
        const size_t cnt = seg_count(op.s);
        r = op.send ? ncclSend(buf[q], cnt, ncclDouble, op.peer, comm, c->stream)
                    : ncclRecv(buf[q], cnt, ncclDouble, op.peer, comm, c->stream);
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
    if (!(c->comm_checked & 2)) {
        c->comm_checked |= 2;
        std::string peers;
        for (const Msg& op : ops)
            peers += std::string(peers.empty() ? "" : ", ") + (op.send ? "send to " : "recv from ") +
                     std::to_string(op.peer) + " (" + std::to_string(seg_count(op.s)) + ")";
        if ((rc = rccl_wait(c, "first halo batch [" + peers + "]"))) return rc;
    }
    return unstage_recvs(c, ops, buf);
}

int run_msgs(iemic_ctx* c, const std::vector<Msg>& ops)
{
    if (c->nranks <= 1 || ops.empty()) return 0;
    c->stat[0]++;
    for (const Msg& op : ops)
        if (op.send) {
            c->stat[1]++;
            c->stat[2] += (int64_t)(sizeof(double) * seg_count(op.s));
        }
    if (c->group) return run_local(c, ops);
    if (c->tp.send) return run_host(c, ops);
    return run_rccl(c, ops);
}

/* the plan of decomp.h on this context's subdomain, as messages on v */
void halo_plan_ext(const iemic_ctx* c, double* v, int width, int depth, std::vector<Msg>& x,
                   std::vector<Msg>& y)
{
    std::vector<MsgD> px, py;
    plan_ext(c->sub, width, depth, px, py);
    for (const MsgD& q : px) x.push_back({q.send != 0, q.peer, Seg{v, q.s.off, q.s.nblk, q.s.len, q.s.stride}});
    for (const MsgD& q : py) y.push_back({q.send != 0, q.peer, Seg{v, q.s.off, q.s.nblk, q.s.len, q.s.stride}});
}

int halo_exchange_w(iemic_ctx* c, double* v, int width, int depth)
{
    if (c->nranks <= 1) return 0;
    std::vector<Msg> x, y;
    halo_plan_ext(c, v, width, depth, x, y);
    int rc = run_msgs(c, x);
    if (rc) return rc;
    return run_msgs(c, y);
}

/* halo of a component-planar vector: nplanes planes of ps doubles (one per unknown, each
 * in the ext cell order), exchanged as one x and one y batch.  RCCL sends each plane's
 * contiguous slab from the vector (one group); the host and in-process transports, whose
 * cost is per message, send the planes' slabs of a message as one strided segment (nplanes
 * blocks at stride ps) -- same plan on every rank, so the pairing rule holds */
int halo_exchange_planar(iemic_ctx* c, double* v, int nplanes, int64_t ps, int depth)
{
    if (c->nranks <= 1) return 0;
    std::vector<Msg> x0, y0, x, y;
    halo_plan_ext(c, v, 1, depth, x0, y0);
    const bool merge = c->group || c->tp.send;
    for (auto* pr : {&x0, &y0}) {
        std::vector<Msg>& out = pr == &x0 ? x : y;
        for (const Msg& m : *pr) {
            if (merge && m.s.nblk == 1) {
                Msg mm = m;
                mm.s.nblk = nplanes;
                mm.s.stride = ps;
                out.push_back(mm);
            } else {
                for (int q = 0; q < nplanes; q++) {
                    Msg mq = m;
                    mq.s.base = v + (int64_t)q * ps;
                    out.push_back(mq);
                }
            }
        }
    }
    int rc = run_msgs(c, x);
    if (rc) return rc;
    return run_msgs(c, y);
}

int comm_verify_plans(iemic_ctx* c)
{
    if (c->nranks <= 1) return 0;
    const int P = c->nranks;
    const int spec[4][2] = {{NUN, HALO}, {NUN, 1}, {1, 1}, {1, HALO}};   /* (width, depth) of the plans */
    /* per plan, per ordered pair (a -> b): message count and sum of (k + 1) * length over
     * the k-th message; the sender adds, the receiver subtracts: all zero when they pair */
    std::vector<double> t((size_t)4 * 2 * P * P, 0.0);
    for (int q = 0; q < 4; q++) {
        std::vector<MsgD> px, py;
        plan_ext(c->sub, spec[q][0], spec[q][1], px, py);
        for (const auto* ph : {&px, &py}) {
            std::map<int, int> ks, kr;
            for (const MsgD& mg : *ph) {
                const int a = mg.send ? c->rank : mg.peer, b = mg.send ? mg.peer : c->rank;
                const int k = mg.send ? ks[b]++ : kr[a]++;
                const double sg = mg.send ? 1.0 : -1.0;
                double* e = t.data() + ((size_t)q * 2 * P + a) * P + b;
                e[0] += sg;
                e[(size_t)P * P] += sg * (k + 1) * (double)(mg.s.nblk * mg.s.len);
            }
        }
    }
    DevBuf<double> d;
    if (d.alloc(t.size())) return IEMIC_ENOMEM;
    int rc = h2d(c, d.p, t.data(), sizeof(double) * t.size());
    if (!rc) rc = allreduce_sum(c, d.p, (int)t.size());
    if (!rc) rc = d2h(c, t.data(), d.p, sizeof(double) * t.size());
    if (rc) return rc;
    for (int q = 0; q < 4; q++)
        for (int a = 0; a < P; a++)
            for (int b = 0; b < P; b++) {
                const double* e = t.data() + ((size_t)q * 2 * P + a) * P + b;
                if (e[0] != 0.0 || e[(size_t)P * P] != 0.0) {
                    set_error("halo plans do not pair: rank " + std::to_string(a) + " -> rank " +
                              std::to_string(b) + " (plan width " + std::to_string(spec[q][0]) + ", depth " +
                              std::to_string(spec[q][1]) + "): sends minus receives " +
                              std::to_string((int)e[0]) + " messages");
                    return IEMIC_EINVAL;
                }
            }
    return 0;
}

/* state-vector halo (NUN doubles per cell) */
int halo_exchange(iemic_ctx* c, double* v, int depth) { return halo_exchange_w(c, v, NUN, depth); }

}  // namespace iemic
