/*
 * local_group.h -- the in-process rank group (test facility of comm.hip): several band
 * contexts of one problem in one process, one host thread each (on one GPU, where RCCL
 * refuses duplicate devices).  Plain C++ with no HIP dependency, so the same code is built
 * into a CPU harness under ThreadSanitizer / AddressSanitizer (tests/emul/local_group_stress.cpp).
 *
 * Collectives are host-staged: an all-reduce writes each rank's slot, meets at a reusable
 * barrier, sums the slots in rank order (results do not depend on thread timing) and meets
 * again before any slot is reused; a halo batch posts its messages into a mailbox keyed by
 * (source, destination, k) -- the k-th message a sends to b is the k-th b receives from a --
 * meets, takes its receives and meets again.
 *
 * Lifetime: the group is freed by whoever created it, but only once no context is attached
 * (release() by the owner marks it orphaned; the last context to leave deletes it), so a
 * context can never wait on a freed barrier.
 */
#ifndef IEMIC_LOCAL_GROUP_H
#define IEMIC_LOCAL_GROUP_H

#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace iemic {

class LocalGroup {
public:
    explicit LocalGroup(int p) : P(p), slot_(p), attached_(p, 0) {}
    const int P;

    /* false when the other ranks did not all arrive within timeout_s (the caller withdraws
     * and reports; the group is unusable afterwards, as a communicator after an abort) */
    bool barrier(double timeout_s)
    {
        std::unique_lock<std::mutex> lk(mu_);
        const long gen = generation_;
        if (++arrived_ == P) {
            arrived_ = 0;
            generation_++;
            cv_.notify_all();
            return true;
        }
        if (cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return generation_ != gen; }))
            return true;
        arrived_--;
        return false;
    }

    /* out[0 .. count) = sum over the ranks of their in[] (rank order); 0, or 1 with err set */
    int sum(int rank, const double* in, double* out, int count, double timeout_s, std::string& err)
    {
        {
            /* own slot only: every other rank finished reading it before the barrier that
             * ended the previous sum */
            std::vector<double>& mine = slot_[rank];
            mine.assign(in, in + count);
        }
        if (!barrier(timeout_s)) return timed_out(err, "all-reduce", rank, timeout_s);
        std::vector<double> s((size_t)count, 0.0);
        for (int r = 0; r < P; r++) {
            const std::vector<double>& v = slot_[r];
            if (v.size() != (size_t)count) {
                err = "rank group: all-reduce of " + std::to_string(count) + " doubles on rank " +
                      std::to_string(rank) + ", " + std::to_string(v.size()) + " on rank " + std::to_string(r);
                /* still meet the second barrier, so the peers are not left waiting */
                barrier(timeout_s);
                return 1;
            }
            for (int q = 0; q < count; q++) s[q] += v[q];
        }
        if (!barrier(timeout_s)) return timed_out(err, "all-reduce", rank, timeout_s);
        for (int q = 0; q < count; q++) out[q] = s[q];
        return 0;
    }

    /* message k from src to dst of the current batch */
    void post(int src, int dst, int k, std::vector<double>&& data)
    {
        std::lock_guard<std::mutex> lk(mu_);
        box_[std::make_tuple(src, dst, k)] = std::move(data);
    }
    /* takes message k from src to dst (expected length n); false if absent or of another length */
    bool take(int src, int dst, int k, size_t n, std::vector<double>& out)
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = box_.find(std::make_tuple(src, dst, k));
        if (it == box_.end() || it->second.size() != n) return false;
        out = std::move(it->second);
        box_.erase(it);
        return true;
    }
    /* messages posted and not taken (a batch whose plans do not pair leaves some behind) */
    size_t pending()
    {
        std::lock_guard<std::mutex> lk(mu_);
        return box_.size();
    }

    static int timed_out(std::string& err, const char* what, int rank, double timeout_s)
    {
        err = std::string("rank group: ") + what + " on rank " + std::to_string(rank) +
              ": the other ranks did not arrive within " + std::to_string(timeout_s) +
              " s (a rank skipped the collective or its exchange plan differs)";
        return 1;
    }

    /* attach / detach a rank's context; release: the owner gives the group up.  Returns true
     * when the caller must delete the group (no context attached and released) */
    void attach(int rank)
    {
        std::lock_guard<std::mutex> lk(mu_);
        attached_[rank]++;
    }
    bool detach(int rank)
    {
        std::lock_guard<std::mutex> lk(mu_);
        attached_[rank]--;
        return released_ && none_attached();
    }
    bool release()
    {
        std::lock_guard<std::mutex> lk(mu_);
        released_ = true;
        return none_attached();
    }

private:
    bool none_attached() const
    {
        for (int a : attached_)
            if (a) return false;
        return true;
    }
    std::mutex mu_;
    std::condition_variable cv_;
    int arrived_ = 0;
    long generation_ = 0;
    std::vector<std::vector<double>> slot_;
    std::map<std::tuple<int, int, int>, std::vector<double>> box_;
    std::vector<int> attached_;
    bool released_ = false;
};

}  // namespace iemic

#endif
