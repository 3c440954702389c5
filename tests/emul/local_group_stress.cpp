// Stress harness for the in-process rank group (i-emic_amd/csrc/local_group.h), built with
// -fsanitize=thread and with -fsanitize=address by tests/test_local_group.py: P host threads
// drive the same sequence the band contexts do (all-reduces of varying length, halo batches
// over the mailbox with several messages per peer, per-rank barriers), the owner releases
// the group while contexts are still attached, and the last context to detach deletes it.
// Every result is checked; any failure or sanitizer report makes the exit status non-zero.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../i-emic_amd/csrc/local_group.h"

using iemic::LocalGroup;

static std::atomic<int> failures{0};

static void fail(const std::string& what)
{
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    failures++;
}

static void rank_main(LocalGroup* g, int r, int P, int iters, std::atomic<LocalGroup*>* slot)
{
    std::string err;
    for (int it = 0; it < iters; it++) {
        // all-reduce: count varies per iteration (the same on every rank)
        const int count = 1 + (it * 7) % 61;
        std::vector<double> v(count), out(count);
        for (int q = 0; q < count; q++) v[q] = r * 1000.0 + q + it;
        if (g->sum(r, v.data(), out.data(), count, 30.0, err)) fail(err);
        for (int q = 0; q < count; q++) {
            const double want = 1000.0 * P * (P - 1) / 2 + P * (double)(q + it);
            if (out[q] != want) {
                fail("sum mismatch");
                break;
            }
        }
        // halo batch: 1 + it % 3 messages to each ring neighbour (both directions), as the
        // band exchanges post them: all sends, meet, all receives, meet
        const int nm = 1 + it % 3;
        const int peers[2] = {(r + 1) % P, (r + P - 1) % P};
        for (int d = 0; d < 2; d++)
            for (int k = 0; k < nm; k++) {
                std::vector<double> msg(5 + k + d, r + 0.5 * k + 0.25 * d + it);
                g->post(r, peers[d], d * nm + k, std::move(msg));
            }
        if (!g->barrier(30.0)) fail("barrier 1");
        for (int d = 0; d < 2; d++)
            for (int k = 0; k < nm; k++) {
                // the sender's direction d' is the opposite of ours: from (r - 1) it came as d = 0
                const int src = peers[1 - d], ds = d;
                std::vector<double> msg;
                if (!g->take(src, r, ds * nm + k, (size_t)(5 + k + ds), msg)) {
                    fail("unmatched receive");
                    continue;
                }
                if (msg[0] != src + 0.5 * k + 0.25 * ds + it) fail("message content");
            }
        if (!g->barrier(30.0)) fail("barrier 2");
    }
    // the owner released the group halfway; the last context to leave deletes it
    if (g->detach(r)) {
        LocalGroup* expect = g;
        if (!slot->compare_exchange_strong(expect, nullptr)) fail("group deleted twice");
        delete g;
    }
}

int main(int argc, char** argv)
{
    const int P = argc > 1 ? std::atoi(argv[1]) : 8;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 400;
    const int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
    for (int round = 0; round < rounds; round++) {
        auto* g = new LocalGroup(P);
        std::atomic<LocalGroup*> live{g};
        std::vector<std::thread> th;
        for (int r = 0; r < P; r++) g->attach(r);      // the contexts exist (iemic_create_local_2d)
        for (int r = 0; r < P; r++) th.emplace_back(rank_main, g, r, P, iters, &live);
        // the owner gives the group up while the ranks still run (iemic_local_group_free)
        if (g->release()) fail("released with contexts attached");
        for (auto& t : th) t.join();
        if (live.load() != nullptr) fail("group not deleted by the last context");
    }
    // a group released with no context attached is deleted by the owner
    {
        LocalGroup g0(2);
        if (!g0.release()) fail("release of an unused group");
    }
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures.load());
        return 1;
    }
    std::printf("local group stress ok: %d ranks x %d iterations x %d groups\n", P, iters, rounds);
    return 0;
}
