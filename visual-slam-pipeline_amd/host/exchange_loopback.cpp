// exchange_loopback.cpp — vs_batch_exchange_loopback (vslam_abi.h, test support): the frame-sharded
// front end's per-step record exchange (csrc/batch_exchange.h, the code vs_batch_step_dev runs over
// RCCL) run for `world` ranks inside one process, one host thread per rank, over an in-memory
// transport: per (sender, receiver) FIFO mailboxes for the ring's send / recv (RCCL matches
// point-to-point messages per peer in issue order, so FIFO order is the same pairing) and a
// two-barrier staging area for the all-gather.  Host memory only, no device: the multi-rank slot /
// peer / halo arithmetic of the C path is testable on the CPU (tests/test_batch_exchange.py) at any
// world size, which one GPU box cannot give RCCL.
#include <condition_variable>
#include <cstring>
#include <exception>
#include <new>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../csrc/batch_exchange.h"
#include "vslam_abi.h"

namespace {

struct Hub {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::deque<std::vector<uint8_t>>> box;  // [src * world + dst]
    // all-gather: staging [world] chunks, a generation barrier
    std::vector<std::vector<uint8_t>> stage;
    int arrived = 0;
    long generation = 0;
    // set by a rank that fails: every wait below also wakes on it and returns VS_ERR_IO, so no rank
    // stays blocked on a message or barrier arrival that will never come
    bool aborted = false;
    explicit Hub(int w) : world(w), box((size_t)w * w), stage(w) {}

    void abort() {
        {
            std::lock_guard<std::mutex> lk(mu);
            aborted = true;
        }
        cv.notify_all();
    }
    int barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return VS_ERR_IO;
        const long gen = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
            if (generation == gen) return VS_ERR_IO;
        }
        return 0;
    }
};

struct Loopback final : vs_bx::Transport {
    Hub& hub;
    int rank;
    Loopback(Hub& h, int r) : hub(h), rank(r) {}
    int copy(void* dst, const void* src, size_t bytes) override {
        std::memmove(dst, src, bytes);
        return 0;
    }
    int group_start() override { return 0; }  // sends are buffered: no deadlock to avoid
    int group_end() override { return 0; }
    int send(const void* buf, size_t bytes, int peer) override {
        if (peer < 0 || peer >= hub.world) return VS_ERR_ARG;
        const auto* p = static_cast<const uint8_t*>(buf);
        {
            std::lock_guard<std::mutex> lk(hub.mu);
            hub.box[(size_t)rank * hub.world + peer].emplace_back(p, p + bytes);
        }
        hub.cv.notify_all();
        return 0;
    }
    int recv(void* buf, size_t bytes, int peer) override {
        if (peer < 0 || peer >= hub.world) return VS_ERR_ARG;
        std::unique_lock<std::mutex> lk(hub.mu);
        auto& q = hub.box[(size_t)peer * hub.world + rank];
        hub.cv.wait(lk, [&] { return !q.empty() || hub.aborted; });
        if (q.empty()) return VS_ERR_IO;
        std::vector<uint8_t> m = std::move(q.front());
        q.pop_front();
        if (m.size() != bytes) return VS_ERR_ARG;  // a message of another size: mismatched pairing
        std::memcpy(buf, m.data(), bytes);
        return 0;
    }
    int all_gather(const void* src, void* dst, size_t bytes_per_rank) override {
        {
            std::lock_guard<std::mutex> lk(hub.mu);
            const auto* p = static_cast<const uint8_t*>(src);
            hub.stage[rank].assign(p, p + bytes_per_rank);
        }
        if (int rc = hub.barrier()) return rc;
        for (int r = 0; r < hub.world; r++) {
            if (hub.stage[r].size() != bytes_per_rank) return VS_ERR_ARG;
            std::memcpy(static_cast<uint8_t*>(dst) + (size_t)r * bytes_per_rank, hub.stage[r].data(), bytes_per_rank);
        }
        return hub.barrier();  // every rank has read the stage before it is reused
    }
};

}  // namespace

extern "C" int vs_batch_exchange_loopback(int world, int B, int cap, int steps, int gather, const vs_keypoint* kps_in,
                                          const float* desc_in, const int* n_in, vs_keypoint* slot0_kps,
                                          float* slot0_desc, int* slot0_n, vs_keypoint* g_kps, float* g_desc,
                                          int* g_n) {
    if (world < 1 || world > 64 || B < 1 || cap < 1 || steps < 1 || !kps_in || !desc_in || !n_in || !slot0_kps ||
        !slot0_desc || !slot0_n || (gather && (!g_kps || !g_desc || !g_n)))
        return VS_ERR_ARG;
    const size_t kb = (size_t)cap * vs_bx::kKpBytes, dfl = (size_t)cap * 256;
    Hub hub(world);
    std::vector<int> rcs(world, 0);
    auto rank_body = [&](int r) {
        // this rank's tables (zeroed: slot 0 / carry hold count 0 before the first step)
        std::vector<uint8_t> kps((size_t)(B + 1) * kb, 0), rx_k(kb, 0), carry_k(kb, 0), gk;
        std::vector<float> desc((size_t)(B + 1) * dfl, 0.f), rx_d(dfl, 0.f), carry_d(dfl, 0.f), gd;
        std::vector<int> n(B + 1, 0), gn;
        int rx_n = 0, carry_n = 0;
        if (gather) {
            gk.assign((size_t)world * B * kb, 0);
            gd.assign((size_t)world * B * dfl, 0.f);
            gn.assign((size_t)world * B, 0);
        }
        vs_bx::Tables t;
        t.B = B, t.cap = cap, t.rank = r, t.world = world, t.gather = gather != 0;
        t.kps = kps.data(), t.desc = desc.data(), t.n = n.data();
        t.g_kps = gather ? gk.data() : nullptr, t.g_desc = gather ? gd.data() : nullptr, t.g_n = gather ? gn.data() : nullptr;
        t.rx_kps = rx_k.data(), t.rx_desc = rx_d.data(), t.rx_n = &rx_n;
        t.carry_kps = carry_k.data(), t.carry_desc = carry_d.data(), t.carry_n = &carry_n;
        Loopback x(hub, r);
        for (int st = 0; st < steps; st++) {
            // slots 1..B <- the step's frames of this rank (global frame r * B + b)
            const size_t f0 = ((size_t)st * world + r) * B;
            std::memcpy(t.kps_slot(1), reinterpret_cast<const uint8_t*>(kps_in) + f0 * kb, (size_t)B * kb);
            std::memcpy(t.desc_slot(1), desc_in + f0 * dfl, (size_t)B * dfl * sizeof(float));
            std::memcpy(t.n + 1, n_in + f0, (size_t)B * sizeof(int));
            const int rc = vs_bx::exchange(t, x);
            if (rc != 0) {
                rcs[r] = rc;
                hub.abort();  // wakes the ranks blocked in recv / barrier: they return VS_ERR_IO
                return;
            }
            const size_t o = (size_t)st * world + r;
            std::memcpy(reinterpret_cast<uint8_t*>(slot0_kps) + o * kb, t.kps_slot(0), kb);
            std::memcpy(slot0_desc + o * dfl, t.desc_slot(0), dfl * sizeof(float));
            slot0_n[o] = t.n[0];
            if (gather) {
                std::memcpy(reinterpret_cast<uint8_t*>(g_kps) + o * world * B * kb, gk.data(), gk.size());
                std::memcpy(g_desc + o * world * B * dfl, gd.data(), gd.size() * sizeof(float));
                std::memcpy(g_n + o * world * B, gn.data(), gn.size() * sizeof(int));
            }
        }
    };
    // no exception crosses the C ABI: a rank that throws (allocation of its tables) records the error
    // and aborts the hub like a failing exchange
    auto rank_main = [&](int r) {
        try {
            rank_body(r);
        } catch (const std::bad_alloc&) {
            rcs[r] = VS_ERR_NOMEM;
            hub.abort();
        } catch (...) {
            rcs[r] = VS_ERR_IO;
            hub.abort();
        }
    };
    std::vector<std::thread> th;
    try {
        th.reserve(world);
        for (int r = 0; r < world; r++) th.emplace_back(rank_main, r);
    } catch (...) {  // thread creation failed: release the ranks already started, then report
        hub.abort();
        for (auto& t : th) t.join();
        return VS_ERR_NOMEM;
    }
    for (auto& t : th) t.join();
    // the first failure is the cause; VS_ERR_IO from the ranks it woke is the consequence
    for (int rc : rcs)
        if (rc != 0 && rc != VS_ERR_IO) return rc;
    for (int rc : rcs)
        if (rc != 0) return rc;
    return VS_OK;
}
