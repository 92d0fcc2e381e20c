// CPU check of the host-buffer entry's copy workers and pinned-range registry (csrc/copy_pool.h, the
// header the library compiles): prints one JSON object for tests/test_copy_pool.py.
//   concurrent_devices  two threads stage "shards" on the pools of devices 0 and 1 at once: their
//                       task windows must overlap (each pool is its own set of workers)
//   same_pool           two threads on ONE pool take turns (a pool runs one call at a time)
//   registry            PinnedRegistry::contains on interior, edge, straddling and foreign ranges
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../indy-plenum_amd/csrc/copy_pool.h"

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

struct Window {
    double start = 1e30, end = 0;
};

// One "shard staging" of k tasks of `ms` each on `pool`; returns the window its tasks ran in.
static Window stage(pvhost::CopyPool& pool, unsigned k, int ms, clk::time_point t0) {
    std::vector<double> s(k), e(k);
    pool.run(k, [&](unsigned i) {
        s[i] = ms_since(t0);
        std::this_thread::sleep_for(std::chrono::milliseconds(ms));
        e[i] = ms_since(t0);
    });
    Window w;
    for (unsigned i = 0; i < k; i++) {
        w.start = std::min(w.start, s[i]);
        w.end = std::max(w.end, e[i]);
    }
    return w;
}

int main() {
    const unsigned k = 4;
    const int ms = 150;
    // two devices' pools, one staging thread per device (pv_verify_batch_multi_gpu's workers)
    pvhost::CopyPool& p0 = pvhost::copy_pool_for<16>(0, 2);
    pvhost::CopyPool& p1 = pvhost::copy_pool_for<16>(1, 2);
    const auto t0 = clk::now();
    Window w0, w1;
    std::thread a([&] { w0 = stage(p0, k, ms, t0); });
    std::thread b([&] { w1 = stage(p1, k, ms, t0); });
    a.join();
    b.join();
    const double wall = ms_since(t0);
    // two callers on one pool
    pvhost::CopyPool& p2 = pvhost::copy_pool_for<16>(2, 2);
    const auto t1 = clk::now();
    Window s0, s1;
    std::thread c([&] { s0 = stage(p2, k, ms, t1); });
    std::thread d([&] { s1 = stage(p2, k, ms, t1); });
    c.join();
    d.join();
    const double wall_same = ms_since(t1);
    // registry
    pvhost::PinnedRegistry r;
    static char blk[4096], blk2[256];
    r.add(blk, sizeof blk);
    r.add(blk2, sizeof blk2);
    const bool inner = r.contains(blk + 100, 1000), whole = r.contains(blk, sizeof blk),
               edge_end = r.contains(blk + sizeof blk, 0), past = r.contains(blk + 4000, 97),
               before = r.contains(blk - 1, 2), other = r.contains(blk2 + 10, 246), other_past = r.contains(blk2 + 10, 247);
    const bool removed = r.remove(blk2), gone = !r.contains(blk2, 1), twice = !r.remove(blk2);
    // pinned block cache (pv_host_free keeps blocks for the next pv_host_alloc of a similar size)
    pvhost::PinnedCache pc(1000);
    static char m1[1], m2[1], m3[1], m4[1];
    const bool pc_empty = pc.take(10).p == nullptr;
    const size_t ev0 = pc.put(m1, 400).size() + pc.put(m2, 300).size();  // 700 held
    const bool pc_small = pc.take(100).p == nullptr;        // 300 > 2 x 100: not handed out
    const bool pc_best = pc.take(250).p == m2;              // the smallest fitting block
    const bool pc_none = pc.take(500).p == nullptr;         // 400 < 500
    const size_t ev1 = pc.put(m3, 500).size();              // 900 held
    auto ev2 = pc.put(m4, 300);                             // 1200 > 1000: the oldest (m1) out
    const bool pc_evict = ev2.size() == 1 && ev2[0].p == m1 && pc.held() == 800;
    auto big = pc.put(m1, 5000);                            // larger than the budget: straight back
    const bool pc_big = big.size() == 1 && big[0].p == m1 && pc.held() == 800;
    const bool pc_drain = pc.drain().size() == 2 && pc.held() == 0 && pc.take(300).p == nullptr;
    printf("{\"pinned_cache\": {\"empty\": %d, \"no_evict\": %d, \"small\": %d, \"best\": %d, \"none\": %d, "
           "\"evict\": %d, \"big\": %d, \"drain\": %d}, ",
           pc_empty, ev0 + ev1 == 0, pc_small, pc_best, pc_none, pc_evict, pc_big, pc_drain);
    printf("\"threads_per_pool\": %u, \"pool_threads_8dev_256hw\": %u, \"pool_threads_1dev_4hw\": %u, "
           "\"concurrent_devices\": {\"w0\": [%.1f, %.1f], \"w1\": [%.1f, %.1f], \"wall_ms\": %.1f, \"task_ms\": %d, "
           "\"tasks\": %u}, \"same_pool\": {\"w0\": [%.1f, %.1f], \"w1\": [%.1f, %.1f], \"wall_ms\": %.1f}, "
           "\"registry\": {\"inner\": %d, \"whole\": %d, \"edge_end\": %d, \"past\": %d, \"before\": %d, "
           "\"other\": %d, \"other_past\": %d, \"removed\": %d, \"gone\": %d, \"twice\": %d}}\n",
           p0.threads(), pvhost::copy_pool_threads(256, 8), pvhost::copy_pool_threads(4, 1), w0.start, w0.end, w1.start,
           w1.end, wall, ms, k, s0.start, s0.end, s1.start, s1.end, wall_same, inner, whole, edge_end, past, before, other,
           other_past, removed, gone, twice);
    fflush(stdout);
    std::_Exit(0);  // the pools' threads sleep forever by design
}
