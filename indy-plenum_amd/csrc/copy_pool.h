// Host-side copy workers of the host-buffer entry (pv_verify_batch / pv_verify_batch_multi_gpu), and
// the registry of library-owned pinned host memory (pv_host_alloc). Plain C++: no HIP, so the CPU
// tests compile this header on its own (tests/native/copy_pool_check.cpp).
//
// A CopyPool is a set of persistent threads (created on first use, so a call pays no thread
// creation). run(k, fn) executes fn(0..k-1) on the pool's threads and the calling thread and returns
// when all are done. Calls on ONE pool take turns; every device context has its own pool
// (pv_copy_pool(dev)), so the per-device workers of a multi-GPU call stage their shards at the same
// time instead of queueing on one process-wide pool.
#ifndef PV_COPY_POOL_H
#define PV_COPY_POOL_H

#include <stdint.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <iterator>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

namespace pvhost {

class CopyPool {
   public:
    explicit CopyPool(unsigned threads) : want_(threads) {}
    void run(unsigned k, const std::function<void(unsigned)>& fn) {
        if (k <= 1) {
            for (unsigned i = 0; i < k; i++) fn(i);
            return;
        }
        std::lock_guard<std::mutex> turn(run_mu_);
        if (workers() == 0) {
            for (unsigned i = 0; i < k; i++) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            next_ = 0;
            total_ = k;
            done_ = 0;
            gen_++;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return done_ == total_; });
        fn_ = nullptr;
    }
    unsigned threads() const { return want_; }

   private:
    unsigned workers() {
        if (!started_) {
            started_ = true;
            for (unsigned i = 0; i + 1 < want_; i++) th_.emplace_back([this] { loop(); });
        }
        return (unsigned)th_.size();
    }
    void drain() {  // take tasks until none is left
        for (;;) {
            unsigned i;
            const std::function<void(unsigned)>* f;
            {
                std::lock_guard<std::mutex> lk(m_);
                if (!fn_ || next_ >= total_) return;
                i = next_++;
                f = fn_;
            }
            (*f)(i);
            std::lock_guard<std::mutex> lk(m_);
            if (++done_ == total_) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
            }
            drain();
        }
    }
    const unsigned want_;
    std::mutex m_, run_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)>* fn_ = nullptr;
    unsigned next_ = 0, total_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool started_ = false;
    std::vector<std::thread> th_;
};

// Threads per device pool: one host thread copies ~23 GB/s pageable -> pinned, eight ~100 GB/s
// (MI355X box, profiles/r05/h2d_bw.txt), against ~57 GB/s of PCIe per device; at most half the host's
// hardware threads over all pools.
inline unsigned copy_pool_threads(unsigned hw, unsigned ndev) {
    hw = std::max(1u, hw);
    ndev = std::max(1u, ndev);
    return std::max(1u, std::min(8u, hw / 2 / ndev));
}

// The pool of device `dev` (0 <= dev < MAXDEV). Pools are never destroyed: their threads sleep on a
// condition variable until the process ends (a forked child, which has none of them, must not run a
// destructor that joins them).
template <int MAXDEV>
CopyPool& copy_pool_for(int dev, unsigned ndev_hint) {
    static std::mutex mu;
    static CopyPool* pools[MAXDEV] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (!pools[dev]) pools[dev] = new CopyPool(copy_pool_threads(std::thread::hardware_concurrency(), ndev_hint));
    return *pools[dev];
}

// Library-owned pinned host ranges (pv_host_alloc / pv_host_register): base -> size. contains() is
// what the host-buffer entry asks before it skips the pageable -> pinned staging copy.
class PinnedRegistry {
   public:
    void add(const void* p, uint64_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        r_[(uintptr_t)p] = bytes;
    }
    bool remove(const void* p) {
        std::lock_guard<std::mutex> lk(mu_);
        return r_.erase((uintptr_t)p) > 0;
    }
    uint64_t size_of(const void* p) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = r_.find((uintptr_t)p);
        return it == r_.end() ? 0 : it->second;
    }
    // [p, p + bytes) lies inside one registered range (bytes == 0: p inside or at the end of one)
    bool contains(const void* p, uint64_t bytes) {
        const uintptr_t a = (uintptr_t)p;
        std::lock_guard<std::mutex> lk(mu_);
        auto it = r_.upper_bound(a);
        if (it == r_.begin()) return false;
        --it;
        return a >= it->first && a - it->first <= it->second && bytes <= it->second - (a - it->first);
    }
    size_t count() {
        std::lock_guard<std::mutex> lk(mu_);
        return r_.size();
    }

   private:
    std::mutex mu_;
    std::map<uintptr_t, uint64_t> r_;
};

// Blocks released by pv_host_free, kept pinned for the next pv_host_alloc of a similar size (a node
// allocates its receive arenas again and again; a fresh pinned allocation costs ~0.1 s per 400 MB,
// and one made late in a long-lived process can land on pages the DMA engines read at half rate --
// profiles/r05/host_path/README.txt). take(bytes) returns the smallest cached block of at least
// `bytes` and at most twice that, or null; put() keeps a block and returns the blocks the total
// budget pushes out (oldest first), which the caller frees; drain() returns all of them.
class PinnedCache {
   public:
    struct Block {
        void* p;
        uint64_t bytes;
    };
    explicit PinnedCache(uint64_t budget) : budget_(budget) {}
    Block take(uint64_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        size_t best = blocks_.size();
        for (size_t i = 0; i < blocks_.size(); i++) {
            const uint64_t b = blocks_[i].bytes;
            if (b >= bytes && b / 2 <= bytes && (best == blocks_.size() || b < blocks_[best].bytes)) best = i;
        }
        if (best == blocks_.size()) return {nullptr, 0};
        const Block r = blocks_[best];
        blocks_.erase(blocks_.begin() + (long)best);
        held_ -= r.bytes;
        return r;
    }
    std::vector<Block> put(void* p, uint64_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        std::vector<Block> out;
        if (bytes > budget_) {
            out.push_back({p, bytes});
            return out;
        }
        blocks_.push_back({p, bytes});
        held_ += bytes;
        while (held_ > budget_) {
            out.push_back(blocks_.front());
            held_ -= blocks_.front().bytes;
            blocks_.erase(blocks_.begin());
        }
        return out;
    }
    std::vector<Block> drain() {
        std::lock_guard<std::mutex> lk(mu_);
        std::vector<Block> out;
        out.swap(blocks_);
        held_ = 0;
        return out;
    }
    uint64_t held() {
        std::lock_guard<std::mutex> lk(mu_);
        return held_;
    }

   private:
    std::mutex mu_;
    const uint64_t budget_;
    uint64_t held_ = 0;
    std::vector<Block> blocks_;
};

}  // namespace pvhost

#endif  // PV_COPY_POOL_H
