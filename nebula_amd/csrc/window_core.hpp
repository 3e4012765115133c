// window_core.hpp — the host-side receive logic of window.cpp that needs no device: Nebula's
// anti-replay window (WindowCore, a restatement of bits.go:15-262), the exact receive order over
// window runs (exact_rounds), and the small thread pool the batched receive spreads windows over
// (RxPool). Header-only so the sanitizer builds (tests/sanitize/, `make -C nebula_amd sanitize`)
// compile exactly this code without HIP.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nebula_aead.h"

namespace neb_rx {

// The batched receive's window simulation and real window pass run on a small persistent pool
// when a batch touches at least kRxMinWindows windows: windows are independent, and each window's
// packets stay on one thread, in arrival order. NEB_RX_THREADS sets the pool size (1 = this
// thread only). Groups under kRxMinPerThread packets are not split.
constexpr uint32_t kRxMinPerThread = 2048, kRxMinWindows = 64, kRxMaxThreads = 8;

class RxPool {
  public:
    explicit RxPool(uint32_t nthreads) {
        for (uint32_t t = 1; t < nthreads; t++) th_.emplace_back([this] { loop(); });
    }
    ~RxPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    uint32_t size() const { return (uint32_t)th_.size() + 1; }
    // fn(j) for j in [0, n), on the pool and this thread; returns when every call has returned.
    // Calls from several threads at once run one after another.
    void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
        if (n <= 1 || th_.empty()) {
            for (uint32_t j = 0; j < n; j++) fn(j);
            return;
        }
        std::lock_guard<std::mutex> serial(run_mu_);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            njobs_ = n;
            next_.store(0);
            left_ = n;
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [&] { return left_ == 0 && active_ == 0; });
        job_ = nullptr;
    }

  private:
    void work() {
        for (;;) {
            const uint32_t j = next_.fetch_add(1);
            if (j >= njobs_) return;
            (*job_)(j);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return quit_ || (gen_ != seen && job_); });
                if (quit_) return;
                seen = gen_;
                active_++;
            }
            work();
            std::lock_guard<std::mutex> g(m_);
            if (--active_ == 0 && left_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_, run_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    uint32_t njobs_ = 0, left_ = 0, active_ = 0;
    std::atomic<uint32_t> next_{0};
    uint64_t gen_ = 0;
    bool quit_ = false;
};

inline RxPool& rx_pool() {
    static RxPool pool([] {
        const char* v = std::getenv("NEB_RX_THREADS");
        int t = v ? std::atoi(v) : (int)std::min(kRxMaxThreads, std::max(1u, std::thread::hardware_concurrency()));
        return (uint32_t)std::max(1, std::min(t, 64));
    }());
    return pool;
}

struct WindowCore {
    uint64_t length = 0, mask = 0, current = 0;
    std::vector<uint64_t> words;
    int64_t lost = 0, dupe = 0, out_of_window = 0;

    bool get(uint64_t i) const {
        const uint64_t p = i & mask;
        return (words[p >> 6] >> (p & 63)) & 1u;
    }
    void set(uint64_t i) {
        const uint64_t p = i & mask;
        words[p >> 6] |= 1ull << (p & 63);
    }
    // clear `count` circular slots from slot `start`; returns how many were set (bits.go:63-118)
    uint64_t clear_range(uint64_t start, uint64_t count) {
        uint64_t was = 0;
        if (count >= length) {
            for (uint64_t& w : words) {
                was += (uint64_t)__builtin_popcountll(w);
                w = 0;
            }
            return was;
        }
        uint64_t pos = start, rem = count;
        while (rem) {
            const uint64_t b = pos & 63;
            const uint64_t take = std::min({64 - b, rem, length - pos});
            const uint64_t m = take == 64 ? ~0ull : ((1ull << take) - 1) << b;
            uint64_t& w = words[pos >> 6];
            was += (uint64_t)__builtin_popcountll(w & m);
            w &= ~m;
            rem -= take;
            pos = (pos + take) & mask;
        }
        return was;
    }
    bool strictly_within(uint64_t i) const {  // bits.go:120-132
        if (i < length && current < length) return true;
        return i > current - length;
    }
    bool check(uint64_t i) const {  // bits.go:134-150
        if (i > current) return true;
        if (strictly_within(i)) return !get(i);
        return false;
    }
    bool update(uint64_t i) {  // bits.go:168-262
        if (i == current + 1) {
            if (i > length && !get(i)) lost++;
            set(i);
            current = i;
            return true;
        }
        if (i > current) {
            const uint64_t top = current + length;
            const uint64_t end = i > top ? top : i;
            const uint64_t count = end - current;
            const uint64_t start = (current + 1) & mask;
            int64_t l = 0;
            if (current >= length) {
                l = (int64_t)count - (int64_t)clear_range(start, count);
            } else {  // warmup: the first window, taken at most once per connection
                for (uint64_t n = current + 1; n <= end; n++)
                    if (!get(n) && n > length) l++;
                clear_range(start, count);
            }
            if (i > top) l += (int64_t)(i - current - length);
            lost += l;
            set(i);
            current = i;
            return true;
        }
        if (strictly_within(i)) {
            if (current == i || get(i)) {
                dupe++;
                return false;
            }
            set(i);
            return true;
        }
        out_of_window++;
        return false;
    }
};

// The exact receive order for some windows' packet runs: Check → tag verdict → Update, packet
// after packet in arrival order (connection_state.go:99-119). A packet not opened yet that its
// window now accepts — an earlier copy of it failed its tag, or a forged counter further ahead held
// it back in the simulation — stops its window there, and the stopped windows' remaining packets
// are opened in one more batch:
//   * first extra round: the rest of each stopped window's run is simulated again from the real
//     state (tags already known to fail skipped, unknown ones assumed to verify) and what the
//     simulation admits is opened in place (the simulation applies a superset of the real
//     updates, so the real pass never refuses such a packet, barring another thread moving the
//     window meanwhile);
//   * any later round: every packet still unopened in the stopped runs is verified speculatively,
//     out of place (spec_fn: plaintext into a scratch copy, the arena untouched); the real pass
//     then knows every verdict and finishes without stopping. The packets it accepts get their
//     plaintext copied into the arena (*commit), those that pass their window but fail their tag
//     get their payload zeroed (*zero), as an in-place open would, and refused ones stay untouched.
// Interleaved forgeries (F1, P1, F2, P2, ...: each forged far-ahead counter holds back the genuine
// packets after it) therefore cost at most two extra batches, not one per forgery.
// opened[i]: 0 = not yet, 1 = opened in place, 2 = verified speculatively.
struct ExactRun {
    uint32_t w, k0, k1;  // window, run positions [k0, k1)
};
template <class Ctr, class Pkt, class WithWin, class OpenFn, class SpecFn, class Par>
int exact_rounds(const std::vector<ExactRun>& runs, uint32_t max_groups, Ctr&& ctr, Pkt&& pkt, uint8_t* opened,
                 int32_t* verd, int32_t* status, WithWin&& with_window, OpenFn&& open_fn, SpecFn&& spec_fn,
                 Par&& par, std::vector<uint32_t>* commit, std::vector<uint32_t>* zero) {
    const bool stats = std::getenv("NEB_RX_STATS") != nullptr;  // rounds and opens to stderr (per call)
    uint32_t rounds = 0, extra_opens = 0, extra_pkts = 0;
    std::vector<uint32_t> pos(runs.size());
    std::vector<uint32_t> active(runs.size());
    for (size_t r = 0; r < runs.size(); r++) {
        pos[r] = runs[r].k0;
        active[r] = (uint32_t)r;
    }
    const uint32_t ng = std::max(1u, std::min(max_groups, (uint32_t)runs.size()));
    std::vector<std::vector<uint32_t>> cm(ng), zr(ng);  // per group: packets to commit / zero
    while (!active.empty()) {
        const uint32_t na = std::max(1u, std::min(ng, (uint32_t)active.size()));
        const bool speculative = extra_opens >= 1;  // the second extra round verifies everything left
        std::vector<std::vector<uint32_t>> want(na);
        par(na, [&](uint32_t gi) {
            const size_t a0 = active.size() * gi / na, a1 = active.size() * (gi + 1) / na;
            for (size_t a = a0; a < a1; a++) {
                const uint32_t r = active[a];
                const ExactRun& R = runs[r];
                with_window(R.w, [&](WindowCore& core) {
                    uint32_t k = pos[r];
                    for (; k < R.k1; k++) {
                        const uint32_t i = pkt(k);
                        const uint64_t c = ctr(k);
                        if (!core.check(c)) {
                            status[i] = NEB_STATUS_REPLAY;
                            continue;
                        }
                        if (!opened[i]) {
                            if (speculative) {
                                for (uint32_t k2 = k; k2 < R.k1; k2++)
                                    if (!opened[pkt(k2)]) want[gi].push_back(pkt(k2));
                                break;
                            }
                            WindowCore sim = core;
                            for (uint32_t k2 = k; k2 < R.k1; k2++) {
                                const uint32_t i2 = pkt(k2);
                                if (opened[i2] && verd[i2] != NEB_STATUS_OK) continue;  // known to fail
                                if (sim.check(ctr(k2))) {
                                    sim.update(ctr(k2));
                                    if (!opened[i2]) want[gi].push_back(i2);
                                }
                            }
                            break;
                        }
                        if (verd[i] != NEB_STATUS_OK) {
                            status[i] = verd[i];
                            if (opened[i] == 2 && verd[i] == NEB_STATUS_AUTH_FAILED) zr[gi].push_back(i);
                            continue;
                        }
                        const bool ok = core.update(c);
                        status[i] = ok ? NEB_STATUS_OK : NEB_STATUS_REPLAY;
                        if (ok && opened[i] == 2) cm[gi].push_back(i);
                    }
                    pos[r] = k;
                });
            }
        });
        std::vector<uint32_t> all, next;
        for (auto& v : want) all.insert(all.end(), v.begin(), v.end());
        for (uint32_t r : active)
            if (pos[r] < runs[r].k1) next.push_back(r);
        if (!all.empty()) {
            // sets opened[] (1 in place, 2 speculative) and the verdicts of these packets
            const int rc = speculative ? spec_fn(all) : open_fn(all);
            if (rc != NEB_OK) return rc;
            extra_opens++;
            extra_pkts += (uint32_t)all.size();
        }
        active.swap(next);
        rounds++;
    }
    for (uint32_t g = 0; g < ng; g++) {
        commit->insert(commit->end(), cm[g].begin(), cm[g].end());
        zero->insert(zero->end(), zr[g].begin(), zr[g].end());
    }
    if (stats)
        std::fprintf(stderr, "rx exact: %zu windows, %u rounds, %u extra opens of %u packets\n", runs.size(), rounds,
                     extra_opens, extra_pkts);
    return NEB_OK;
}

}  // namespace neb_rx
