// window.cpp — the receive-side anti-replay window and the batched RX open that drives it
// (include/nebula_aead.h, "replay window + batched receive").
//
// WindowCore restates nebula.Bits (bits.go:15-262): a power-of-two circular bitmap of seen
// counters, slot 0 seeded so counter 0 reads as received (:47-48), Check (:134-150), Update with
// its fast path (:168-186) and slow path (:188-262: jump with lost accounting, in-window backfill
// or duplicate, out of window). Arithmetic is uint64 with wraparound, as in Go.
//
// neb_rx_open_batch_host is ConnectionState.Decrypt (connection_state.go:99-119) for a whole
// receive batch, with results identical to running it packet by packet in arrival order:
//   1. sequential simulation on private copies of the touched windows, assuming every tag
//      verifies: a packet the simulation refuses (replay, duplicate inside the batch, out of
//      window) is held back; the rest go to the GPU in one batch;
//   2. the real windows, in arrival order: Check, then the GPU's tag verdict, then Update — the
//      reference's order. A held-back packet whose real Check passes (possible only after an
//      earlier copy of it failed authentication) is opened right there, before the packets after it.
// Check only ever refuses more as updates accumulate, so the simulation (the real updates plus
// the ones for packets whose tag later fails) never lets through a packet the real window refuses
// unless another thread moved that window meanwhile. Statuses, window state and the lost /
// duplicate / out-of-window counters equal the sequential run; a refused packet's buffer is left
// untouched, as the reference leaves it, except in that concurrent case.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nebula_aead.h"
#include "rxwin.hpp"

// engine.cpp
bool neb_desc_in_arena(const neb_desc& d, int open, size_t arena_len);
extern "C" {  // internal (hidden), defined inside engine.cpp's extern "C" block
bool neb_rx_pipe_begin(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t n, uint32_t nchunks,
                       neb_desc** h_desc, int32_t** h_status, int* rc);
int neb_rx_pipe_submit(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t c0, uint32_t cnt,
                       uint32_t k);
int neb_rx_pipe_wait(neb_engine* e, uint32_t k);
void neb_rx_pipe_end(neb_engine* e);
int neb_engine_device_of(const neb_engine* e);
int neb_check_batch_args(neb_engine* e, int alg, uint32_t key_hint);
int neb_open_batch_count(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, const uint32_t* d_n,
                         uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, hipStream_t s);
}

namespace {

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

RxPool& rx_pool() {
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

}  // namespace

struct neb_window {
    WindowCore core;
    mutable std::mutex mu;  // ConnectionState.decryptLock (connection_state.go:100,112)
};

extern "C" {

NEB_API int neb_window_create(uint64_t length, neb_window** out) {
    if (!out) return NEB_ERR_INVALID;
    *out = nullptr;
    if (length == 0 || (length & (length - 1))) return NEB_ERR_INVALID;  // NewBits panics (bits.go:29-31)
    neb_window* w = new (std::nothrow) neb_window;
    if (!w) return NEB_ERR_INVALID;
    w->core.length = length;
    w->core.mask = length - 1;
    w->core.words.assign(length >= 64 ? length / 64 : 1, 0);
    w->core.words[0] = 1;  // no counter 0: seeded as received (bits.go:47-48)
    *out = w;
    return NEB_OK;
}

NEB_API int neb_window_destroy(neb_window* w) {
    delete w;
    return NEB_OK;
}

NEB_API int neb_window_check(neb_window* w, uint64_t counter) {
    if (!w) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(w->mu);
    return w->core.check(counter) ? 1 : 0;
}

NEB_API int neb_window_update(neb_window* w, uint64_t counter) {
    if (!w) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(w->mu);
    return w->core.update(counter) ? 1 : 0;
}

NEB_API int neb_window_state(const neb_window* w, uint64_t* current, int64_t counters[3]) {
    if (!w) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(w->mu);
    if (current) *current = w->core.current;
    if (counters) {
        counters[0] = w->core.lost;
        counters[1] = w->core.dupe;
        counters[2] = w->core.out_of_window;
    }
    return NEB_OK;
}

NEB_API int neb_window_slot(const neb_window* w, uint64_t slot) {
    if (!w) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(w->mu);
    return w->core.get(slot) ? 1 : 0;
}

NEB_API int neb_window_reset_counters(neb_window* w) {
    if (!w) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(w->mu);
    w->core.lost = w->core.dupe = w->core.out_of_window = 0;
    return NEB_OK;
}

NEB_API int neb_rx_open_batch_host(neb_engine* e, int alg, neb_window* const* windows, uint32_t nwindows,
                                   const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len,
                                   int32_t* status, uint32_t key_hint) {
    if (!e || (n && (!desc || !arena || !status || !windows))) return NEB_ERR_INVALID;
    if (n == 0) return NEB_OK;
    static const bool prof = std::getenv("NEB_RX_PROF") != nullptr;  // phase times to stderr
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    const auto t0 = now();
    RxPool& pool = rx_pool();
    // packet ranges for the per-packet phases: one (measured: spread over the pool they gained
    // nothing against the wake-ups, profiles/r2_host/rx_threads.log), the code stays range-based
    const uint32_t nr = 1;
    auto range = [&](uint32_t r) { return std::make_pair((uint64_t)n * r / nr, (uint64_t)n * (r + 1) / nr); };

    // an invalid batch is refused before any window moves or any packet is opened
    std::vector<uint8_t> bad(nr, 0);
    pool.run(nr, [&](uint32_t r) {
        const auto [i0, i1] = range(r);
        for (uint64_t i = i0; i < i1; i++)
            if (!neb_desc_in_arena(desc[i], 1, arena_len)) {
                bad[r] = 1;
                return;
            }
    });
    for (uint8_t b : bad)
        if (b) return NEB_ERR_INVALID;
    const auto ta = now();
    auto group_of = [&](const neb_desc& d) -> uint32_t {
        return (d.key_id < nwindows && windows[d.key_id]) ? d.key_id : nwindows;  // nwindows: no window
    };

    // Group by window, arrival order kept inside each (a counting sort whose ranges are counted
    // and scattered in parallel, ranges in arrival order).
    const uint32_t ng = nwindows + 1;
    std::vector<uint32_t> cnt((size_t)nr * ng, 0), start(ng + 1, 0), order(n);
    pool.run(nr, [&](uint32_t r) {
        const auto [i0, i1] = range(r);
        uint32_t* c = cnt.data() + (size_t)r * ng;
        for (uint64_t i = i0; i < i1; i++) c[group_of(desc[i])]++;
    });
    {
        uint32_t acc = 0;
        for (uint32_t g = 0; g < ng; g++) {
            start[g] = acc;
            for (uint32_t r = 0; r < nr; r++) {
                const uint32_t c = cnt[(size_t)r * ng + g];
                cnt[(size_t)r * ng + g] = acc;
                acc += c;
            }
        }
        start[ng] = acc;
    }
    pool.run(nr, [&](uint32_t r) {
        const auto [i0, i1] = range(r);
        uint32_t* c = cnt.data() + (size_t)r * ng;
        for (uint64_t i = i0; i < i1; i++) order[c[group_of(desc[i])]++] = (uint32_t)i;
    });
    const auto tb = now();
    // window groups for the per-window phases: contiguous runs of windows with about equal packets,
    // spread over the pool when the batch touches many windows (C3, 4096 tunnels: simulation 456 ->
    // 221 us, real pass 728 -> 472 us on 8 threads); one window's packets always stay on one thread
    uint32_t touched = 0;
    for (uint32_t g = 0; g < nwindows; g++) touched += start[g] != start[g + 1];
    const uint32_t nwg = touched < kRxMinWindows ? 1u
                                                  : std::max(1u, std::min(pool.size(), start[nwindows] / kRxMinPerThread));
    std::vector<uint32_t> wsplit(nwg + 1, nwindows);
    {
        wsplit[0] = 0;
        uint32_t g = 0;
        for (uint32_t t = 1; t < nwg; t++) {
            const uint64_t want = (uint64_t)start[nwindows] * t / nwg;
            while (g < nwindows && start[g + 1] <= want) g++;
            wsplit[t] = std::max(g, wsplit[t - 1]);
        }
    }

    const auto tc = now();
    // 1. simulation on a private copy of each window: which packets would the sequential receive
    //    path decrypt? (one scratch window per thread, reused window after window)
    enum : uint8_t { kToGpu, kHeld };
    std::vector<uint8_t> plan(n, kHeld);
    pool.run(nwg, [&](uint32_t t) {
        WindowCore sim;
        for (uint32_t g = wsplit[t]; g < wsplit[t + 1]; g++) {
            if (start[g] == start[g + 1]) continue;
            {
                std::lock_guard<std::mutex> lk(windows[g]->mu);
                sim = windows[g]->core;
            }
            for (uint32_t k = start[g]; k < start[g + 1]; k++) {
                const uint32_t i = order[k];
                if (sim.check(desc[i].counter)) {
                    sim.update(desc[i].counter);
                    plan[i] = kToGpu;
                }
            }
        }
    });
    const auto t1 = now();

    // 2. one GPU open for everything the simulation lets through, compacted in arrival order into
    //    the engine's pinned staging buffer (a zero-copy arena, opened on the receive stream) or
    //    a private vector (any other arena: neb_open_batch_host)
    neb_desc* h_desc = nullptr;
    int32_t* h_status = nullptr;
    int rc = NEB_OK;
    const bool piped = neb_rx_pipe_begin(e, alg, key_hint, arena, n, 1, &h_desc, &h_status, &rc);
    if (!piped && rc != NEB_OK) return rc;
    std::vector<uint32_t> sub_of(n, 0), before(nr + 1, 0);
    pool.run(nr, [&](uint32_t r) {
        const auto [i0, i1] = range(r);
        uint32_t c = 0;
        for (uint64_t i = i0; i < i1; i++) c += plan[i] == kToGpu;
        before[r + 1] = c;
    });
    for (uint32_t r = 0; r < nr; r++) before[r + 1] += before[r];
    const uint32_t ngpu = before[nr];
    std::vector<neb_desc> sub(piped ? 0 : ngpu);
    std::vector<int32_t> sub_status(piped ? 0 : ngpu, NEB_STATUS_BAD_KEY);
    neb_desc* out = piped ? h_desc : sub.data();
    pool.run(nr, [&](uint32_t r) {
        const auto [i0, i1] = range(r);
        uint32_t j = before[r];
        if (before[r + 1] - j == i1 - i0) {  // every packet of the range: one copy
            std::memcpy(out + j, desc + i0, (size_t)(i1 - i0) * sizeof(neb_desc));
            for (uint64_t i = i0; i < i1; i++) sub_of[i] = j++;
            return;
        }
        for (uint64_t i = i0; i < i1; i++)
            if (plan[i] == kToGpu) {
                sub_of[i] = j;
                out[j++] = desc[i];
            }
    });
    const int32_t* gst = piped ? h_status : sub_status.data();
    const auto ts = now();
    if (ngpu) {
        if (piped) {
            rc = neb_rx_pipe_submit(e, alg, key_hint, arena, 0, ngpu, 0);
            if (rc == NEB_OK) rc = neb_rx_pipe_wait(e, 0);
        } else {
            rc = neb_open_batch_host(e, alg, sub.data(), ngpu, arena, arena_len, sub_status.data(), key_hint);
        }
    }
    const auto td = now();
    // The verdicts are copied out of the staging statuses before the pipeline is released: gst is
    // the engine's shared pinned buffer, which the next receive call on this engine (another
    // thread) overwrites, or frees and reallocates for a larger batch, as soon as it holds rx.mu.
    std::vector<uint8_t> opened(n, 0);
    std::vector<int32_t> verd(n, NEB_STATUS_BAD_KEY);
    if (rc == NEB_OK)
        for (uint32_t i = 0; i < n; i++)
            if (plan[i] == kToGpu) {
                opened[i] = 1;
                verd[i] = gst[sub_of[i]];
            }
    if (piped) neb_rx_pipe_end(e);
    if (rc != NEB_OK) return rc;
    const auto t2 = now();

    // 3. the real windows, each in arrival order: Check → tag verdict → Update (exact_rounds: a
    //    packet held back that its window accepts is opened with the rest of its window's run)
    for (uint32_t k = start[nwindows]; k < start[nwindows + 1]; k++) status[order[k]] = NEB_STATUS_BAD_KEY;
    std::vector<ExactRun> runs;
    for (uint32_t g = 0; g < nwindows; g++)
        if (start[g] != start[g + 1]) runs.push_back({g, start[g], start[g + 1]});
    // speculative verifications (exact_rounds' later rounds): each packet's AAD and ciphertext+tag
    // copied into a private arena and opened there; pt_at[i] = its plaintext's offset in it
    std::vector<uint8_t> spec;
    std::vector<uint64_t> pt_at;
    std::vector<uint32_t> commit, zero;
    rc = exact_rounds(
        runs, nwg, [&](uint32_t k) { return desc[order[k]].counter; }, [&](uint32_t k) { return order[k]; },
        opened.data(), verd.data(), status,
        [&](uint32_t g, auto&& fn) {
            std::lock_guard<std::mutex> lk(windows[g]->mu);
            fn(windows[g]->core);
        },
        [&](const std::vector<uint32_t>& pk) -> int {
            std::vector<neb_desc> ds(pk.size());
            std::vector<int32_t> st(pk.size(), NEB_STATUS_BAD_KEY);
            for (size_t j = 0; j < pk.size(); j++) ds[j] = desc[pk[j]];
            const int r = neb_open_batch_host(e, alg, ds.data(), (uint32_t)ds.size(), arena, arena_len, st.data(),
                                              key_hint);
            if (r != NEB_OK) return r;
            for (size_t j = 0; j < pk.size(); j++) {
                opened[pk[j]] = 1;
                verd[pk[j]] = st[j];
            }
            return NEB_OK;
        },
        [&](const std::vector<uint32_t>& pk) -> int {
            std::vector<neb_desc> ds(pk.size());
            size_t total = 0;
            for (uint32_t i : pk) total += (((size_t)desc[i].aad_len + 15) & ~(size_t)15) + desc[i].len + 16 + 16;
            spec.assign(total, 0);
            pt_at.assign(n, 0);
            size_t off = 0;
            for (size_t j = 0; j < pk.size(); j++) {
                const neb_desc& d = desc[pk[j]];
                neb_desc s2 = d;
                s2.aad_off = off;
                std::memcpy(spec.data() + off, arena + d.aad_off, d.aad_len);
                off += ((size_t)d.aad_len + 15) & ~(size_t)15;
                s2.src_off = s2.dst_off = off;
                std::memcpy(spec.data() + off, arena + d.src_off, (size_t)d.len + 16);
                pt_at[pk[j]] = off;
                off += (((size_t)d.len + 16) + 15) & ~(size_t)15;
                ds[j] = s2;
            }
            std::vector<int32_t> st(pk.size(), NEB_STATUS_BAD_KEY);
            const int r = neb_open_batch_host(e, alg, ds.data(), (uint32_t)ds.size(), spec.data(), spec.size(),
                                              st.data(), key_hint);
            if (r != NEB_OK) return r;
            for (size_t j = 0; j < pk.size(); j++) {
                opened[pk[j]] = 2;
                verd[pk[j]] = st[j];
            }
            return NEB_OK;
        },
        [&](uint32_t cnt, auto&& fn) { pool.run(cnt, fn); }, &commit, &zero);
    if (rc != NEB_OK) return rc;
    for (uint32_t i : commit) std::memcpy(arena + desc[i].dst_off, spec.data() + pt_at[i], desc[i].len);
    for (uint32_t i : zero) std::memset(arena + desc[i].dst_off, 0, desc[i].len);
    if (rc != NEB_OK) return rc;
    if (prof)
        std::fprintf(stderr,
                     "rx n=%u threads %u/%u plan %.1f us (validate %.1f group %.1f split %.1f sim %.1f) stage+gpu %.1f "
                     "(submit->done %.1f) real %.1f us\n",
                     n, nr, nwg, us(t0, t1), us(t0, ta), us(ta, tb), us(tb, tc), us(tc, t1), us(t1, t2), us(ts, td),
                     us(t2, now()));
    return NEB_OK;
}

// ---- replay windows in device memory (rxwin.hip) ----------------------------------------------

}  // extern "C"

struct neb_dwindows {
    neb_engine* e = nullptr;
    neb::RxDevWin win{};
    uint8_t* mem = nullptr;
    std::mutex mu;  // one receive batch at a time on a window set
    uint8_t* ws_mem = nullptr;
    size_t ws_bytes = 0;
    neb::RxDevWs ws{};
    uint32_t ws_n = 0;
    uint32_t* h_host = nullptr;  // pinned, mapped: the finish sets it when a window needs the host
};

namespace {

#define RX_HIP(x)                               \
    do {                                        \
        if ((x) != hipSuccess) return NEB_ERR_HIP; \
    } while (0)

// Device slot w <-> a WindowCore (same length and word packing)
int dw_read(const neb_dwindows* d, uint32_t w, WindowCore& c) {
    const auto& v = d->win;
    c.length = v.length;
    c.mask = v.length - 1;
    c.words.resize(v.words);
    RX_HIP(hipMemcpy(&c.current, v.cur + w, 8, hipMemcpyDeviceToHost));
    RX_HIP(hipMemcpy(&c.lost, v.lost + w, 8, hipMemcpyDeviceToHost));
    RX_HIP(hipMemcpy(&c.dupe, v.dupe + w, 8, hipMemcpyDeviceToHost));
    RX_HIP(hipMemcpy(&c.out_of_window, v.oow + w, 8, hipMemcpyDeviceToHost));
    RX_HIP(hipMemcpy(c.words.data(), v.bits + (size_t)w * v.words, (size_t)v.words * 8, hipMemcpyDeviceToHost));
    return NEB_OK;
}
int dw_write(neb_dwindows* d, uint32_t w, const WindowCore& c) {
    const auto& v = d->win;
    const uint32_t one = 1;
    RX_HIP(hipMemcpy(v.cur + w, &c.current, 8, hipMemcpyHostToDevice));
    RX_HIP(hipMemcpy(v.lost + w, &c.lost, 8, hipMemcpyHostToDevice));
    RX_HIP(hipMemcpy(v.dupe + w, &c.dupe, 8, hipMemcpyHostToDevice));
    RX_HIP(hipMemcpy(v.oow + w, &c.out_of_window, 8, hipMemcpyHostToDevice));
    RX_HIP(hipMemcpy(v.bits + (size_t)w * v.words, c.words.data(), (size_t)v.words * 8, hipMemcpyHostToDevice));
    RX_HIP(hipMemcpy(v.present + w, &one, 4, hipMemcpyHostToDevice));
    return NEB_OK;
}

template <class T>
int d2h(std::vector<T>& h, const T* d, size_t n, hipStream_t s) {
    h.resize(n);
    if (n) RX_HIP(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    return NEB_OK;
}

}  // namespace

extern "C" {

NEB_API int neb_dwindows_create(neb_engine* e, uint32_t count, uint64_t length, neb_dwindows** out) {
    if (!e || !out || count == 0 || length == 0 || (length & (length - 1)) || length > (1ull << 24))
        return NEB_ERR_INVALID;
    *out = nullptr;
    hipSetDevice(neb_engine_device_of(e));
    neb_dwindows* d = new (std::nothrow) neb_dwindows;
    if (!d) return NEB_ERR_INVALID;
    d->e = e;
    auto& v = d->win;
    v.count = count;
    v.length = length;
    v.words = length >= 64 ? (uint32_t)(length / 64) : 1u;
    v.words_lg = 0;
    while ((1u << v.words_lg) < v.words) v.words_lg++;
    const size_t b_present = neb::rx_align((size_t)count * 4), b_word = neb::rx_align((size_t)count * 8);
    const size_t bytes = b_present + 4 * b_word + (size_t)count * v.words * 8;
    if (hipMalloc((void**)&d->mem, bytes) != hipSuccess || hipMemset(d->mem, 0, bytes) != hipSuccess) {
        if (d->mem) hipFree(d->mem);
        delete d;
        return NEB_ERR_HIP;
    }
    if (hipHostMalloc((void**)&d->h_host, sizeof(uint32_t), hipHostMallocMapped) != hipSuccess) {
        d->h_host = nullptr;
        hipFree(d->mem);
        delete d;
        return NEB_ERR_HIP;
    }
    uint8_t* m = d->mem;
    v.present = (uint32_t*)m;
    m += b_present;
    v.cur = (uint64_t*)m;
    m += b_word;
    v.lost = (int64_t*)m;
    m += b_word;
    v.dupe = (int64_t*)m;
    m += b_word;
    v.oow = (int64_t*)m;
    m += b_word;
    v.bits = (uint64_t*)m;
    *out = d;
    return NEB_OK;
}

NEB_API int neb_dwindows_destroy(neb_dwindows* d) {
    if (!d) return NEB_ERR_INVALID;
    hipSetDevice(neb_engine_device_of(d->e));
    {
        // neb_rx_open_batch returns only once its stream has run the batch, and holds d->mu
        // throughout: with the lock taken, nothing of this window set is in flight
        std::lock_guard<std::mutex> g(d->mu);
        if (d->ws_mem) hipFree(d->ws_mem);
        if (d->mem) hipFree(d->mem);
        if (d->h_host) hipHostFree(d->h_host);
    }
    delete d;
    return NEB_OK;
}

NEB_API int neb_dwindows_load(neb_dwindows* d, uint32_t idx, const neb_window* w) {
    if (!d || idx >= d->win.count) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(d->mu);
    hipSetDevice(neb_engine_device_of(d->e));
    if (!w) {
        const uint32_t zero = 0;
        RX_HIP(hipMemcpy(d->win.present + idx, &zero, 4, hipMemcpyHostToDevice));
        return NEB_OK;
    }
    WindowCore c;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        c = w->core;
    }
    if (c.length != d->win.length) return NEB_ERR_INVALID;
    return dw_write(d, idx, c);
}

NEB_API int neb_dwindows_store(neb_dwindows* d, uint32_t idx, neb_window* w) {
    if (!d || !w || idx >= d->win.count) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(d->mu);
    hipSetDevice(neb_engine_device_of(d->e));
    uint32_t present = 0;
    RX_HIP(hipMemcpy(&present, d->win.present + idx, 4, hipMemcpyDeviceToHost));
    if (!present) return NEB_ERR_INVALID;
    WindowCore c;
    const int rc = dw_read(d, idx, c);
    if (rc != NEB_OK) return rc;
    std::lock_guard<std::mutex> lk(w->mu);
    if (w->core.length != c.length) return NEB_ERR_INVALID;
    w->core = c;
    return NEB_OK;
}

NEB_API int neb_rx_open_batch(neb_engine* e, int alg, neb_dwindows* d, const neb_desc* d_desc, uint32_t n,
                              uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream) {
    if (!e || !d || d->e != e || (n && (!d_desc || !d_arena || !d_status))) return NEB_ERR_INVALID;
    int rc = neb_check_batch_args(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    std::lock_guard<std::mutex> g(d->mu);
    hipSetDevice(neb_engine_device_of(e));
    hipStream_t s = (hipStream_t)stream;
    auto& v = d->win;
    if (n > d->ws_n) {
        const size_t bytes = neb::rx_ws_layout(n, v.count, v.words, nullptr, nullptr);
        RX_HIP(hipStreamSynchronize(s));
        if (d->ws_mem) hipFree(d->ws_mem);
        d->ws_mem = nullptr;
        d->ws_n = 0;
        RX_HIP(hipMalloc((void**)&d->ws_mem, bytes));
        neb::rx_ws_layout(n, v.count, v.words, d->ws_mem, &d->ws);
        // the scratch bitmap is zeroed once here and again by each batch as it is consumed
        RX_HIP(hipMemsetAsync(d->ws.scratch, 0, ((size_t)v.count << v.words_lg) * 8, s));
        RX_HIP(hipMemsetAsync(d->ws.mixed, 0, 4, s));  // no generation is 0
        d->ws.gen = UINT32_MAX;  // the first batch clears the first-occurrence table
        d->ws_bytes = bytes;
        d->ws_n = n;
    }
    // a new generation per batch empties the first-occurrence table; cleared for real at wrap
    if (++d->ws.gen == 0) {
        RX_HIP(hipMemsetAsync(d->ws.tab_owner, 0, (size_t)8 << d->ws.tab_lg, s));
        RX_HIP(hipMemsetAsync(d->ws.tab_min, 0, (size_t)8 << d->ws.tab_lg, s));
        d->ws.gen = 1;
    }
    *d->h_host = 0;
    d->ws.need_host = d->h_host;
    const neb::RxDevWs& ws = d->ws;

    static const bool prof = std::getenv("NEB_RX_PROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    const auto t0 = now();
    // Everything is queued at once, one host read at the end: windows whose counters come within
    // 2^62 of wrapping hold all their packets back (admitted by none), and exact_rounds opens what
    // their real pass accepts in batches, like the windows where a tag failed.
    // 1. group by window, prefix maxima, first occurrences; admission for the safe windows
    RX_HIP(neb_rxdev_plan(d_desc, n, &v, &ws, d_status, s));
    const auto t1 = now();
    // 2. one open of every admitted packet (compacted by the plan)
    rc = neb_open_batch_count(e, alg, ws.sub_desc, n, ws.nsub, d_arena, ws.sub_status, key_hint, s);
    if (rc != NEB_OK) return rc;
    const auto t2 = now();
    // 3. the parallel finish of every window whose admitted packets all verified
    RX_HIP(neb_rxdev_finish(n, &v, &ws, d_status, s));
    const auto t3 = now();
    RX_HIP(hipStreamSynchronize(s));
    if (prof)
        std::fprintf(stderr, "rxdev n=%u enqueue plan %.1f, open %.1f, finish %.1f us, wait %.1f us\n", n, us(t0, t1),
                     us(t1, t2), us(t2, t3), us(t3, now()));
    // the finish flags, in pinned host memory, whether any window needs the sequential finish
    if (__atomic_load_n(d->h_host, __ATOMIC_ACQUIRE) == 0) return NEB_OK;
    std::vector<uint32_t> flag;
    if (d2h(flag, ws.wflag, v.count, s) != NEB_OK) return NEB_ERR_HIP;
    RX_HIP(hipStreamSynchronize(s));
    std::vector<uint32_t> run_w, run_i;
    std::vector<uint64_t> run_c;
    std::vector<uint8_t> adm;
    // windows' packet runs in run order (sorted by window: the runs are contiguous)
    auto runs_of = [&](const std::vector<uint32_t>& ws_list, auto&& fn) -> int {
        size_t k = 0;
        for (uint32_t w : ws_list) {
            while (k < n && run_w[k] < w) k++;
            const size_t k0 = k;
            while (k < n && run_w[k] == w) k++;
            const int r = fn(w, k0, k);
            if (r != NEB_OK) return r;
        }
        return NEB_OK;
    };
    std::vector<uint32_t> slow;
    for (uint32_t w = 0; w < v.count; w++)
        if ((flag[w] & neb::kRxTouched) && (flag[w] & (neb::kRxRisky | neb::kRxSlow))) slow.push_back(w);
    if (slow.empty()) return NEB_OK;
    // test hook: NEB_RXDEV_STRICT=1 refuses the host finish, to prove a batch ran the parallel form
    if (std::getenv("NEB_RXDEV_STRICT")) return NEB_ERR_INVALID;
    std::vector<int32_t> verdict, status;
    if (d2h(run_w, ws.run_w, n, s) || d2h(run_i, ws.run_i, n, s) || d2h(run_c, ws.run_c, n, s) ||
        d2h(adm, ws.adm, n, s) || d2h(verdict, ws.verdict, n, s) || d2h(status, d_status, n, s))
        return NEB_ERR_HIP;
    RX_HIP(hipStreamSynchronize(s));
    std::vector<ExactRun> runs;
    std::vector<WindowCore> cores(slow.size());
    std::vector<uint32_t> core_of(v.count, 0);
    rc = runs_of(slow, [&](uint32_t w, size_t k0, size_t k1) -> int {
        core_of[w] = (uint32_t)runs.size();
        runs.push_back({w, (uint32_t)k0, (uint32_t)k1});
        return dw_read(d, w, cores[core_of[w]]);
    });
    if (rc != NEB_OK) return rc;
    // speculative verifications: packets copied into a device scratch arena and opened there
    uint8_t* d_spec = nullptr;
    std::vector<neb_desc> h_desc(n);
    std::vector<uint64_t> pt_at;
    std::vector<uint32_t> commit, zero;
    RX_HIP(hipMemcpyAsync(h_desc.data(), d_desc, (size_t)n * sizeof(neb_desc), hipMemcpyDeviceToHost, s));
    RX_HIP(hipStreamSynchronize(s));
    auto run_spans = [&](const uint8_t* src, uint8_t* dst, const std::vector<neb_span>& sp) -> int {
        if (sp.empty()) return NEB_OK;
        neb_span* d_sp = nullptr;
        RX_HIP(hipMalloc((void**)&d_sp, sp.size() * sizeof(neb_span)));
        hipError_t err = hipMemcpyAsync(d_sp, sp.data(), sp.size() * sizeof(neb_span), hipMemcpyHostToDevice, s);
        if (err == hipSuccess) err = neb_rxdev_spans(src, dst, d_sp, (uint32_t)sp.size(), s);
        if (err == hipSuccess) err = hipStreamSynchronize(s);
        hipFree(d_sp);
        return err == hipSuccess ? NEB_OK : NEB_ERR_HIP;
    };
    rc = exact_rounds(
        runs, 1, [&](uint32_t k) { return run_c[k]; }, [&](uint32_t k) { return run_i[k]; }, adm.data(),
        verdict.data(), status.data(), [&](uint32_t w, auto&& fn) { fn(cores[core_of[w]]); },
        [&](const std::vector<uint32_t>& pk) -> int {  // one device open of these packets, in place
            const uint32_t cnt = (uint32_t)pk.size();
            RX_HIP(hipMemcpyAsync(ws.sub_map, pk.data(), (size_t)cnt * 4, hipMemcpyHostToDevice, s));
            RX_HIP(hipMemcpyAsync(ws.nsub, &cnt, 4, hipMemcpyHostToDevice, s));
            RX_HIP(neb_rxdev_gather(d_desc, cnt, &ws, s));
            const int r = neb_open_batch_count(e, alg, ws.sub_desc, cnt, nullptr, d_arena, ws.sub_status, key_hint, s);
            if (r != NEB_OK) return r;
            std::vector<int32_t> st(cnt);
            RX_HIP(hipMemcpyAsync(st.data(), ws.sub_status, (size_t)cnt * 4, hipMemcpyDeviceToHost, s));
            RX_HIP(hipStreamSynchronize(s));
            for (uint32_t j = 0; j < cnt; j++) {
                adm[pk[j]] = 1;
                verdict[pk[j]] = st[j];
            }
            return NEB_OK;
        },
        [&](const std::vector<uint32_t>& pk) -> int {  // out of place, into a scratch arena
            const uint32_t cnt = (uint32_t)pk.size();
            std::vector<neb_span> sp;
            std::vector<neb_desc> ds(cnt);
            pt_at.assign(n, 0);
            uint64_t off = 0;
            for (uint32_t j = 0; j < cnt; j++) {
                const neb_desc& dd = h_desc[pk[j]];
                neb_desc s2 = dd;
                s2.aad_off = off;
                sp.push_back({dd.aad_off, off, dd.aad_len, 0});
                off += ((uint64_t)dd.aad_len + 15) & ~15ull;
                s2.src_off = s2.dst_off = off;
                sp.push_back({dd.src_off, off, dd.len + 16u, 0});
                pt_at[pk[j]] = off;
                off += ((uint64_t)dd.len + 16 + 15) & ~15ull;
                ds[j] = s2;
            }
            if (d_spec) hipFree(d_spec);
            d_spec = nullptr;
            RX_HIP(hipMalloc((void**)&d_spec, off + 16));
            int r = run_spans(d_arena, d_spec, sp);
            if (r != NEB_OK) return r;
            neb_desc* d_ds = nullptr;
            int32_t* d_st = nullptr;
            RX_HIP(hipMalloc((void**)&d_ds, (size_t)cnt * sizeof(neb_desc)));
            if (hipMalloc((void**)&d_st, (size_t)cnt * 4) != hipSuccess) {
                hipFree(d_ds);
                return NEB_ERR_HIP;
            }
            std::vector<int32_t> st(cnt, NEB_STATUS_BAD_KEY);
            hipError_t err = hipMemcpyAsync(d_ds, ds.data(), (size_t)cnt * sizeof(neb_desc), hipMemcpyHostToDevice, s);
            r = err == hipSuccess ? neb_open_batch_count(e, alg, d_ds, cnt, nullptr, d_spec, d_st, key_hint, s)
                                  : NEB_ERR_HIP;
            if (r == NEB_OK && (hipMemcpyAsync(st.data(), d_st, (size_t)cnt * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                                hipStreamSynchronize(s) != hipSuccess))
                r = NEB_ERR_HIP;
            hipFree(d_ds);
            hipFree(d_st);
            if (r != NEB_OK) return r;
            for (uint32_t j = 0; j < cnt; j++) {
                adm[pk[j]] = 2;
                verdict[pk[j]] = st[j];
            }
            return NEB_OK;
        },
        [](uint32_t cnt, auto&& fn) {
            for (uint32_t j = 0; j < cnt; j++) fn(j);
        },
        &commit, &zero);
    if (rc == NEB_OK && (!commit.empty() || !zero.empty())) {
        std::vector<neb_span> back, zsp;
        for (uint32_t i : commit) back.push_back({pt_at[i], h_desc[i].dst_off, h_desc[i].len, 0});
        for (uint32_t i : zero) zsp.push_back({0, h_desc[i].dst_off, h_desc[i].len, 0});
        rc = run_spans(d_spec, d_arena, back);
        if (rc == NEB_OK) rc = run_spans(nullptr, d_arena, zsp);
    }
    if (d_spec) hipFree(d_spec);
    if (rc != NEB_OK) return rc;
    for (size_t r = 0; r < runs.size(); r++)
        if ((rc = dw_write(d, runs[r].w, cores[r])) != NEB_OK) return rc;
    if (rc != NEB_OK) return rc;
    RX_HIP(hipMemcpyAsync(d_status, status.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
    RX_HIP(hipStreamSynchronize(s));
    return NEB_OK;
}

}  // extern "C"
