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
#include "host_common.hpp"
#include "knobs.hpp"
#include "rxwin.hpp"
#include "hip_guard.hpp"
#include "window_core.hpp"

// engine.cpp
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
                         uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, hipStream_t s, const uint8_t* rx,
                         void* prebinned);
void* neb_sched_space_new();
void neb_sched_space_free(void* p);
int neb_rx_sched_begin(neb_engine* e, uint32_t n, void* sched, hipStream_t s, neb::SchedWs* ws, uint32_t* max_keys);
void neb_rx_sched_abort(void* sched);
}

using namespace neb_rx;


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
    DeviceGuard dg;
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
    uint32_t* h_host = nullptr;  // pinned, mapped, 2 words (RxDevWs::need_host): a window needs the host; the scan failed
    uint8_t* wire_mem = nullptr;  // neb_rx_open_wire_batch: descriptors + gate statuses
    uint32_t wire_n = 0;
    uint32_t spin_limit = neb::kRxSpinLimit;  // neb_dwindows_set_spin_limit
    void* sched = nullptr;  // mixed-key AES-GCM receives: the open's scheduler workspace (rxwin.hpp RxBin)
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
    // null-stream copies: complete before a non-blocking stream's batch reads the slot
    RX_HIP(hipStreamSynchronize(nullptr));
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
    DeviceGuard dg(neb_engine_device_of(e));
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
    if (hipMalloc((void**)&d->mem, bytes) != hipSuccess || hipMemset(d->mem, 0, bytes) != hipSuccess ||
        hipStreamSynchronize(nullptr) != hipSuccess) {
        if (d->mem) hipFree(d->mem);
        delete d;
        return NEB_ERR_HIP;
    }
    if (hipHostMalloc((void**)&d->h_host, 2 * sizeof(uint32_t), hipHostMallocMapped) != hipSuccess) {
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
    DeviceGuard dg(neb_engine_device_of(d->e));
    {
        // neb_rx_open_batch returns only once its stream has run the batch, and holds d->mu
        // throughout: with the lock taken, nothing of this window set is in flight
        std::lock_guard<std::mutex> g(d->mu);
        if (d->sched) neb_sched_space_free(d->sched);
        if (d->ws_mem) hipFree(d->ws_mem);
        if (d->wire_mem) hipFree(d->wire_mem);
        if (d->mem) hipFree(d->mem);
        if (d->h_host) hipHostFree(d->h_host);
    }
    delete d;
    return NEB_OK;
}

NEB_API int neb_dwindows_load(neb_dwindows* d, uint32_t idx, const neb_window* w) {
    if (!d || idx >= d->win.count) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(d->mu);
    DeviceGuard dg(neb_engine_device_of(d->e));
    if (!w) {
        const uint32_t zero = 0;
        RX_HIP(hipMemcpy(d->win.present + idx, &zero, 4, hipMemcpyHostToDevice));
        RX_HIP(hipStreamSynchronize(nullptr));
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

NEB_API int neb_dwindows_set_spin_limit(neb_dwindows* d, uint32_t limit) {
    if (!d) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(d->mu);
    d->spin_limit = limit;
    return NEB_OK;
}

NEB_API int neb_dwindows_store(neb_dwindows* d, uint32_t idx, neb_window* w) {
    if (!d || !w || idx >= d->win.count) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(d->mu);
    DeviceGuard dg(neb_engine_device_of(d->e));
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

}  // extern "C"

// neb_rx_open_batch with d->mu held (the wire form builds its descriptors under the same lock)
static int rx_open_batch_locked(neb_engine* e, int alg, neb_dwindows* d, const neb_desc* d_desc, uint32_t n,
                                uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream) {
    int rc = NEB_OK;
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
    if (++d->ws.gen == 0) {  // (every generation-tagged word: the table, the block granules, wrisky)
        const size_t nblk = ((size_t)d->ws_n + neb::kRxBlock - 1) / neb::kRxBlock;
        RX_HIP(hipMemsetAsync(d->ws.tab_owner, 0, (size_t)8 << d->ws.tab_lg, s));
        RX_HIP(hipMemsetAsync(d->ws.tab_min, 0, (size_t)8 << d->ws.tab_lg, s));
        RX_HIP(hipMemsetAsync(d->ws.blk_pub, 0, nblk * 3 * 8, s));
        RX_HIP(hipMemsetAsync(d->ws.wrisky, 0, (size_t)v.count * 4, s));
        d->ws.gen = 1;
    }
    d->h_host[0] = d->h_host[1] = 0;
    d->ws.need_host = d->h_host;
    d->ws.spin_limit = d->spin_limit;
    const neb::RxDevWs& ws = d->ws;

    static const bool prof = std::getenv("NEB_RX_PROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    const auto t0 = now();
    // Everything is queued at once, one host read at the end: windows whose counters come within
    // 2^62 of wrapping hold all their packets back (admitted by none), and exact_rounds opens what
    // their real pass accepts in batches, like the windows where a tag failed.
    // 0. mixed-key AES-GCM: the open's binning (sched_body.hpp) reads only the descriptors, so extra
    //    workgroups of the plan's own launches run it (rxwin.hpp RxBin): three launches off the chain.
    //    A batch large enough for sub-bins is binned by the open itself.
    void* prebinned = nullptr;
    neb::RxBin bin{};
    if (alg == NEB_ALG_AESGCM && key_hint == NEB_KEYS_MIXED && (int64_t)n < neb::knob(NEB_KNOB_SUB_BINS_FROM)) {
        if (!d->sched && !(d->sched = neb_sched_space_new())) return NEB_ERR_HIP;
        if ((rc = neb_rx_sched_begin(e, n, d->sched, s, &bin.ws, &bin.max_keys)) != NEB_OK) return rc;
        bin.on = 1;
        prebinned = d->sched;
    }
    // 1. group by window, prefix maxima, first occurrences; admission for the safe windows
    if (neb_rxdev_plan(d_desc, n, &v, &ws, d_status, &bin, s) != hipSuccess) {
        if (prebinned) neb_rx_sched_abort(prebinned);
        return NEB_ERR_HIP;
    }
    const auto t1 = now();
    // 2. one open over the batch that runs the admitted packets only (the plan's mask), writing their
    //    statuses at their arrival indices
    rc = neb_open_batch_count(e, alg, d_desc, n, nullptr, d_arena, d_status, key_hint, s, ws.adm, prebinned);
    if (rc != NEB_OK) return rc;
    const auto t2 = now();
    // 3. the verdicts into the windows, and the parallel finish of every window whose packets all verified
    RX_HIP(neb_rxdev_finish(n, &v, &ws, d_status, s));
    const auto t3 = now();
    RX_HIP(hipStreamSynchronize(s));
    if (prof)
        std::fprintf(stderr, "rxdev n=%u enqueue plan %.1f, open %.1f, finish %.1f us, wait %.1f us\n", n, us(t0, t1),
                     us(t1, t2), us(t2, t3), us(t3, now()));
    // the plan and the open flag, in pinned host memory, whether any window needs the sequential finish
    const uint32_t need = __atomic_load_n(d->h_host, __ATOMIC_ACQUIRE);
    if (__atomic_load_n(d->h_host + 1, __ATOMIC_ACQUIRE)) return NEB_ERR_HIP;  // a scan lookback timed out
    if (need == 0) return NEB_OK;
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
    if (neb::knob(NEB_KNOB_RX_STRICT)) return NEB_ERR_INVALID;
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
            const int r =
                neb_open_batch_count(e, alg, ws.sub_desc, cnt, nullptr, d_arena, ws.sub_status, key_hint, s, nullptr, nullptr);
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
            r = err == hipSuccess ? neb_open_batch_count(e, alg, d_ds, cnt, nullptr, d_spec, d_st, key_hint, s, nullptr, nullptr)
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

extern "C" {

NEB_API int neb_rx_open_batch(neb_engine* e, int alg, neb_dwindows* d, const neb_desc* d_desc, uint32_t n,
                              uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream) {
    if (!e || !d || d->e != e || (n && (!d_desc || !d_arena || !d_status))) return NEB_ERR_INVALID;
    int rc = neb_check_batch_args(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    DeviceGuard dg;
    std::lock_guard<std::mutex> g(d->mu);
    return rx_open_batch_locked(e, alg, d, d_desc, n, d_arena, d_status, key_hint, stream);
}

// readOutsidePackets' gate (neb_rx_wire_gate) on the host, then the batched receive over the
// descriptors it builds; refused packets carry an empty descriptor with no key (untouched by the
// receive) and get the gate's status.
NEB_API int neb_rx_open_wire_batch_host(neb_engine* e, int alg, neb_window* const* windows, uint32_t nwindows,
                                        const neb_rx_packet* pk, uint32_t n, uint8_t* arena, size_t arena_len,
                                        int32_t* status, uint32_t key_hint) {
    if (!e || (n && (!pk || !arena || !status || !windows))) return NEB_ERR_INVALID;
    if (n == 0) return NEB_OK;
    for (uint32_t i = 0; i < n; i++)  // every wire packet inside the arena (sums cannot wrap)
        if (pk[i].off > arena_len || neb_rx_len(pk[i]) > arena_len - pk[i].off) return NEB_ERR_INVALID;
    std::vector<neb_desc> desc(n);
    std::vector<int32_t> gate(n);
    for (uint32_t i = 0; i < n; i++) {
        neb_desc dd{pk[i].off, pk[i].off, pk[i].off, 0, 0, 0, NEB_KEYS_MIXED, 0};
        gate[i] = neb_rx_wire_gate(arena + pk[i].off, pk[i], &dd);
        if (gate[i] != NEB_STATUS_OK) dd = neb_desc{pk[i].off, pk[i].off, pk[i].off, 0, 0, 0, NEB_KEYS_MIXED, 0};
        desc[i] = dd;
    }
    const int rc = neb_rx_open_batch_host(e, alg, windows, nwindows, desc.data(), n, arena, arena_len, status, key_hint);
    if (rc != NEB_OK) return rc;
    for (uint32_t i = 0; i < n; i++)
        if (gate[i] != NEB_STATUS_OK) status[i] = gate[i];
    return NEB_OK;
}

NEB_API int neb_rx_open_wire_batch(neb_engine* e, int alg, neb_dwindows* d, const neb_rx_packet* d_pk, uint32_t n,
                                   uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream) {
    if (!e || !d || d->e != e || (n && (!d_pk || !d_arena || !d_status))) return NEB_ERR_INVALID;
    int rc = neb_check_batch_args(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    std::lock_guard<std::mutex> g(d->mu);
    DeviceGuard dg(neb_engine_device_of(e));
    hipStream_t s = (hipStream_t)stream;
    if (n > d->wire_n) {
        RX_HIP(hipStreamSynchronize(s));
        if (d->wire_mem) hipFree(d->wire_mem);
        d->wire_mem = nullptr;
        d->wire_n = 0;
        RX_HIP(hipMalloc((void**)&d->wire_mem, (size_t)n * (sizeof(neb_desc) + 4)));
        d->wire_n = n;
    }
    neb_desc* wd = (neb_desc*)d->wire_mem;
    int32_t* gate = (int32_t*)(d->wire_mem + (size_t)d->wire_n * sizeof(neb_desc));
    RX_HIP(neb_rxdev_wire(d_pk, n, d_arena, wd, gate, s));
    rc = rx_open_batch_locked(e, alg, d, wd, n, d_arena, d_status, key_hint, stream);
    if (rc != NEB_OK) return rc;
    RX_HIP(neb_rxdev_wire_fix(gate, d_status, n, s));
    RX_HIP(hipStreamSynchronize(s));
    return NEB_OK;
}

}  // extern "C"
