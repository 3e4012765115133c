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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nebula_aead.h"

// engine.cpp
bool neb_desc_in_arena(const neb_desc& d, int open, size_t arena_len);
extern "C" {  // internal (hidden), defined inside engine.cpp's extern "C" block
bool neb_rx_pipe_begin(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t n, uint32_t nchunks,
                       neb_desc** h_desc, int32_t** h_status, int* rc);
int neb_rx_pipe_submit(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t c0, uint32_t cnt,
                       uint32_t k);
int neb_rx_pipe_wait(neb_engine* e, uint32_t k);
void neb_rx_pipe_end(neb_engine* e);
}

namespace {

// Zero-copy receive batches can be opened in up to kRxChunks pieces (NEB_RX_CHUNKS, at least
// kRxMinChunk packets each) so that the host-side window work overlaps the GPU. Measured (C2 / C3,
// 64 Ki packets, profiles/r2_host/rx_chunks.log): 1 chunk 22.8 / 15.5-17.9 GiB/s, 2 chunks 22.5 /
// 15.8, 4 chunks 21.4 / 15.0 — the window passes run slower beside the zero-copy kernels'
// host-memory traffic than they save. Default 1.
constexpr uint32_t kRxChunks = 4, kRxMinChunk = 8192, kRxDefaultChunks = 1;

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
    const auto t0 = now();
    // an invalid batch is refused before any window moves or any packet is opened
    for (uint32_t i = 0; i < n; i++)
        if (!neb_desc_in_arena(desc[i], 1, arena_len)) return NEB_ERR_INVALID;
    auto group_of = [&](const neb_desc& d) -> uint32_t {
        return (d.key_id < nwindows && windows[d.key_id]) ? d.key_id : nwindows;  // nwindows: no window
    };

    // A zero-copy arena is opened in chunks of arrival order queued on the engine's receive stream:
    // chunk k's GPU open overlaps the simulation of chunk k+1 and the real window pass of chunk
    // k-1 on this thread. The simulation is the same sequential run one batch would get, only in
    // pieces: the private window copies persist across chunks. Any other arena: one synchronous
    // neb_open_batch_host, as before.
    neb_desc* h_desc = nullptr;
    int32_t* h_status = nullptr;
    int prc = NEB_OK;
    const bool piped = neb_rx_pipe_begin(e, alg, key_hint, arena, n, kRxChunks + 1, &h_desc, &h_status, &prc);
    if (!piped && prc != NEB_OK) return prc;
    static const uint32_t nch = [] {
        const char* v = std::getenv("NEB_RX_CHUNKS");
        const int c = v ? std::atoi(v) : (int)kRxDefaultChunks;
        return (uint32_t)std::min(std::max(c, 1), (int)kRxChunks);
    }();
    uint32_t chunk = n;
    if (piped && nch > 1) {
        chunk = n / nch + 1;
        chunk = std::max(chunk, std::min(n, kRxMinChunk));
    }
    const uint32_t nchunks = (n + chunk - 1) / chunk;
    enum : uint8_t { kToGpu, kHeld };
    std::vector<uint8_t> plan(n, kHeld);
    std::vector<uint32_t> sub_of(n, 0);
    struct Chunk {
        uint32_t c0 = 0, c1 = 0, k = 0;
        std::vector<uint32_t> start, order;  // this chunk's packets grouped by window, arrival order kept
        uint32_t ngpu = 0;                   // the packets the simulation lets through
        std::vector<neb_desc> sub;           // (synchronous path) their descriptors and statuses
        std::vector<int32_t> sub_status;
        const int32_t* st = nullptr;         // their statuses once opened
        bool queued = false;
    };
    std::vector<Chunk> ch(nchunks);
    // private window copies: one per touched window when the batch is chunked (they persist from
    // chunk to chunk), else one scratch copy reused window after window
    std::vector<WindowCore> sim(nchunks > 1 ? nwindows : 0);
    std::vector<uint8_t> sim_taken(nchunks > 1 ? nwindows : 0, 0);
    WindowCore scratch;
    double us_plan = 0, us_real = 0;
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };

    auto simulate = [&](Chunk& c) -> int {
        const uint32_t m = c.c1 - c.c0;
        c.start.assign(nwindows + 2, 0);
        c.order.resize(m);
        for (uint32_t i = c.c0; i < c.c1; i++) c.start[group_of(desc[i]) + 1]++;
        for (uint32_t g = 0; g <= nwindows; g++) c.start[g + 1] += c.start[g];
        {
            std::vector<uint32_t> fill(c.start.begin(), c.start.end() - 1);
            for (uint32_t i = c.c0; i < c.c1; i++) c.order[fill[group_of(desc[i])]++] = i;
        }
        uint32_t ngpu = 0;
        for (uint32_t g = 0; g < nwindows; g++) {
            if (c.start[g] == c.start[g + 1]) continue;
            WindowCore* wp = &scratch;
            if (nchunks > 1) {
                wp = &sim[g];
                if (!sim_taken[g]) {  // a private copy, first time this batch touches the window
                    std::lock_guard<std::mutex> lk(windows[g]->mu);
                    sim[g] = windows[g]->core;
                    sim_taken[g] = 1;
                }
            } else {
                std::lock_guard<std::mutex> lk(windows[g]->mu);
                scratch = windows[g]->core;  // reuses the scratch bitmap's storage
            }
            WindowCore& w = *wp;
            for (uint32_t k = c.start[g]; k < c.start[g + 1]; k++) {
                const uint32_t i = c.order[k];
                if (w.check(desc[i].counter)) {
                    w.update(desc[i].counter);
                    plan[i] = kToGpu;
                    ngpu++;
                }
            }
        }
        c.ngpu = ngpu;
        neb_desc* out = nullptr;
        if (piped) {
            out = h_desc + c.c0;  // chunk k's slice of the pinned staging buffer
        } else {
            c.sub.resize(ngpu);
            c.sub_status.assign(ngpu, NEB_STATUS_BAD_KEY);
            out = c.sub.data();
        }
        if (ngpu == m) {
            std::memcpy(out, desc + c.c0, (size_t)m * sizeof(neb_desc));
            for (uint32_t i = c.c0; i < c.c1; i++) sub_of[i] = i - c.c0;
        } else {
            uint32_t j = 0;
            for (uint32_t i = c.c0; i < c.c1; i++)
                if (plan[i] == kToGpu) {
                    sub_of[i] = j;
                    out[j++] = desc[i];
                }
        }
        c.st = piped ? h_status + c.c0 : c.sub_status.data();
        if (ngpu && piped) {
            c.queued = true;
            return neb_rx_pipe_submit(e, alg, key_hint, arena, c.c0, ngpu, c.k);
        }
        return NEB_OK;
    };
    // the real windows, each in arrival order: Check → tag verdict → Update
    auto real = [&](Chunk& c) -> int {
        for (uint32_t k = c.start[nwindows]; k < c.start[nwindows + 1]; k++) status[c.order[k]] = NEB_STATUS_BAD_KEY;
        for (uint32_t g = 0; g < nwindows; g++) {
            if (c.start[g] == c.start[g + 1]) continue;
            neb_window* w = windows[g];
            std::unique_lock<std::mutex> lk(w->mu);
            for (uint32_t k = c.start[g]; k < c.start[g + 1]; k++) {
                const uint32_t i = c.order[k];
                const neb_desc& d = desc[i];
                if (!w->core.check(d.counter)) {
                    status[i] = NEB_STATUS_REPLAY;
                    continue;
                }
                int32_t st;
                if (plan[i] == kToGpu) {
                    st = c.st[sub_of[i]];
                } else {  // held back, yet the real window accepts it: an earlier copy failed its tag
                    lk.unlock();
                    const int rc = neb_open_batch_host(e, alg, &d, 1, arena, arena_len, &st, key_hint);
                    if (rc != NEB_OK) return rc;
                    lk.lock();
                    if (st == NEB_STATUS_OK && !w->core.check(d.counter)) {  // moved by another thread meanwhile
                        status[i] = NEB_STATUS_REPLAY;
                        continue;
                    }
                }
                if (st != NEB_STATUS_OK) {
                    status[i] = st;
                    continue;
                }
                status[i] = w->core.update(d.counter) ? NEB_STATUS_OK : NEB_STATUS_REPLAY;
            }
        }
        return NEB_OK;
    };
    // the chunk's statuses: the queued open's event, or (synchronous path) the open itself
    auto gpu_done = [&](Chunk& c) -> int {
        if (piped) return c.queued ? neb_rx_pipe_wait(e, c.k) : NEB_OK;
        if (!c.ngpu) return NEB_OK;
        return neb_open_batch_host(e, alg, c.sub.data(), c.ngpu, arena, arena_len, c.sub_status.data(), key_hint);
    };

    int rc = NEB_OK;
    for (uint32_t k = 0; k <= nchunks && rc == NEB_OK; k++) {
        if (k < nchunks) {
            const auto ta = now();
            ch[k].k = k;
            ch[k].c0 = k * chunk;
            ch[k].c1 = std::min(n, (k + 1) * chunk);
            rc = simulate(ch[k]);
            us_plan += us(ta, now());
        }
        if (k > 0 && rc == NEB_OK) {
            rc = gpu_done(ch[k - 1]);
            const auto ta = now();
            if (rc == NEB_OK) rc = real(ch[k - 1]);
            us_real += us(ta, now());
        }
    }
    if (piped) neb_rx_pipe_end(e);  // waits for anything still queued
    if (prof)
        std::fprintf(stderr, "rx n=%u chunks %u total %.1f us (sim %.1f, real %.1f on this thread)\n", n, nchunks,
                     us(t0, now()), us_plan, us_real);
    return rc;
}

}  // extern "C"
