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
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nebula_aead.h"

bool neb_desc_in_arena(const neb_desc& d, int open, size_t arena_len);  // engine.cpp

namespace {

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
    // an invalid batch is refused before any window moves or any packet is opened
    for (uint32_t i = 0; i < n; i++)
        if (!neb_desc_in_arena(desc[i], 1, arena_len)) return NEB_ERR_INVALID;
    // Windows are independent: group the batch by window (stable, so each window sees its packets
    // in arrival order) and run each window's sequence under one lock acquisition.
    std::vector<uint32_t> start(nwindows + 2, 0), order(n);
    auto group_of = [&](const neb_desc& d) -> uint32_t {
        return (d.key_id < nwindows && windows[d.key_id]) ? d.key_id : nwindows;  // nwindows: no window
    };
    for (uint32_t i = 0; i < n; i++) start[group_of(desc[i]) + 1]++;
    for (uint32_t g = 0; g <= nwindows; g++) start[g + 1] += start[g];
    {
        std::vector<uint32_t> fill(start.begin(), start.end() - 1);
        for (uint32_t i = 0; i < n; i++) order[fill[group_of(desc[i])]++] = i;
    }
    enum : uint8_t { kToGpu, kHeld };
    std::vector<uint8_t> plan(n, kHeld);
    std::vector<neb_desc> sub;
    std::vector<uint32_t> sub_of(n, 0);
    sub.reserve(n);

    // 1. simulation on a private copy of each window: which packets would the sequential receive
    //    path decrypt? (the GPU batch keeps arrival order inside each window's run)
    WindowCore sim;
    for (uint32_t g = 0; g < nwindows; g++) {
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
    for (uint32_t i = 0; i < n; i++)
        if (plan[i] == kToGpu) {
            sub_of[i] = (uint32_t)sub.size();
            sub.push_back(desc[i]);
        }

    // 2. one GPU open for everything the simulation lets through
    std::vector<int32_t> sub_status(sub.size(), NEB_STATUS_BAD_KEY);
    if (!sub.empty()) {
        const int rc = neb_open_batch_host(e, alg, sub.data(), (uint32_t)sub.size(), arena, arena_len,
                                           sub_status.data(), key_hint);
        if (rc != NEB_OK) return rc;
    }

    // 3. the real windows, each in arrival order: Check → tag verdict → Update
    for (uint32_t k = start[nwindows]; k < start[nwindows + 1]; k++) status[order[k]] = NEB_STATUS_BAD_KEY;
    for (uint32_t g = 0; g < nwindows; g++) {
        if (start[g] == start[g + 1]) continue;
        neb_window* w = windows[g];
        std::unique_lock<std::mutex> lk(w->mu);
        for (uint32_t k = start[g]; k < start[g + 1]; k++) {
            const uint32_t i = order[k];
            const neb_desc& d = desc[i];
            if (!w->core.check(d.counter)) {
                status[i] = NEB_STATUS_REPLAY;
                continue;
            }
            int32_t st;
            if (plan[i] == kToGpu) {
                st = sub_status[sub_of[i]];
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
}

}  // extern "C"
