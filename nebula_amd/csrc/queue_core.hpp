// queue_core.hpp — the submission queue's batching state machine (include/nebula_aead.h,
// "submission queue"), independent of the device: queue.cpp instantiates it over the engine, the
// sanitizer tests (tests/sanitize/queue_test.cpp, ASan/UBSan and TSan builds) over a CPU device.
//
// Nebula seals at most 128 packets per TX flush (overlay/batch/tx_batch.go:5, interface.go:465-469)
// and opens at most listen.batch = 64 per RX flush (main.go:181, interface.go:395-400), from
// `routines` goroutines at once (interface.go:320-335). A device batch only pays for itself at
// thousands of packets, so submit() lets every routine hand over its flush as is: the packets are
// copied into staging, joined with the other routines' flushes into one batch, sealed or opened by
// one device launch, and copied back; the call returns when its own packets are done, with the same
// arena bytes and statuses as neb_seal_batch_host / neb_open_batch_host.
//
// A batch goes to the device when it reaches max_packets, when the next submission would not fit
// its staging, when flush() asks, or max_delay_us after its first submission. `depth` staging
// batches rotate: one filling, the others on the device or being copied out.
//
// Zero-copy submissions: when the caller's arena is pinned, mapped host memory (neb_host_alloc,
// Dev::mapped), only its descriptors are staged. They point at the caller's arena itself — every
// descriptor offset of a batch is relative to the batch's staging base, as a wrapping 64-bit
// offset for a caller's arena — so the kernels read and write the caller's bytes in place, as the
// zero-copy neb_*_batch_host does, and only the statuses are copied back.
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nebula_aead.h"
#include "host_common.hpp"


namespace neb_q {

using Clock = std::chrono::steady_clock;

enum class BState { kFree, kFilling, kSealed, kLaunched, kDone };

template <class Tok>
struct QBatch {
    // pinned, mapped staging: the kernels read and write it in place
    uint8_t* arena = nullptr;
    neb_desc* desc = nullptr;
    int32_t* status = nullptr;
    Tok tok{};  // the device's completion marker
    BState state = BState::kFree;
    uint32_t npk = 0, subs = 0, writers = 0, readers = 0;
    size_t used = 0;
    uint32_t key0 = NEB_KEYS_MIXED;  // the one key every packet uses so far, or NEB_KEYS_MIXED
    bool one_key = true;
    Clock::time_point first{}, sealed_at{}, launched_at{};
    int rc = NEB_OK;
};

size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

// staging bytes one packet takes: AAD, the source (payload, + tag when opening), and a separate
// destination when the descriptor is not in place
size_t staged_bytes(const neb_desc& d, int open) {
    const size_t src = (size_t)d.len + (open ? 16u : 0u), dst = (size_t)d.len + (open ? 0u : 16u);
    const size_t in_place = d.src_off == d.dst_off ? 0 : up16(dst);
    return up16(d.aad_len) + up16(std::max(src, dst)) + in_place;
}

// defaults and limits of a neb_queue_config; false = out of range
inline bool normalize(neb_queue_config& c) {
    if (c.max_packets == 0) c.max_packets = 16384;
    if (c.max_delay_us == 0) c.max_delay_us = 100;
    if (c.arena_bytes == 0) c.arena_bytes = (uint64_t)c.max_packets * 1536;
    if (c.depth == 0) c.depth = 3;
    return c.depth >= 2 && c.depth <= 16 && c.max_packets <= (1u << 22) && c.arena_bytes <= (1ull << 36);
}

// The queue's state machine over a device policy Dev:
//   Dev::Token                               a completion marker per staging batch
//   int  launch(i, desc, n, arena, status, key_hint, Token&)  queue staging batch i (in launch
//                                            order; batches may run concurrently on the device)
//   int  wait(Token&)                        block until that batch is done and visible
//   bool key_ok(key)                         the key is installed for the queue's algorithm
//   bool mapped(arena)                       the kernels can address the arena in place
// queue.cpp binds it to the engine (zero-copy kernels on pinned staging, HIP events); the
// sanitizer tests (tests/sanitize/queue_test.cpp) to a CPU device running the oracle.
template <class Dev>
struct Queue {
    using Batch = QBatch<typename Dev::Token>;
    Dev dev;
    int open = 0;
    neb_queue_config cfg{};
    std::vector<Batch> b;
    uint32_t cur = 0;          // the batch accepting submissions
    uint32_t next_launch = 0;  // batches launch and complete in ring order
    std::mutex mu;
    std::condition_variable cv;   // submitters: a batch became free or done
    std::condition_variable fcv;  // the flusher: a batch has work / was sealed / writers finished
    bool flush_req = false, quit = false;
    std::thread flusher, completer;
    uint64_t n_batches = 0, n_packets = 0, n_subs = 0, n_bytes = 0, n_zc = 0;
    // phase times (ns, summed; neb_queue_phases): per batch fill (first submission -> sealed),
    // drain (sealed -> launched: the last writers' copy-in and the flusher's wake-up) and device
    // (launched -> done: the launch and the kernel); per submission copy-in, wait (copy-in done ->
    // its batch done) and copy-out
    uint64_t ns_fill = 0, ns_drain = 0, ns_device = 0, ns_copy_in = 0, ns_wait = 0, ns_copy_out = 0;
    static uint64_t ns_between(Clock::time_point a, Clock::time_point b) {
        return b > a ? (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count() : 0u;
    }

    // seal the filling batch and move `cur` to the next one (caller holds mu)
    void seal_current() {
        Batch& x = b[cur];
        if (x.state != BState::kFilling) return;
        x.state = BState::kSealed;
        x.sealed_at = Clock::now();
        cur = (cur + 1) % (uint32_t)b.size();
        fcv.notify_all();
    }

    void flush_loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            Batch& x = b[next_launch];
            if (quit && x.state != BState::kSealed && (x.state != BState::kFilling || x.subs == 0)) return;
            if (x.state == BState::kFilling && x.subs > 0) {
                const auto due = x.first + std::chrono::microseconds(cfg.max_delay_us);
                if (flush_req || quit || Clock::now() >= due) {
                    flush_req = false;
                    if (cur == next_launch) seal_current();
                    continue;
                }
                // a timed wait on the system clock (pthread_cond_timedwait); the deadline itself is
                // kept on the steady clock above
                fcv.wait_until(lk, std::chrono::system_clock::now() + (due - Clock::now()));
                continue;
            }
            if (x.state != BState::kSealed || x.writers > 0) {
                fcv.wait(lk);
                continue;
            }
            // sealed and every submitter's copy-in is done: launch it
            const uint32_t n = x.npk;
            uint32_t hint = x.one_key ? x.key0 : NEB_KEYS_MIXED;
            lk.unlock();
            // one tunnel's packets run the single-key kernel, if that key is installed for this
            // algorithm (otherwise the mixed path reports NEB_STATUS_BAD_KEY per packet)
            if (hint != NEB_KEYS_MIXED && !dev.key_ok(hint)) hint = NEB_KEYS_MIXED;
            const Clock::time_point tl = Clock::now();
            const int rc = dev.launch(next_launch, x.desc, n, x.arena, x.status, hint, x.tok);
            lk.lock();
            x.rc = rc;
            x.state = BState::kLaunched;
            x.launched_at = tl;
            ns_fill += ns_between(x.first, x.sealed_at);
            ns_drain += ns_between(x.sealed_at, tl);
            n_batches++;
            n_packets += n;
            next_launch = (next_launch + 1) % (uint32_t)b.size();
            fcv.notify_all();  // the completer
        }
    }

    void complete_loop() {
        uint32_t i = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            Batch& x = b[i];
            if (x.state != BState::kLaunched) {
                if (quit && x.state != BState::kSealed && x.state != BState::kFilling) return;
                fcv.wait(lk);
                continue;
            }
            lk.unlock();
            const int wrc = x.rc == NEB_OK ? dev.wait(x.tok) : NEB_OK;
            lk.lock();
            if (wrc != NEB_OK && x.rc == NEB_OK) x.rc = wrc;
            x.state = BState::kDone;
            ns_device += ns_between(x.launched_at, Clock::now());
            cv.notify_all();
            i = (i + 1) % (uint32_t)b.size();
        }
    }
    // neb_queue_submit (include/nebula_aead.h)
    int submit(const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status) {
    Queue* q = this;
    if (n && (!desc || !arena || !status)) return NEB_ERR_INVALID;
    if (n == 0) return NEB_OK;
    // validated before anything is staged: a bad batch leaves the arena and statuses untouched
    for (uint32_t i = 0; i < n; i++)
        if (!neb_desc_in_arena(desc[i], open, arena_len)) return NEB_ERR_INVALID;
    const bool zc = q->dev.mapped(arena);  // stage descriptors only
    // the submission in pieces that each fit one batch
    uint32_t p0 = 0;
    while (p0 < n) {
        uint32_t cnt = 0;
        size_t bytes = 0;
        while (p0 + cnt < n && cnt < q->cfg.max_packets) {
            const size_t sb = zc ? 0 : staged_bytes(desc[p0 + cnt], open);
            if (bytes + sb > q->cfg.arena_bytes) break;
            bytes += sb;
            cnt++;
        }
        if (cnt == 0) return NEB_ERR_INVALID;  // one packet larger than the whole staging
        // reserve room in the filling batch
        Batch* x = nullptr;
        uint32_t pk0 = 0;
        size_t off0 = 0;
        {
            std::unique_lock<std::mutex> lk(q->mu);
            for (;;) {
                if (q->quit) return NEB_ERR_INVALID;
                Batch& c = q->b[q->cur];
                if (c.state == BState::kFree) {
                    c.state = BState::kFilling;
                    c.npk = c.subs = c.writers = c.readers = 0;
                    c.used = 0;
                    c.one_key = true;
                    c.key0 = NEB_KEYS_MIXED;
                    c.rc = NEB_OK;
                }
                if (c.state == BState::kFilling) {
                    if (c.npk + cnt <= q->cfg.max_packets && c.used + bytes <= q->cfg.arena_bytes) break;
                    q->seal_current();  // full for this submission: it goes out, the next one fills
                    continue;
                }
                q->cv.wait(lk);  // every staging batch is busy
            }
            Batch& c = q->b[q->cur];
            x = &c;
            pk0 = c.npk;
            off0 = c.used;
            c.npk += cnt;
            c.used += bytes;
            if (c.subs++ == 0) {
                c.first = Clock::now();
                q->fcv.notify_all();  // the flusher starts this batch's deadline
            }
            c.writers++;
            c.readers++;
            q->n_subs++;
            q->n_bytes += bytes;
            q->n_zc += zc;
            for (uint32_t i = 0; i < cnt; i++) {
                const uint32_t k = desc[p0 + i].key_id;
                if (c.key0 == NEB_KEYS_MIXED && c.one_key) c.key0 = k;
                else if (c.key0 != k) c.one_key = false;
            }
            if (c.npk == q->cfg.max_packets) q->seal_current();
        }
        // copy the packets into the staging (outside the lock: submitters copy in parallel)
        const Clock::time_point t_in = Clock::now();
        size_t off = off0;
        const uint64_t rebase = (uint64_t)(uintptr_t)arena - (uint64_t)(uintptr_t)x->arena;  // wraps
        for (uint32_t i = 0; i < cnt; i++) {
            const neb_desc& d = desc[p0 + i];
            neb_desc s = d;
            if (zc) {  // the caller's own bytes, in place
                s.aad_off = d.aad_off + rebase;
                s.src_off = d.src_off + rebase;
                s.dst_off = d.dst_off + rebase;
                s.flags = 0;
                x->desc[pk0 + i] = s;
                x->status[pk0 + i] = -1;
                continue;
            }
            const size_t src = (size_t)d.len + (open ? 16u : 0u), dst = (size_t)d.len + (open ? 0u : 16u);
            s.aad_off = off;
            if (d.aad_len) std::memcpy(x->arena + off, arena + d.aad_off, d.aad_len);
            off += up16(d.aad_len);
            s.src_off = off;
            std::memcpy(x->arena + off, arena + d.src_off, src);
            if (d.src_off == d.dst_off) {
                s.dst_off = off;
                off += up16(std::max(src, dst));
            } else {
                off += up16(std::max(src, dst));
                s.dst_off = off;
                off += up16(dst);
            }
            s.flags = 0;
            x->desc[pk0 + i] = s;
            x->status[pk0 + i] = -1;
        }
        const Clock::time_point t_copied = Clock::now();
        {
            std::unique_lock<std::mutex> lk(q->mu);
            if (--x->writers == 0) q->fcv.notify_all();
            q->cv.wait(lk, [x] { return x->state == BState::kDone; });
        }
        const Clock::time_point t_done = Clock::now();
        const int rc = x->rc;
        if (rc == NEB_OK && zc) {
            for (uint32_t i = 0; i < cnt; i++) status[p0 + i] = x->status[pk0 + i];
        } else if (rc == NEB_OK) {
            for (uint32_t i = 0; i < cnt; i++) {
                const neb_desc& d = desc[p0 + i];
                const neb_desc& s = x->desc[pk0 + i];
                const int32_t st = x->status[pk0 + i];
                status[p0 + i] = st;
                // what the in-place batch writes: the sealed payload + tag, or the opened (or, on a
                // failed tag, zeroed) payload; nothing for a refused key or an exhausted counter
                if (st == NEB_STATUS_OK || (open && st == NEB_STATUS_AUTH_FAILED))
                    std::memcpy(arena + d.dst_off, x->arena + s.dst_off, (size_t)d.len + (open ? 0u : 16u));
            }
        }
        {
            std::lock_guard<std::mutex> g(q->mu);
            q->ns_copy_in += ns_between(t_in, t_copied);
            q->ns_wait += ns_between(t_copied, t_done);
            q->ns_copy_out += ns_between(t_done, Clock::now());
            if (--x->readers == 0) {
                x->state = BState::kFree;
                q->cv.notify_all();
            }
        }
        if (rc != NEB_OK) return rc;
        p0 += cnt;
    }
    return NEB_OK;
}

    int flush() {
        std::lock_guard<std::mutex> g(mu);
        flush_req = true;
        fcv.notify_all();
        return NEB_OK;
    }
    void stats(uint64_t s[4]) {
        std::lock_guard<std::mutex> g(mu);
        s[0] = n_batches;
        s[1] = n_packets;
        s[2] = n_subs;
        s[3] = n_bytes;
    }
    void phases(uint64_t ns[6]) {
        std::lock_guard<std::mutex> g(mu);
        ns[0] = ns_fill;
        ns[1] = ns_drain;
        ns[2] = ns_device;
        ns[3] = ns_copy_in;
        ns[4] = ns_wait;
        ns[5] = ns_copy_out;
    }
    uint64_t zero_copy_submissions() {
        std::lock_guard<std::mutex> g(mu);
        return n_zc;
    }
    void start() {
        flusher = std::thread([this] { flush_loop(); });
        completer = std::thread([this] { complete_loop(); });
    }
    // send out what is queued, wait for it and for every submitter to have copied its results out
    void shutdown() {
        {
            std::lock_guard<std::mutex> g(mu);
            quit = true;
            fcv.notify_all();
            cv.notify_all();
        }
        if (flusher.joinable()) flusher.join();
        {
            std::lock_guard<std::mutex> g(mu);
            fcv.notify_all();
        }
        if (completer.joinable()) completer.join();
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] {
            for (Batch& x : b)
                if (x.readers > 0) return false;
            return true;
        });
    }
};

}  // namespace neb_q
