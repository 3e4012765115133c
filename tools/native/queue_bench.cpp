// queue_bench.cpp — the submission queue and the per-packet surface driven from native threads (no
// interpreter between the caller and the C ABI): T threads, each a Nebula routine that seals its
// flush of F packets (SendBatchCap = 128, overlay/batch/tx_batch.go:5) through a seal queue and
// opens it back through an open queue (listen.batch = 64, main.go:181), in a loop; or T threads
// calling neb_encrypt_danger / neb_decrypt_danger packet by packet. Prints one JSON line per
// configuration. Build: make -C tools/native; run on the GPU box.
//   queue_bench queue|queuezc <threads> <flush> <deadline_us> <max_packets> <seconds>
//     [depth]  (queuezc: each thread's arena from neb_host_alloc, so its flushes are submitted
//     zero-copy; depth: staging batches per queue, default 4)
//   queue_bench percall <threads> <seconds>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/nebula_aead.h"

using Clock = std::chrono::steady_clock;

static double pct(std::vector<double>& v, double p) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1)))];
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const bool percall = !std::strcmp(argv[1], "percall");
    const bool zc = !std::strcmp(argv[1], "queuezc");
    const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
    const int flush = percall ? 1 : (argc > 3 ? std::atoi(argv[3]) : 128);
    const uint32_t deadline = percall ? 0 : (argc > 4 ? (uint32_t)std::atoi(argv[4]) : 100);
    const uint32_t maxpk = percall ? 0 : (argc > 5 ? (uint32_t)std::atoi(argv[5]) : 8192);
    const int si = percall ? 3 : 6;  // the seconds argument
    const double secs = argc > si ? std::atof(argv[si]) : 1.5;
    const uint32_t depth = !percall && argc > 7 ? (uint32_t)std::atoi(argv[7]) : 4;
    const uint32_t kTunnels = 64, kLen = 1300, kSlot = 1344;
    neb_engine* e = nullptr;
    if (neb_engine_create(0, 4096, &e) != NEB_OK) {
        std::fprintf(stderr, "engine: %s\n", neb_last_error());
        return 1;
    }
    std::vector<neb_cipher*> keys(kTunnels);
    for (uint32_t k = 0; k < kTunnels; k++) {
        uint8_t key[32];
        for (int i = 0; i < 32; i++) key[i] = (uint8_t)(k * 31 + i);
        neb_cipher_create(e, NEB_ALG_AESGCM, key, &keys[k]);
    }
    neb_queue *sq = nullptr, *oq = nullptr;
    if (!percall) {
        neb_queue_config c{maxpk, deadline, (uint64_t)maxpk * 1536, depth, 0};
        if (neb_queue_create(e, NEB_ALG_AESGCM, 0, &c, &sq) != NEB_OK || neb_queue_create(e, NEB_ALG_AESGCM, 1, &c, &oq) != NEB_OK) {
            std::fprintf(stderr, "queue: %s\n", neb_last_error());
            return 1;
        }
    }
    std::atomic<bool> go{false}, stop{false};
    std::atomic<uint64_t> pkts{0};
    std::atomic<int> errs{0};
    std::vector<std::vector<double>> lat(threads);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            std::vector<uint8_t> heap;
            uint8_t* arena_p = nullptr;
            const size_t arena_n = (size_t)flush * kSlot;
            if (zc) {
                void* p = nullptr;
                if (neb_host_alloc(arena_n, &p) != NEB_OK) {
                    errs++;
                    return;
                }
                arena_p = static_cast<uint8_t*>(p);
                std::memset(arena_p, t, arena_n);
            } else {
                heap.assign(arena_n, (uint8_t)t);
                arena_p = heap.data();
            }
            struct View {
                uint8_t* p;
                size_t n;
                uint8_t* data() { return p; }
                size_t size() const { return n; }
            } arena{arena_p, arena_n};
            std::vector<neb_desc> d(flush);
            std::vector<int32_t> st(flush);
            uint64_t ctr = (uint64_t)t << 40;
            for (int i = 0; i < flush; i++) {
                const uint64_t b = (uint64_t)i * kSlot;
                d[i] = neb_desc{b + 16, b + 16, b, 0, kLen, 16, neb_cipher_key_id(keys[(t * 7 + i) % kTunnels]), 0};
            }
            std::vector<uint8_t> out(kLen + 64), back(kLen + 64);
            bool counting = false;
            while (!stop.load(std::memory_order_relaxed)) {
                if (!counting && go.load()) {
                    counting = true;
                    lat[t].clear();
                }
                const auto t0 = Clock::now();
                auto t1q = t0;
                if (percall) {
                    size_t rl = 0;
                    neb_cipher* c = keys[t % kTunnels];
                    int rc = neb_encrypt_danger(c, out.data(), 0, out.size(), arena.data(), 16, arena.data() + 16, kLen,
                                                ++ctr, nullptr, &rl);
                    rc |= neb_decrypt_danger(c, back.data(), 0, back.size(), arena.data(), 16, out.data(), kLen + 16, ctr,
                                             nullptr, &rl);
                    if (rc) errs++;
                } else {
                    for (auto& x : d) x.counter = ++ctr;
                    const int rc1 = neb_queue_submit(sq, d.data(), flush, arena.data(), arena.size(), st.data());
                    int bad1 = 0;
                    for (int32_t s : st) bad1 += s != 0;
                    const auto t1 = Clock::now();
                    t1q = t1;
                    if (counting) lat[t].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                    const int rc2 = neb_queue_submit(oq, d.data(), flush, arena.data(), arena.size(), st.data());
                    int bad2 = 0, first = 0;
                    for (int32_t s : st)
                        if (s) {
                            if (!bad2) first = s;
                            bad2++;
                        }
                    if (rc1 || rc2 || bad1 || bad2) {
                        if (errs++ < 5)
                            std::fprintf(stderr, "thread %d: seal rc %d bad %d, open rc %d bad %d (first status %d)\n", t,
                                         rc1, bad1, rc2, bad2, first);
                    }
                }
                const auto t2 = Clock::now();
                if (counting) {
                    // per call: the two calls' mean (percall); the open submit's own time (queue; the
                    // seal submit's was taken above)
                    if (percall)
                        lat[t].push_back(std::chrono::duration<double, std::micro>(t2 - t0).count() / 2);
                    else
                        lat[t].push_back(std::chrono::duration<double, std::micro>(t2 - t1q).count());
                    pkts += flush;
                }
            }
            if (zc) neb_host_free(arena_p);
        });
    std::this_thread::sleep_for(std::chrono::milliseconds(400));
    uint64_t s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, o0[4] = {0, 0, 0, 0}, o1[4] = {0, 0, 0, 0};
    uint64_t ph0[2][6] = {}, ph1[2][6] = {};
    go = true;
    pkts = 0;
    if (sq) {
        neb_queue_stats(sq, s0);
        neb_queue_stats(oq, o0);
        neb_queue_phases(sq, ph0[0]);
        neb_queue_phases(oq, ph0[1]);
    }
    const auto t0 = Clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    const uint64_t n = pkts.load();
    if (sq) {
        neb_queue_stats(sq, s1);
        neb_queue_stats(oq, o1);
        neb_queue_phases(sq, ph1[0]);
        neb_queue_phases(oq, ph1[1]);
    }
    stop = true;
    for (auto& x : th) x.join();
    std::vector<double> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    const double p50 = pct(all, 0.5), p99 = pct(all, 0.99);
    const double gibs = 2.0 * n * kLen / dt / (1 << 30);
    if (percall)
        std::printf("{\"bench\": \"percall_native\", \"threads\": %d, \"calls_per_s\": %.0f, \"gibs\": %.4f, "
                    "\"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f, \"errors\": %d}\n",
                    threads, 2.0 * n / dt, gibs, p50, p99, errs.load());
    else
        std::printf("{\"bench\": \"%s\", \"threads\": %d, \"flush_packets\": %d, \"deadline_us\": %u, "
                    "\"max_packets\": %u, \"depth\": %u, \"gibs\": %.3f, \"packets_per_s\": %.0f, \"submit_latency_us_p50\": %.1f, "
                    "\"submit_latency_us_p99\": %.1f, \"seal_batches_per_s\": %.1f, \"mean_seal_batch_packets\": %.1f, "
                    "\"errors\": %d}\n",
                    zc ? "queue_native_zero_copy" : "queue_native", threads, flush, deadline, maxpk, depth, gibs, n / dt, p50, p99, (s1[0] - s0[0]) / dt,
                    (double)(s1[1] - s0[1]) / std::max<uint64_t>(1, s1[0] - s0[0]), errs.load());
    if (!percall) {
        // where the time goes (neb_queue_phases), mean µs: per device batch fill / drain / device, per
        // submission copy-in / wait / copy-out; seal queue, then open queue
        const char* nm[2] = {"seal", "open"};
        for (int k = 0; k < 2; k++) {
            const uint64_t* a = ph0[k];
            const uint64_t* b = ph1[k];
            const double nb = (double)std::max<uint64_t>(1, (k ? o1[0] - o0[0] : s1[0] - s0[0]));
            const double ns = (double)std::max<uint64_t>(1, (k ? o1[2] - o0[2] : s1[2] - s0[2]));
            std::printf("{\"bench\": \"queue_phases\", \"queue\": \"%s\", \"threads\": %d, \"zero_copy\": %s, "
                        "\"batches\": %.0f, \"fill_us\": %.1f, \"drain_us\": %.1f, \"device_us\": %.1f, "
                        "\"copy_in_us\": %.1f, \"wait_us\": %.1f, \"copy_out_us\": %.1f}\n",
                        nm[k], threads, zc ? "true" : "false", nb, (b[0] - a[0]) / nb / 1e3, (b[1] - a[1]) / nb / 1e3,
                        (b[2] - a[2]) / nb / 1e3, (b[3] - a[3]) / ns / 1e3, (b[4] - a[4]) / ns / 1e3,
                        (b[5] - a[5]) / ns / 1e3);
        }
    }
    if (sq) neb_queue_destroy(sq);
    if (oq) neb_queue_destroy(oq);
    for (auto* k : keys) neb_cipher_destroy(k);
    neb_engine_destroy(e);
    return errs ? 1 : 0;
}
