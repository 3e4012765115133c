// queue_test.cpp — sanitizer test (ASan + UBSan, and TSan) of the submission queue's state machine
// (nebula_amd/csrc/queue_core.hpp) on a CPU device: a worker thread that seals / opens each staged
// batch with the plain-C oracle (oracle/aead_oracle.c, test infrastructure). 16 threads submit
// Nebula-sized flushes (128 and 64 packets, interface.go:381-487) through seal and open queues with
// short deadlines, explicit flushes, a two-deep ring, submissions larger than a batch (pieces), an
// uninstalled key, an exhausted counter and a descriptor past the arena; every result must equal
// the oracle run directly on the same descriptors. TEST INFRASTRUCTURE; `make -C tests/sanitize`.
#include <atomic>
#include <cinttypes>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <memory>
#include <random>
#include <set>

#include "../../nebula_amd/csrc/queue_core.hpp"

extern "C" void ora_batch(int alg, int open, const uint8_t* keys, const neb_desc* d, size_t n, uint8_t* arena,
                          int32_t* status);

static int fails = 0;
#define CHECK(x)                                                                              \
    do {                                                                                      \
        if (!(x)) {                                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #x);        \
            fails++;                                                                          \
        }                                                                                     \
    } while (0)

constexpr uint32_t kKeys = 8;
static uint8_t g_keys[32 * kKeys];

// Arenas the CpuDev treats as mapped (the zero-copy submissions): registered by the test.
static std::mutex g_mapped_mu;
static std::set<const void*> g_mapped;
static void set_mapped(const void* p, bool on) {
    std::lock_guard<std::mutex> g(g_mapped_mu);
    if (on) g_mapped.insert(p); else g_mapped.erase(p);
}

// A device that runs batches in launch order on one worker thread (as a stream would). Descriptor
// offsets are relative to the batch's base as wrapping 64-bit offsets (a zero-copy submission's
// point into its caller's arena): each packet is rebased to its lowest byte before the oracle runs
// it, so no pointer arithmetic wraps here.
struct CpuDev {
    struct Job {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false;
    };
    using Token = std::shared_ptr<Job>;
    int alg = 1, open = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> work;
    bool quit = false;
    std::thread th;
    void start() {
        th = std::thread([this] {
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return quit || !work.empty(); });
                    if (work.empty()) return;
                    f = std::move(work.front());
                    work.pop_front();
                }
                f();
            }
        });
    }
    void stop() {
        {
            std::lock_guard<std::mutex> g(mu);
            quit = true;
        }
        cv.notify_all();
        th.join();
    }
    int launch(uint32_t, neb_desc* desc, uint32_t n, uint8_t* arena, int32_t* status, uint32_t hint, Token& tok) {
        tok = std::make_shared<Job>();
        Token t = tok;
        const int a = alg, o = open;
        std::lock_guard<std::mutex> g(mu);
        work.push_back([=] {
            for (uint32_t i = 0; i < n; i++) {
                if (desc[i].key_id >= kKeys || (hint != NEB_KEYS_MIXED && desc[i].key_id != hint)) {
                    status[i] = NEB_STATUS_BAD_KEY;
                    continue;
                }
                const uint64_t base = (uint64_t)(uintptr_t)arena;
                const uint64_t aad = base + desc[i].aad_off, src = base + desc[i].src_off, dst = base + desc[i].dst_off;
                const uint64_t lo = std::min(aad, std::min(src, dst));
                neb_desc d = desc[i];
                d.aad_off = aad - lo;
                d.src_off = src - lo;
                d.dst_off = dst - lo;
                ora_batch(a, o, g_keys, &d, 1, reinterpret_cast<uint8_t*>((uintptr_t)lo), status + i);
            }
            std::lock_guard<std::mutex> g2(t->mu);
            t->done = true;
            t->cv.notify_all();
        });
        cv.notify_all();
        return NEB_OK;
    }
    int wait(Token& tok) {
        std::unique_lock<std::mutex> lk(tok->mu);
        tok->cv.wait(lk, [&] { return tok->done; });
        return NEB_OK;
    }
    bool key_ok(uint32_t key) { return key < kKeys; }
    bool mapped(const uint8_t* arena) {
        std::lock_guard<std::mutex> g(g_mapped_mu);
        return g_mapped.count(arena) != 0;
    }
};

using Q = neb_q::Queue<CpuDev>;

static std::unique_ptr<Q> make_queue(int alg, int open, uint32_t max_packets, uint32_t delay_us, uint32_t depth,
                                     uint64_t arena_bytes) {
    auto q = std::make_unique<Q>();
    neb_queue_config c{max_packets, delay_us, arena_bytes, depth, 0};
    if (!neb_q::normalize(c)) return nullptr;
    q->cfg = c;
    q->open = open;
    q->dev.alg = alg;
    q->dev.open = open;
    q->b.resize(c.depth);
    for (auto& x : q->b) {
        x.arena = new uint8_t[c.arena_bytes];
        x.desc = new neb_desc[c.max_packets];
        x.status = new int32_t[c.max_packets];
    }
    q->dev.start();
    q->start();
    return q;
}

static void free_queue(std::unique_ptr<Q>& q) {
    q->shutdown();
    q->dev.stop();
    for (auto& x : q->b) {
        delete[] x.arena;
        delete[] x.desc;
        delete[] x.status;
    }
    q.reset();
}

// one thread's flush: n packets of mixed sizes in its own arena
struct Flush {
    std::vector<uint8_t> arena;
    std::vector<neb_desc> desc;
};

static Flush make_flush(std::mt19937_64& rng, uint32_t n, uint64_t ctr0) {
    static const uint32_t sizes[] = {0, 1, 16, 90, 576, 1300};
    Flush f;
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t len = sizes[rng() % 6];
        neb_desc d{};
        d.aad_off = off;
        d.aad_len = 16;
        d.src_off = d.dst_off = off + 16 + (rng() % 3 == 0 ? 1 : 0);  // some payloads off alignment
        if (rng() % 7 == 0) d.dst_off = d.src_off + len + 64;         // and some out of place
        d.len = len;
        d.counter = ctr0 + i;
        d.key_id = (uint32_t)(rng() % kKeys);
        f.desc.push_back(d);
        off = std::max(d.src_off, d.dst_off) + len + 16 + 64;
    }
    f.arena.resize(off + 64);
    for (auto& b : f.arena) b = (uint8_t)rng();
    return f;
}

static void stress(int alg, uint32_t flush_pk, uint32_t max_packets, uint32_t delay_us, uint32_t depth,
                   uint64_t arena_bytes, int threads, int rounds) {
    auto sq = make_queue(alg, 0, max_packets, delay_us, depth, arena_bytes);
    auto oq = make_queue(alg, 1, max_packets, delay_us, depth, arena_bytes);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            std::mt19937_64 rng(100 + t);
            for (int r = 0; r < rounds; r++) {
                Flush f = make_flush(rng, flush_pk, ((uint64_t)t << 40) + (uint64_t)r * 1000);
                const bool zc = (t + r) % 2 == 1;  // half the flushes submitted zero-copy
                set_mapped(f.arena.data(), zc);
                std::vector<uint8_t> ref = f.arena;
                std::vector<int32_t> st(f.desc.size(), -1), rst(f.desc.size(), -1);
                ora_batch(alg, 0, g_keys, f.desc.data(), f.desc.size(), ref.data(), rst.data());
                if (sq->submit(f.desc.data(), (uint32_t)f.desc.size(), f.arena.data(), f.arena.size(), st.data()) != NEB_OK ||
                    st != rst || f.arena != ref)
                    bad++;
                ora_batch(alg, 1, g_keys, f.desc.data(), f.desc.size(), ref.data(), rst.data());
                if (oq->submit(f.desc.data(), (uint32_t)f.desc.size(), f.arena.data(), f.arena.size(), st.data()) != NEB_OK ||
                    st != rst || f.arena != ref)
                    bad++;
                set_mapped(f.arena.data(), false);
                if (r % 5 == 4) sq->flush();
            }
        });
    for (auto& x : th) x.join();
    CHECK(bad == 0);
    uint64_t s[4];
    sq->stats(s);
    CHECK(s[2] >= (uint64_t)threads * rounds);
    CHECK(sq->zero_copy_submissions() > 0 && sq->zero_copy_submissions() < s[2]);
    free_queue(sq);
    free_queue(oq);
}

static void edge_cases() {
    auto q = make_queue(1, 0, 64, 50, 2, 64 * 1536);
    std::mt19937_64 rng(3);
    // larger than one batch: goes through in pieces
    Flush f = make_flush(rng, 300, 5);
    std::vector<uint8_t> ref = f.arena;
    std::vector<int32_t> st(300, -1), rst(300, -1);
    ora_batch(1, 0, g_keys, f.desc.data(), 300, ref.data(), rst.data());
    CHECK(q->submit(f.desc.data(), 300, f.arena.data(), f.arena.size(), st.data()) == NEB_OK);
    CHECK(st == rst && f.arena == ref);
    // an exhausted counter and an uninstalled key: refused, nothing written
    Flush g = make_flush(rng, 8, 9);
    g.desc[2].counter = ~0ull - (1ull << 40);
    g.desc[5].key_id = kKeys + 3;
    std::vector<uint8_t> before = g.arena;
    std::vector<int32_t> st2(8, -1);
    CHECK(q->submit(g.desc.data(), 8, g.arena.data(), g.arena.size(), st2.data()) == NEB_OK);
    CHECK(st2[2] == NEB_STATUS_EXHAUSTED && st2[5] == NEB_STATUS_BAD_KEY);
    for (uint32_t i : {2u, 5u}) {
        const neb_desc& d = g.desc[i];
        CHECK(std::equal(g.arena.begin() + d.dst_off, g.arena.begin() + d.dst_off + d.len + 16, before.begin() + d.dst_off));
    }
    // a descriptor past the arena: refused before anything is staged
    Flush h = make_flush(rng, 4, 11);
    h.desc[3].len = (uint32_t)h.arena.size();
    before = h.arena;
    std::vector<int32_t> st3(4, 77);
    CHECK(q->submit(h.desc.data(), 4, h.arena.data(), h.arena.size(), st3.data()) == NEB_ERR_INVALID);
    CHECK(h.arena == before && st3[0] == 77);
    free_queue(q);
}

int main() {
    std::mt19937_64 rng(1);
    for (auto& k : g_keys) k = (uint8_t)rng();
    edge_cases();
    stress(1, 128, 4096, 100, 3, 0, 16, 12);   // TX-sized flushes, AES-GCM
    stress(2, 64, 1024, 20, 2, 0, 16, 12);     // RX-sized, ChaCha20-Poly1305, two-deep ring
    stress(1, 128, 512, 1000, 4, 0, 8, 10);    // batches filled by size, not by deadline
    std::printf("queue_test: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
