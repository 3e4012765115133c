// window_test.cpp — sanitizer test (ASan + UBSan, and TSan) of the host receive logic in
// nebula_amd/csrc/window_core.hpp: Nebula's replay window (WindowCore, bits.go:15-262), the exact
// receive order over window runs (exact_rounds) and the thread pool the batched receive spreads
// windows over (RxPool). TEST INFRASTRUCTURE; built and run by `make -C tests/sanitize`.
//
//  1. random Check/Update streams over every window length 1..8192, counters near 0 and near 2^64
//     (clear_range's circular slot arithmetic, the warmup path, jumps past the window);
//  2. exact_rounds over many windows with forged packets, against the packet-by-packet loop
//     (connection_state.go:99-119): statuses, commits and window states must match, with the
//     per-window groups spread over an RxPool and several threads running batches at once;
//  3. RxPool::run from several threads at once.
#include <cassert>
#include <cinttypes>
#include <cstdio>
#include <random>

#include "../../nebula_amd/csrc/window_core.hpp"

using namespace neb_rx;

static WindowCore make_window(uint64_t length) {
    WindowCore w;
    w.length = length;
    w.mask = length - 1;
    w.words.assign(length >= 64 ? length / 64 : 1, 0);
    w.words[0] = 1;  // counter 0 seeded as received (bits.go:47-48)
    return w;
}

static bool same(const WindowCore& a, const WindowCore& b) {
    return a.current == b.current && a.words == b.words && a.lost == b.lost && a.dupe == b.dupe &&
           a.out_of_window == b.out_of_window;
}

static int fails = 0;
#define CHECK(x)                                                                 \
    do {                                                                         \
        if (!(x)) {                                                              \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #x); \
            fails++;                                                             \
        }                                                                        \
    } while (0)

static void random_streams() {
    std::mt19937_64 rng(7);
    for (uint64_t len = 1; len <= 8192; len <<= 1) {
        for (int base_kind = 0; base_kind < 3; base_kind++) {
            WindowCore w = make_window(len);
            uint64_t base = base_kind == 0 ? 0 : base_kind == 1 ? (1ull << 62) : ~0ull - 20000;
            if (base) w.update(base);
            for (int k = 0; k < 1000; k++) {
                const uint64_t r = rng();
                uint64_t c;
                switch (r % 5) {
                    case 0: c = w.current + 1; break;
                    case 1: c = w.current - (r >> 8) % (2 * len + 3); break;
                    case 2: c = w.current + (r >> 8) % (3 * len + 5); break;
                    case 3: c = w.current + (r >> 8) % 4; break;
                    default: c = (r >> 3) % 4 == 0 ? ~0ull - (r >> 8) % 64 : w.current + 2; break;
                }
                const uint64_t before = w.current;
                const bool ok = w.check(c);
                const bool up = w.update(c);
                // an update never accepts what check refused on the same state, except Go's uint64
                // wrap at the top of the counter space (i == current + 1 == 0, bits.go:171)
                CHECK(!up || ok || before == ~0ull);
            }
        }
    }
}

struct Pkt {
    uint32_t w;
    uint64_t c;
    bool forged;
};

// the packet-by-packet receive (connection_state.go:99-119) over private copies of the windows
static void sequential(std::vector<WindowCore>& wins, const std::vector<Pkt>& pk, std::vector<int32_t>& st) {
    for (size_t i = 0; i < pk.size(); i++) {
        WindowCore& w = wins[pk[i].w];
        if (!w.check(pk[i].c)) {
            st[i] = NEB_STATUS_REPLAY;
            continue;
        }
        if (pk[i].forged) {
            st[i] = NEB_STATUS_AUTH_FAILED;
            continue;
        }
        st[i] = w.update(pk[i].c) ? NEB_STATUS_OK : NEB_STATUS_REPLAY;
    }
}

// exact_rounds over the same batch, starting from nothing opened (every packet held back)
static void exact(std::vector<WindowCore>& wins, std::vector<std::mutex>& mus, const std::vector<Pkt>& pk,
                  std::vector<int32_t>& st, RxPool& pool, uint32_t groups, uint32_t* opens) {
    const uint32_t n = (uint32_t)pk.size(), nw = (uint32_t)wins.size();
    std::vector<uint32_t> order;
    std::vector<ExactRun> runs;
    for (uint32_t w = 0; w < nw; w++) {
        const uint32_t k0 = (uint32_t)order.size();
        for (uint32_t i = 0; i < n; i++)
            if (pk[i].w == w) order.push_back(i);
        if (order.size() > k0) runs.push_back({w, k0, (uint32_t)order.size()});
    }
    std::vector<uint8_t> opened(n, 0);
    std::vector<int32_t> verd(n, NEB_STATUS_BAD_KEY);
    std::vector<uint32_t> commit, zero;
    auto verify = [&](const std::vector<uint32_t>& p, uint8_t how) {
        for (uint32_t i : p) {
            CHECK(!opened[i]);
            opened[i] = how;
            verd[i] = pk[i].forged ? NEB_STATUS_AUTH_FAILED : NEB_STATUS_OK;
        }
        (*opens)++;
        return NEB_OK;
    };
    const int rc = exact_rounds(
        runs, groups, [&](uint32_t k) { return pk[order[k]].c; }, [&](uint32_t k) { return order[k]; },
        opened.data(), verd.data(), st.data(),
        [&](uint32_t w, auto&& fn) {
            std::lock_guard<std::mutex> g(mus[w]);
            fn(wins[w]);
        },
        [&](const std::vector<uint32_t>& p) { return verify(p, 1); },
        [&](const std::vector<uint32_t>& p) { return verify(p, 2); },
        [&](uint32_t cnt, auto&& fn) { pool.run(cnt, fn); }, &commit, &zero);
    CHECK(rc == NEB_OK);
    for (uint32_t i : commit) CHECK(opened[i] == 2 && st[i] == NEB_STATUS_OK);
    for (uint32_t i : zero) CHECK(opened[i] == 2 && st[i] == NEB_STATUS_AUTH_FAILED);
}

static void exact_vs_sequential(uint64_t seed, RxPool& pool) {
    std::mt19937_64 rng(seed);
    const uint32_t nw = 1 + rng() % 40;
    const uint64_t len = 1ull << (rng() % 11);
    std::vector<Pkt> pk;
    std::vector<uint64_t> cur(nw, 2);
    for (int i = 0; i < 4000; i++) {
        const uint32_t w = rng() % nw;
        const uint64_t r = rng();
        uint64_t c;
        if (r % 100 < 4) c = cur[w] + 100000 + r % 1000000;  // a forged far-ahead counter
        else if (r % 100 < 70) c = ++cur[w];
        else c = cur[w] - r % (len + 4) + 1;
        pk.push_back({w, c, r % 100 < 4 || (r >> 20) % 50 == 0});
    }
    std::vector<WindowCore> a, b;
    for (uint32_t w = 0; w < nw; w++) {
        a.push_back(make_window(len));
        a.back().update(1);
        a.back().update(2);
    }
    b = a;
    std::vector<std::mutex> mus(nw);
    std::vector<int32_t> sa(pk.size(), -1), sb(pk.size(), -1);
    sequential(a, pk, sa);
    uint32_t opens = 0;
    exact(b, mus, pk, sb, pool, 4, &opens);
    CHECK(sa == sb);
    for (uint32_t w = 0; w < nw; w++) CHECK(same(a[w], b[w]));
    CHECK(opens <= 3);  // the simulation's batch, then at most one in-place and one speculative round
}

int main() {
    random_streams();
    RxPool pool(4);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; t++)
        th.emplace_back([t, &pool] {
            for (int k = 0; k < 6; k++) exact_vs_sequential(1000 * t + k, pool);
        });
    for (auto& x : th) x.join();
    std::atomic<uint64_t> sum{0};
    std::vector<std::thread> runners;
    for (int t = 0; t < 4; t++)
        runners.emplace_back([&] {
            for (int k = 0; k < 50; k++) pool.run(16, [&](uint32_t j) { sum += j; });
        });
    for (auto& x : runners) x.join();
    CHECK(sum == 4ull * 50 * 120);
    std::printf("window_test: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
