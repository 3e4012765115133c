// rxwin.hpp — device replay windows and the workspace of the device batched receive (rxwin.hip),
// shared with window.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/nebula_aead.h"

namespace neb {

// A window whose counters come this close to 2^64 takes the sequential path (no uint64 wrap in
// the parallel form). No sender reaches it: counters stop at RejectAfterMessages = 2^64 - 2^40 - 1,
// and 2^62 messages is far beyond any tunnel's life; forged counters may, and are then exact too.
constexpr uint64_t kRxRiskyCounter = 1ull << 62;
enum : uint32_t { kRxTouched = 1u, kRxRisky = 2u, kRxSlow = 4u };
// run-order elements per workgroup of the scan and admission kernels (one per thread: their
// per-packet chains of dependent loads and atomics are latency-bound)
constexpr uint32_t kRxThreads = 256, kRxItems = 1, kRxBlock = kRxThreads * kRxItems;
static_assert(kRxItems == 1, "rx_scan_admit_kernel's per-window pending counts take one packet per thread");
// the stable sort by window (rxwin.hip): at most kRxSortBlocks workgroups of 256 x items packets,
// digits of at most 8 bits for one pass, else passes of at most kRxSortDigit bits
constexpr uint32_t kRxSortBlocks = 64, kRxSortDigit = 7, kRxSortMaxPasses = 5, kRxSortLoad = 4;
// polls of a scan-admit lookback before the batch fails (≈ 0.1 s)
constexpr uint32_t kRxSpinLimit = 1u << 20;

struct RxDevWin {  // a set of windows of one length in device memory (neb_dwindows)
    uint32_t count;
    uint32_t words;     // bitmap words per window (a power of two)
    uint32_t words_lg;
    uint64_t length;    // power of two
    uint32_t* present;  // 0 = no window at this index
    uint64_t* cur;
    int64_t* lost;
    int64_t* dupe;
    int64_t* oow;
    uint64_t* bits;     // count x words
};

struct RxDevWs {
    // per packet (arrival index)
    uint32_t* keyw;  // window, or count for none
    uint64_t* ctr;
    uint8_t* adm;
    int32_t* verdict;
    // the sort: per pass, per workgroup digit counts; ping-pong keys / arrival indices
    uint32_t* sort_hist;  // kRxSortMaxPasses x kRxSortBlocks x 256
    uint32_t* tmp_k;
    uint32_t* tmp_v;
    // run order (sorted by window, arrival order kept)
    uint32_t* run_w;
    uint32_t* run_i;
    uint64_t* run_c;  // the counters in run order (read by the host's exact pass)
    // per block of kRxBlock run positions, published inside rx_scan_admit_kernel for the blocks
    // after it: 3 granules {gen:32 | value:32} = the position of its first run head (kRxBlock:
    // none), then the low and high words of the segmented max at its last element
    uint64_t* blk_pub;
    uint32_t* ticket;  // the scan-admit blocks' order of start (zeroed by the keys kernel)
    uint32_t* err;     // nonzero: a scan-admit lookback timed out (zeroed by the keys kernel)
    uint32_t spin_limit;  // kRxSpinLimit; 0 (a test, neb_dwindows_debug) fails every lookback that waits
    // first occurrences: an open-addressing table keyed by (window, counter), 2^tab_lg >= 4n slots,
    // tagged with the batch generation (an entry of an older batch is empty, so the table is
    // never cleared between batches); a slot's owner (gen:32 | arrival index + 1) names its key
    // through keyw / ctr
    uint64_t* tab_owner;
    uint64_t* tab_min;  // gen:32 | ~(the earliest arrival with that key), by atomicMax
    uint32_t tab_lg;
    uint32_t gen;
    // admitted packets, compacted
    uint32_t* sub_map;
    neb_desc* sub_desc;
    int32_t* sub_status;
    uint32_t* nsub;
    // per window
    uint32_t* wrisky;  // the generation of the last batch with a counter >= kRxRiskyCounter in it
    uint32_t* wflag;
    uint64_t* curnew;
    uint64_t* exit_lo;
    uint64_t* exit_hi;
    uint64_t* recv;
    uint64_t* scratch;  // count x words
    uint32_t* need_host;  // pinned host words: [0] nonzero when a touched window is risky or slow,
                          // [1] nonzero on a lookback timeout (an internal error: the batch fails)
    uint32_t* pending;    // per window: admitted packets whose verdict is not settled yet (RxFold)
    struct RxFold* fold;  // device copy of this workspace's RxFold (the open kernels' epilogue)
    // the generation of the last batch whose packets named more than one window (written by the
    // keys kernel); any other value lets the sort passes write the identity order (one window)
    uint32_t* mixed;
};

// The receive's settle and window finish, folded into the open kernels (aes_gcm.hip
// gcm_packet_group, chacha_poly.hip chacha_group: GcmArgs::rx / ChachaArgs::rx). The open runs
// over the whole batch in arrival order and skips the packets rx_scan_admit_kernel did not admit
// (adm[i] == 0: their statuses are already written, their bytes are never touched), so there is
// no compaction and the mixed-key binning can run beside the plan on a second stream (window.cpp).
// As a packet's verdict is known, rx_fold_settle writes it, ORs its counter into the window's
// scratch bitmap (or counts it as received when it leaves the window) and counts it against its
// window in the workgroup's LDS table (RxWgTab); at the end of the workgroup, rx_wg_flush takes
// those counts off the windows' pending counts, and the wave whose decrement brings a window to
// zero holds its last verdict, so it finishes the window right there (rx_fold_finish): the bitmap,
// lost count and current of a window whose packets all verified, or only the scratch cleared for
// one that goes to the host. No settle or finish launch (round 5: 6 → 4 window launches).
struct RxFold {
    RxDevWin win;
    const uint8_t* adm;  // per arrival: admitted by the plan (the open runs only these)
    int32_t* verdict;
    const uint32_t* keyw;
    const uint64_t* ctr;
    uint32_t* wflag;
    const uint64_t* curnew;
    const uint64_t* exit_lo;
    const uint64_t* exit_hi;
    uint64_t* recv;
    uint64_t* scratch;
    uint32_t* pending;
    const uint32_t* err;
    uint32_t* need_host;
};

// Per workgroup of an open kernel: its settled packets counted per window, flushed at its end (one
// pending decrement per workgroup and window: a per-wave returning atomic after a drain of the
// wave's stores cost the C2 receive 466 → 416 GiB/s, one tunnel's 4096 waves on one word). A full
// table takes the per-wave path.
constexpr uint32_t kRxWgSlots = 64;
struct RxWgTab {
    uint32_t w[kRxWgSlots];
    uint32_t n[kRxWgSlots];
};

inline size_t rx_align(size_t x) { return (x + 255) & ~(size_t)255; }

// Carve an RxDevWs for n packets over `count` windows of `words` bitmap words out of base
// (nullptr: only size it). Returns the bytes needed.
inline size_t rx_ws_layout(uint32_t n, uint32_t count, uint32_t words, uint8_t* base, RxDevWs* ws) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t* p = base ? base + off : nullptr;
        off += rx_align(std::max<size_t>(bytes, 1));
        return p;
    };
    RxDevWs w{};
    w.keyw = (uint32_t*)take((size_t)n * 4);
    w.ctr = (uint64_t*)take((size_t)n * 8);
    w.adm = (uint8_t*)take(n);
    w.verdict = (int32_t*)take((size_t)n * 4);
    w.sort_hist = (uint32_t*)take((size_t)kRxSortMaxPasses * kRxSortBlocks * 256 * 4);
    w.tmp_k = (uint32_t*)take((size_t)n * 4);
    w.tmp_v = (uint32_t*)take((size_t)n * 4);
    w.run_w = (uint32_t*)take((size_t)n * 4);
    w.run_i = (uint32_t*)take((size_t)n * 4);
    w.run_c = (uint64_t*)take((size_t)n * 8);
    const size_t nblk = ((size_t)n + kRxBlock - 1) / kRxBlock;
    w.blk_pub = (uint64_t*)take(nblk * 3 * 8);
    w.ticket = (uint32_t*)take(4);
    w.err = (uint32_t*)take(4);
    w.spin_limit = kRxSpinLimit;
    w.tab_lg = 1;
    while ((1ull << w.tab_lg) < 4ull * n) w.tab_lg++;  // at most a quarter full
    w.tab_owner = (uint64_t*)take((size_t)8 << w.tab_lg);
    w.tab_min = (uint64_t*)take((size_t)8 << w.tab_lg);
    w.sub_map = (uint32_t*)take((size_t)n * 4);
    w.sub_desc = (neb_desc*)take((size_t)n * sizeof(neb_desc));
    w.sub_status = (int32_t*)take((size_t)n * 4);
    w.nsub = (uint32_t*)take(4);
    w.wrisky = (uint32_t*)take((size_t)count * 4);
    w.wflag = (uint32_t*)take((size_t)count * 4);
    w.curnew = (uint64_t*)take((size_t)count * 8);
    w.exit_lo = (uint64_t*)take((size_t)count * 8);
    w.exit_hi = (uint64_t*)take((size_t)count * 8);
    w.recv = (uint64_t*)take((size_t)count * 8);
    w.scratch = (uint64_t*)take((size_t)count * words * 8);
    w.mixed = (uint32_t*)take(4);
    w.pending = (uint32_t*)take((size_t)count * 4);
    w.fold = (RxFold*)take(sizeof(RxFold));
    if (ws) *ws = w;
    return off;
}

inline RxFold rx_fold_of(const RxDevWin& win, const RxDevWs& ws) {
    return RxFold{win,        ws.adm,     ws.verdict, ws.keyw,    ws.ctr,     ws.wflag, ws.curnew,
                  ws.exit_lo, ws.exit_hi, ws.recv,    ws.scratch, ws.pending, ws.err,   ws.need_host};
}

__device__ __forceinline__ bool rx_fast_flag(uint32_t fl) { return (fl & kRxTouched) && !(fl & (kRxRisky | kRxSlow)); }

// bits of the slots [a, b) within the word whose first slot is q0 (nb slots)
__device__ __forceinline__ uint64_t rx_seg_mask(uint64_t q0, uint32_t nb, uint64_t a, uint64_t b) {
    const uint64_t lo = max(a, q0), hi = min(b, q0 + nb);
    if (lo >= hi) return 0;
    const uint32_t m = (uint32_t)(hi - lo);
    return (m == 64u ? ~0ull : ((1ull << m) - 1u)) << (lo - q0);
}
// ... within the circular slot range [start, start + count) mod len (start < len)
__device__ __forceinline__ uint64_t rx_ring_mask(uint64_t q0, uint32_t nb, uint64_t start, uint64_t count,
                                                 uint64_t len) {
    if (count == 0) return 0;
    if (count >= len) return nb == 64u ? ~0ull : ((1ull << nb) - 1u);
    uint64_t m = rx_seg_mask(q0, nb, start, min(start + count, len));
    if (start + count > len) m |= rx_seg_mask(q0, nb, 0, start + count - len);
    return m;
}

// Window w's finish, by the whole wave, once every admitted packet of w has its verdict (the wave
// whose pending decrement reached zero; every other settle's atomics completed before its own
// decrement). The slots of the counters new in (cur0, cur] are cleared and the admitted counters
// (the scratch bitmap) ORed in; the old window's counters that leave it are counted as received
// where their old bit is set (tools/rxwin_model.py finish_ranges, checked against the oracle); then
// the window's lost count and current. The scratch is read and cleared with atomic exchanges (it
// was written by other workgroups' atomics in this launch). A window that goes to the host (a
// failed verdict, a counter near the wrap) or a batch whose scan failed only gets its scratch
// cleared.
__device__ __forceinline__ void rx_fold_finish(const RxFold& f, uint32_t w) {
    const uint32_t lane = __lane_id();
    const uint32_t fl = __builtin_amdgcn_readfirstlane(atomicOr(&f.wflag[w], 0u));
    const bool fast = rx_fast_flag(fl) && *f.err == 0u;
    const RxDevWin& win = f.win;
    uint64_t* scr = f.scratch + ((size_t)w << win.words_lg);
    uint64_t r = 0, cur = 0, lo = 1, hi = 0, cur0 = 0;
    if (fast) {
        cur0 = win.cur[w];
        cur = f.curnew[w];
        lo = f.exit_lo[w];
        hi = f.exit_hi[w];
    }
    const uint64_t len = win.length, mask = len - 1u;
    const uint32_t nb = len < 64u ? (uint32_t)len : 64u;
    const uint64_t base = (cur >= len && cur - len > cur0) ? cur - len : cur0;
    const uint64_t ehi = min(hi, cur0);
    uint64_t* bits = win.bits + ((size_t)w << win.words_lg);
    for (uint32_t q = lane; q < win.words; q += 64u) {
        const uint64_t s = atomicExch(reinterpret_cast<unsigned long long*>(scr + q), 0ull);
        if (fast) {
            const uint64_t q0 = (uint64_t)q * 64u;
            const uint64_t clear = rx_ring_mask(q0, nb, (base + 1u) & mask, cur - base, len);
            const uint64_t leaving = ehi >= lo ? rx_ring_mask(q0, nb, lo & mask, ehi - lo + 1u, len) : 0ull;
            const uint64_t old = bits[q];
            bits[q] = (old & ~clear) | s;
            r += (uint32_t)__popcll(old & leaving);
        }
    }
    if (!fast) return;  // (wave-uniform)
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    if (lane == 0) {
        const uint64_t recv = atomicAdd(reinterpret_cast<unsigned long long*>(f.recv + w), 0ull);
        const uint64_t exits = hi >= lo ? hi - lo + 1u : 0u;
        win.lost[w] += (int64_t)(exits - recv - r);
        win.cur[w] = cur;
    }
}

// Take k settled packets off window w's pending count; the wave that reaches zero finishes w (every
// lane calls it with the same w and k; its own stores and atomics are complete).
__device__ __forceinline__ void rx_fold_release(const RxFold& f, uint32_t w, uint32_t k) {
    uint32_t last = 0;
    if (__lane_id() == 0) last = atomicSub(&f.pending[w], k) == k;
    if (__shfl(last, 0)) rx_fold_finish(f, w);
}

__device__ __forceinline__ void rx_wg_init(RxWgTab& t, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < kRxWgSlots; i += nthreads) {
        t.w[i] = ~0u;
        t.n[i] = 0;
    }
}

// One open wave's verdicts (every lane calls it; `holder` lanes hold the status st of packet i):
// the verdict at i, the counter into the scratch bitmap when it stays in the final window or into
// the received count when it leaves it — one atomic per (wave, window, word), not one per packet
// (one tunnel's batch would serialise tens of thousands of atomics on one address) — and the count
// per window into the workgroup's table.
__device__ __noinline__ void rx_fold_settle(const RxFold& f, RxWgTab& t, int32_t* status, uint32_t i, int32_t st,
                                            bool holder) {
    const uint32_t lane = __lane_id();
    uint32_t w = f.win.count;
    uint64_t c = 0, cur = 0, lo = 1, hi = 0;
    bool ok = false;
    if (holder) {
        w = f.keyw[i];
        c = f.ctr[i];
        f.verdict[i] = st;
        status[i] = st;
        ok = st == NEB_STATUS_OK;
        if (!ok) {
            atomicOr(&f.wflag[w], kRxSlow);
            f.need_host[0] = 1u;  // (pinned host word)
        }
        cur = f.curnew[w];
        lo = f.exit_lo[w];
        hi = f.exit_hi[w];
    }
    const uint64_t len = f.win.length;
    const bool in_final = ok && (cur < len || c > cur - len);
    const bool leaves = ok && c >= lo && c <= hi;
    const uint64_t p = c & (len - 1u);
    const uint64_t wkey = in_final ? (((uint64_t)w << 32) | (p >> 6)) : ~0ull;
    uint64_t pending = __ballot(in_final);
    while (pending) {
        const uint32_t leader = __builtin_ctzll(pending);
        const uint64_t lk = __shfl(wkey, (int)leader);
        const bool mine = in_final && wkey == lk;
        uint64_t b = mine ? 1ull << (p & 63) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) b |= __shfl_xor(b, o);
        if (lane == leader)
            atomicOr(reinterpret_cast<unsigned long long*>(f.scratch + ((size_t)w << f.win.words_lg) + (p >> 6)), b);
        pending &= ~__ballot(mine);
    }
    uint64_t pend2 = __ballot(leaves);
    while (pend2) {
        const uint32_t leader = __builtin_ctzll(pend2);
        const uint32_t lw = __shfl(w, (int)leader);
        const uint64_t same = __ballot(leaves && w == lw);
        if (lane == leader) atomicAdd(reinterpret_cast<unsigned long long*>(f.recv + w), (unsigned long long)__popcll(same));
        pend2 &= ~same;
    }
    uint64_t todo = __ballot(holder);
    while (todo) {
        const uint32_t leader = __builtin_ctzll(todo);
        const uint32_t lw = __shfl(w, (int)leader);
        const uint64_t same = __ballot(holder && w == lw);
        const uint32_t k = (uint32_t)__popcll(same);
        uint32_t full = 0;
        if (lane == leader) {  // the window's slot in the table (open addressing), or none left
            full = 1;
            for (uint32_t q = 0, h = lw % kRxWgSlots; q < kRxWgSlots; q++, h = (h + 1u) % kRxWgSlots) {
                const uint32_t o = atomicCAS(&t.w[h], ~0u, lw);
                if (o == ~0u || o == lw) {
                    atomicAdd(&t.n[h], k);
                    full = 0;
                    break;
                }
            }
        }
        if (__shfl(full, (int)leader)) {  // no room: this wave releases its packets itself
            // its bitmap and count atomics complete first (CDNA's vmcnt counts stores and atomics)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            rx_fold_release(f, lw, k);
        }
        todo &= ~same;
    }
}

// The end of an open workgroup (every thread, after its last packet): once every wave's stores and
// atomics are complete, each counted window's packets come off its pending count, wave by wave.
__device__ __forceinline__ void rx_wg_flush(const RxFold& f, RxWgTab& t, uint32_t tid, uint32_t nthreads) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t wave = tid >> 6, nwaves = nthreads >> 6;
    for (uint32_t h = wave; h < kRxWgSlots; h += nwaves) {
        const uint32_t w = t.w[h];
        if (w != ~0u) rx_fold_release(f, w, t.n[h]);
    }
}

}  // namespace neb

extern "C" hipError_t neb_rxdev_plan(const neb_desc* d_desc, uint32_t n, const neb::RxDevWin* win,
                                     const neb::RxDevWs* ws, int32_t* d_status, hipStream_t s);
extern "C" hipError_t neb_rxdev_gather(const neb_desc* d_desc, uint32_t n, const neb::RxDevWs* ws, hipStream_t s);
// readOutsidePackets (outside.go:30-114) for one wire packet, up to the decrypt: returns
// NEB_STATUS_OK with *d describing the Decrypt (header as AAD, in place) or the VerifyRelay (GMAC
// over packet[:len-16]), or the status the packet ends with. h: the first 16 bytes (read only when
// len >= 16). Shared by the host (window.cpp) and the device (rx_wire_kernel) forms.
__host__ __device__ inline uint32_t neb_rx_len(const neb_rx_packet& p) { return p.len & ~NEB_RX_OWN_SOURCE; }
__host__ __device__ inline int32_t neb_rx_wire_gate(const uint8_t* h, const neb_rx_packet& p, neb_desc* d) {
    const uint32_t len = neb_rx_len(p);
    if (len < 16u) return NEB_STATUS_INVALID;  // h.Parse: ErrHeaderTooShort (header.go:144-146)
    const uint32_t ver = h[0] >> 4, type = h[0] & 15u, sub = h[1];
    if (ver != 1u) return NEB_STATUS_INVALID;  // header.Version (outside.go:49-55)
    // IsValidSubType (header.go:192-205): Message 0/1, Handshake 0 (IXPSK0), Test 0/1, RecvError,
    // LightHouse, CloseTunnel, Control 0
    const bool valid = (type == 1u || type == 4u) ? sub <= 1u : (type == 0u || (type >= 2u && type <= 6u)) && sub == 0u;
    if (!valid) return NEB_STATUS_INVALID;
    // the caller's double-encryption check (outside.go:66-74: not relayed, UDP source inside the
    // node's own VPN networks), which needs the source address the batch does not carry
    if (p.len & NEB_RX_OWN_SOURCE) return NEB_STATUS_INVALID;
    if (type == 0u || type == 2u) return NEB_STATUS_NOT_MESSAGE;  // handshake, recv error (outside.go:83-89)
    if (p.key_id == NEB_KEYS_MIXED) return NEB_STATUS_BAD_KEY;    // no hostinfo (outside.go:100-106)
    if (len < 32u) return NEB_STATUS_INVALID;                     // header.Len + Overhead (outside.go:108-114)
    uint64_t c = 0;
    for (int i = 8; i < 16; i++) c = c << 8 | h[i];
    d->counter = c;
    d->key_id = p.key_id;
    d->flags = 0;
    d->aad_off = p.off;
    if (type == 1u && sub == 1u) {  // VerifyRelay: AD = everything but the trailing tag
        d->aad_len = len - 16u;
        d->src_off = d->dst_off = p.off + len - 16u;
        d->len = 0;
    } else {  // Decrypt: in place after the header
        d->aad_len = 16u;
        d->src_off = d->dst_off = p.off + 16u;
        d->len = len - 32u;
    }
    return NEB_STATUS_OK;
}

// Byte spans between two device buffers, one wave per span (the exact receive pass's speculative
// opens: packets copied out of the arena into a scratch buffer, plaintext copied back for the ones
// the windows accept, zeros for the ones that pass their window but fail their tag). src == NULL
// writes zeros.
struct neb_span {
    uint64_t src, dst;
    uint32_t len, pad;
};
extern "C" hipError_t neb_rxdev_spans(const uint8_t* src, uint8_t* dst, const neb_span* d_spans, uint32_t n,
                                      hipStream_t s);
// the gate over a device batch of wire packets: descriptors (refused packets: a harmless empty
// descriptor with key NEB_KEYS_MIXED, so the receive leaves them alone) and the gate's statuses
extern "C" hipError_t neb_rxdev_wire(const neb_rx_packet* d_pk, uint32_t n, const uint8_t* d_arena, neb_desc* d_desc,
                                     int32_t* d_gate, hipStream_t s);
// status[i] = gate[i] wherever the gate refused the packet
extern "C" hipError_t neb_rxdev_wire_fix(const int32_t* d_gate, int32_t* d_status, uint32_t n, hipStream_t s);
