// rxwin.hpp — device replay windows and the workspace of the device batched receive (rxwin.hip),
// shared with window.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/nebula_aead.h"
#include "sched.hpp"

namespace neb {

// A window whose counters come this close to 2^64 takes the sequential path (no uint64 wrap in
// the parallel form). No sender reaches it: counters stop at RejectAfterMessages = 2^64 - 2^40 - 1,
// and 2^62 messages is far beyond any tunnel's life; forged counters may, and are then exact too.
constexpr uint64_t kRxRiskyCounter = 1ull << 62;
enum : uint32_t { kRxTouched = 1u, kRxRisky = 2u, kRxSlow = 4u };
// run-order elements per workgroup of the scan and admission kernels (one per thread: their
// per-packet chains of dependent loads and atomics are latency-bound)
constexpr uint32_t kRxThreads = 256, kRxItems = 1, kRxBlock = kRxThreads * kRxItems;
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

// The mixed-key open's binning (sched_body.hpp), run by extra workgroups of the plan's own launches
// instead of three launches of its own: the histogram beside the keys, the allocation beside the
// first sort pass, the scatter beside the second (a launch of its own after a one-pass sort). The
// passes depend only on the descriptors and on each other, so each role waits on nothing inside its
// launch. The scan then marks every packet it did not admit as skipped in sorted[] (kSortedSkip),
// so the open runs the plain chunk kernel. on = 0: no binning (one key, ChaCha20-Poly1305, or a batch large
// enough for sub-bins: the open bins it itself).
struct RxBin {
    SchedWs ws;
    uint32_t on;
    uint32_t max_keys;
    uint32_t hist_blocks, alloc_blocks, scatter_blocks;
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
    // the generation of the last batch whose packets named more than one window (written by the
    // keys kernel); any other value lets the sort passes write the identity order (one window)
    uint32_t* mixed;
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
    if (ws) *ws = w;
    return off;
}

}  // namespace neb

extern "C" hipError_t neb_rxdev_plan(const neb_desc* d_desc, uint32_t n, const neb::RxDevWin* win,
                                     const neb::RxDevWs* ws, int32_t* d_status, const neb::RxBin* bin,
                                     hipStream_t s);
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
// After the open (which ran the admitted packets only, ws->adm, writing their statuses): verdicts,
// the admitted counters into the windows, and the finish of every window whose packets all verified.
extern "C" hipError_t neb_rxdev_finish(uint32_t n, const neb::RxDevWin* win, const neb::RxDevWs* ws,
                                       int32_t* d_status, hipStream_t s);
