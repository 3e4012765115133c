// engine.cpp — host side of the C ABI in include/nebula_aead.h.
//
// Owns one HIP device per engine: its stream, the device key table, pinned staging for the
// per-packet CipherState calls, and the double-buffered host-resident batch pipeline. All packet
// arithmetic runs in the gfx950 kernels (aes_gcm.hip, chacha_poly.hip); there is no CPU path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <cstring>
#include <cxxabi.h>
#include <cstdlib>
#include <climits>
#include <dlfcn.h>
#include <linux/futex.h>
#include <mutex>
#include <new>
#include <string>
#include <sys/syscall.h>
#include <thread>
#include <type_traits>
#include <unistd.h>
#include <vector>

#include "../../include/nebula_aead.h"
#include "hip_guard.hpp"
#include "knobs.hpp"
#include "host_common.hpp"
#include "layout.hpp"
#include "rxwin.hpp"
#include "sched.hpp"
#include "timing.hpp"
#include "tx.hpp"

// n keys (32 B each, mapped host memory) into the records of key slots slots[0..n): one launch
extern "C" hipError_t neb_gcm_key_setup(const uint8_t* keys, const uint32_t* slots, uint32_t n, uint32_t* table,
                                        hipStream_t s);
extern "C" hipError_t neb_chacha_key_setup(const uint8_t* keys, const uint32_t* slots, uint32_t n, uint32_t* table,
                                           hipStream_t s);
extern "C" hipError_t neb_fence_keys(const neb_desc* in, neb_desc* out, uint32_t n, const uint8_t* bad,
                                     uint32_t nbad, hipStream_t s);
extern "C" hipError_t neb_gcm_batch_single(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                           const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                           int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                           int hdr_from_dst, hipEvent_t stop, const uint8_t* rx);
extern "C" hipError_t neb_gcm_one(int open, const uint8_t* aad, uint32_t aad_len, const uint8_t* in, uint32_t in_len,
                                  uint32_t len, uint64_t counter, uint8_t* out, int32_t* status, const uint32_t* d_keys,
                                  uint32_t max_keys, uint32_t key, hipStream_t s);
extern "C" hipError_t neb_copy_span(void* dst, const void* src, size_t bytes, hipStream_t s);
extern "C" hipError_t neb_copy_desc(neb_desc* dst, const neb_desc* src, uint32_t n, hipStream_t s);
extern "C" hipError_t neb_gcm_one_batch(int open, const neb_desc* descs, int32_t* status, uint8_t* slots, uint32_t n,
                                        const uint32_t* d_keys, uint32_t max_keys, hipStream_t s);
extern "C" hipError_t neb_chacha_one(int open, const uint8_t* aad, uint32_t aad_len, const uint8_t* in,
                                     uint32_t in_len, uint32_t len, uint64_t counter, uint8_t* out, int32_t* status,
                                     const uint32_t* d_keys, uint32_t max_keys, uint32_t key, hipStream_t s);
extern "C" hipError_t neb_gcm_batch_chunked(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                            const uint32_t* d_keys, uint32_t max_keys, int32_t* d_status,
                                            const uint32_t* d_sorted, const uint4* d_chunks,
                                            uint32_t* d_counters, uint32_t max_chunks,
                                            int cu_count, hipStream_t s, int hdr_from_dst, hipEvent_t stop,
                                            const uint8_t* rx);
extern "C" hipError_t neb_gcm_probe(void);
extern "C" uint32_t neb_gcm_single_slots(uint32_t n, int cu_count, int open, int hdr_from_dst);
#ifndef NEB_TX_CSUM_SEAL
#define NEB_TX_CSUM_SEAL 1  // 0: the segment kernel sums every checksum (A/B)
#endif
extern "C" hipError_t neb_chacha_batch(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                       const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                       int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                       int hdr_from_dst, hipEvent_t stop, const uint8_t* rx);

// The stream a workspace's `done` event was last recorded on. A batch on that same stream is
// ordered after it already and skips the cross-stream wait (a barrier packet that cost ≈ 5 µs between
// kernels). The handle alone does not name a stream: one destroyed with work still pending is
// released when the work ends, and a stream created meanwhile may get its address; so the identity
// is the handle together with HIP's per-stream id (hipStreamGetId, HIP >= 7.1, looked up at run time:
// a process may run an older HIP runtime, as PyTorch's wheel does). Without it the handle alone is
// the identity, and a caller must not destroy a stream while the engine's batches on it are pending
// (streams).
struct StreamTag {
    using GetId = hipError_t (*)(hipStream_t, unsigned long long*);
    hipStream_t h = nullptr;
    unsigned long long id = 0;
    bool valid = false;
    static unsigned long long id_of(hipStream_t s) {
        static const GetId get = (GetId)dlsym(RTLD_DEFAULT, "hipStreamGetId");
        unsigned long long v = 0;
        return get && get(s, &v) == hipSuccess ? v : 0ull;
    }
    bool same(hipStream_t s) const { return valid && h == s && id_of(s) == id; }
    void set(hipStream_t s) {
        h = s;
        id = id_of(s);
        valid = true;
    }
};

// Device workspace of the mixed-key scheduler (sched.hpp). One per engine; a batch waits on the
// previous user's event before reusing it, so batches on different streams never overlap in it.
struct SchedSpace {
    uint8_t* mem = nullptr;
    size_t bytes = 0;
    uint32_t n_cap = 0;
    neb::SchedWs ws{};
    hipEvent_t done = nullptr;
    StreamTag last;  // the stream `done` was last recorded on
    bool dirty = true;  // the bin counts need a clear (new buffer, or a batch that failed to launch)
    std::mutex mu;
};

namespace {

constexpr size_t kStageMin = 1 << 16;
// The staged host pipeline (batch_host, round 6): chunks of kPipeChunkPkts packets through
// kPipeSlots device buffers, with the copies in, the kernels and the copies back on three streams
// of their own, chained by events: chunk k + 1's copy-in then runs beside chunk k - 1's copy-back
// (PCIe carries both directions at once: 56 GB/s each alone, 96 GB/s together on this box).
// Chunks ramp up from kPipeFirst packets (doubling) to kPipeChunkPkts and back down at the end, so the
// first copy-in and the last copy-back, which run with nothing beside them, are short. A/B on C2
// (profiles/r6/host/): chunks of 4096 / 8192 / 12288 / 16384 / 32768 packets 23.9 / 26.6 / 32.6-33.2 /
// 32.6 / 28.5 GiB/s; a 16384-packet copy-in runs 395 µs alone and 520 µs beside a copy-back (42 + 51
// GB/s), and the first and last of each call ran alone for ≈ 0.9 of its 2.7 ms.
constexpr int kPipeSlots = 4;
#ifndef NEB_PIPE_CHUNK
#define NEB_PIPE_CHUNK 16384
#endif
#ifndef NEB_PIPE_FIRST
#define NEB_PIPE_FIRST 4096
#endif
constexpr uint32_t kPipeChunkPkts = NEB_PIPE_CHUNK;  // packets per staged host chunk at most
constexpr uint32_t kPipeFirst = NEB_PIPE_FIRST;      // the first and last chunks' packets

// chunk sizes for a batch of n packets: kPipeFirst, 2 kPipeFirst, ... up to kPipeChunkPkts at both
// ends (while the rest still holds 4x the next size), full chunks between
std::vector<uint32_t> pipe_plan(uint32_t n) {
    std::vector<uint32_t> head, plan;
    uint32_t rem = n;
    for (uint32_t s = kPipeFirst; s < kPipeChunkPkts && rem >= 4u * s; s *= 2u) {
        head.push_back(s);
        rem -= 2u * s;
    }
    plan = head;
    for (; rem; rem -= std::min(rem, kPipeChunkPkts)) plan.push_back(std::min(rem, kPipeChunkPkts));
    plan.insert(plan.end(), head.rbegin(), head.rend());
    return plan;
}

struct PipeSlot {
    uint8_t* d_buf = nullptr;
    size_t d_cap = 0;
    neb_desc* h_desc = nullptr;  // pinned: the chunk's rebased descriptors
    neb_desc* d_desc = nullptr;  // their device copy, which the kernels read
    int32_t* h_status = nullptr; // pinned, mapped: the kernels write it in place
    int32_t* user_status = nullptr;
    uint32_t user_begin = 0, count = 0;
    uint64_t lo = 0, hi = 0;        // arena span of the chunk in flight (count > 0)
    hipEvent_t in_done = nullptr;   // the chunk's copies in are done (the kernel waits for it)
    hipEvent_t k_done = nullptr;    // its kernel is done (the copies back wait for it)
    hipEvent_t done = nullptr;      // its span and statuses are back (the slot is free)
    bool back_pending = false;      // statuses taken at k_done; the copy back may still read d_buf
};
struct Pipe {
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    PipeSlot slot[kPipeSlots];
    SchedSpace* sched = nullptr;  // the compute stream's mixed-key workspace
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }


}  // namespace


namespace {

// Host batch path: NEB_HOST_MODE = "zc" (the kernels on the mapped arena, the default) or "dma"
// (hipMemcpyAsync staging); NEB_HOST_STAGED=1 is the older name of "dma". Measured on one MI355X
// (C2 seal+open, 64 Ki x 1300 B): zero-copy 28.4 GiB/s against 23.9 for DMA staging.
enum HostMode { kHostZeroCopy, kHostDma };
HostMode host_mode() {  // NEB_KNOB_HOST_MODE, read per batch, so a process can switch between batches
    return neb::knob(NEB_KNOB_HOST_MODE) == 1 ? kHostDma : kHostZeroCopy;
}

}  // namespace

// Device workspace of the transmit batch (tx.hpp) plus device staging for its host-memory form.
struct TxSpace {
    uint8_t* mem = nullptr;
    size_t bytes = 0;
    uint32_t n_cap = 0, tun_cap = 0, wire_cap = 0;
    neb::TxWs ws{};
    hipEvent_t done = nullptr;
    StreamTag last;  // the stream `done` was last recorded on
    uint8_t* d_io = nullptr;  // neb_tx_seal_batch_host staging
    size_t io_cap = 0;
    std::mutex mu;
};

// Per-packet CipherState calls (neb_encrypt_danger / neb_decrypt_danger) and key installs share a
// fixed pool of kPktSlots slots per engine: a stream and pinned, mapped staging the kernel reads
// and writes in place ([desc 64 B | status 64 B | aad | payload + tag]). The box grants a process 4
// hardware queues, so more streams only queue behind each other in the driver. A call takes a free
// slot, or joins one FIFO of waiters and sleeps until a finishing call hands it its slot directly
// (one wake-up per hand-off, nobody spins): the wait of a call is bounded by the calls ahead of
// it, however many threads call. (Round 3 gave every calling OS thread its own slot and stream,
// kept until the engine died: the count grew with the threads cgo ever used, a thread alternating
// over more than 8 engines leaked one per call, and at 64 threads p99 was 100x p50.)
constexpr uint32_t kPktSlots = 4;
struct PktSlot {
    hipStream_t stream = nullptr;
    uint8_t* h = nullptr;
    size_t cap = 0;
};
struct PktWaiter {
    std::condition_variable cv;
    PktSlot* got = nullptr;
};
struct PktPool {
    std::mutex mu;
    PktSlot slot[kPktSlots];
    PktSlot* free_[kPktSlots] = {};
    uint32_t nfree = 0;
    std::deque<PktWaiter*> waiters;
    std::atomic<uint64_t> calls{0}, waits{0};
};
// Per-packet AES-256-GCM calls that arrive while kPktSlots launches are in flight (round 6): they join
// one pinned batch of up to kCombMax requests, which its first request (the leader) launches as a
// whole (gcm_one_batch_kernel) as soon as one of the launches ahead completes; the leader polls
// every status, wakes the others, and each copies its own result out. A call that finds a launch
// free launches alone as before (the packet in the kernel arguments), so up to kPktSlots threads see
// no change; past that the batches grow with the offered load.
constexpr uint32_t kCombMax = 32;
constexpr uint32_t kCombSlot = 2048u + 64u;  // aes_gcm.hip kCombSlot: AAD | payload (+ tag) of one request
constexpr size_t kCombDescOff = 0, kCombStatusOff = 2048, kCombSlotsOff = 4096;
constexpr size_t kCombBytes = kCombSlotsOff + (size_t)kCombMax * kCombSlot;
struct CombBatch {
    uint8_t* h = nullptr;  // pinned, mapped: descriptors | statuses | slots
    uint32_t n = 0;        // requests joined
    int alg = 0, open = 0;
    bool launched = false;  // (PktComb::mu)
    hipStream_t stream = nullptr;
    std::atomic<uint32_t> left{0};  // requests whose owner has not copied its result out yet
    // The leader saw every status: the owners may copy out. A futex word of the batch's own, so the
    // owners wake without queueing on a mutex (64 threads on a 16-CPU share: p99 23 ms when they
    // woke through the engine's combiner mutex).
    std::atomic<uint32_t> done{0};
    bool failed = false;  // written before done's release
    void finish(bool f) {
        failed = f;
        done.store(1, std::memory_order_release);
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&done), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
    }
    bool wait() {  // the failure flag
        while (!done.load(std::memory_order_acquire))
            syscall(SYS_futex, reinterpret_cast<uint32_t*>(&done), FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
        return failed;
    }
    neb_desc* desc() const { return reinterpret_cast<neb_desc*>(h + kCombDescOff); }
    int32_t* status() const { return reinterpret_cast<int32_t*>(h + kCombStatusOff); }
    uint8_t* slots() const { return h + kCombSlotsOff; }
};
struct PktComb {
    std::mutex mu;
    uint32_t inflight = 0;          // launches (alone or combined) not yet complete, at most pkt_inflight()
    uint32_t solo = 0;              // of them alone (each holds a pool slot), at most kPktSlots
    std::condition_variable launch_cv;  // a launch completed (the leaders of gathering batches wait)
    CombBatch* open[2][2] = {};     // accepting requests: [AES-GCM / ChaCha20][seal / open]
    std::vector<CombBatch*> free_, all;
    uint32_t next = 0;              // the per-packet pool's streams carry the combined launches in turn
    std::atomic<uint64_t> launches{0}, combined{0};
};
struct KeyUse {
    hipStream_t s;
    hipEvent_t ev;
};

struct neb_engine {
    int device = 0;
    int cu_count = 0;
    hipStream_t stream = nullptr;
    uint32_t max_keys = 0;
    uint32_t* d_keys = nullptr;
    std::vector<int> slot_alg;  // 0 = free, -1 = reserved by an install in progress
    // Install id of the key in each slot (0 = none): unique per neb_cipher_create /
    // neb_cipher_create_batch key, shared by the engines of one neb_cipher_create_multi. Batches
    // over several engines check that every shard's engine holds the same install as engine 0.
    std::vector<uint64_t> slot_tag;
    uint64_t key_epoch = 0;  // bumped by every install and destroy (under key_mu)
    std::mutex key_mu;
    uint64_t installs = 0;

    PktPool pkt;  // per-packet calls and key installs
    PktComb comb; // per-packet calls combined into one launch

    // Asynchronous batches still queued when a key is destroyed: per key slot, the last
    // single-key batch the engine launched on each stream, and the last mixed-key batch per
    // stream (its keys are only known on the device). neb_cipher_destroy waits for those events
    // only, not for the device.
    std::mutex use_mu;
    std::vector<std::vector<KeyUse>> key_use;
    std::vector<KeyUse> mixed_use;

    std::mutex pipe_mu;
    Pipe pipe;
    // zero-copy host batches: device copies of pageable descriptors / statuses
    neb_desc* zc_desc = nullptr;
    int32_t* zc_status = nullptr;
    uint32_t zc_cap = 0;

    SchedSpace sched;
    TxSpace tx;

    // Pipelined batched receive (window.cpp): each chunk's open on a stream (and mixed-key
    // workspace) of its own, so consecutive chunks overlap on the device; descriptors and statuses
    // staged in pinned memory; one event per chunk.
    struct RxSlot {
        hipStream_t stream = nullptr;
        hipEvent_t ev = nullptr;
        SchedSpace* sched = nullptr;
    };
    struct RxSpace {
        std::mutex mu;  // held from neb_rx_pipe_begin to neb_rx_pipe_end
        neb_desc* h_desc = nullptr;
        int32_t* h_status = nullptr;
        neb_desc* d_desc = nullptr;
        int32_t* d_status = nullptr;
        uint32_t cap = 0;
        std::vector<RxSlot> slot;
    } rx;

};

struct neb_cipher {
    neb_engine* e;
    uint32_t key_id;
    int alg;
    uint64_t tag;  // neb_engine::slot_tag of the install
};

static thread_local char g_last_error[256] = "";

// neb_set_knob: the environment's values, read once on first use
static std::atomic<int64_t> g_knobs[NEB_KNOB_COUNT];
int64_t neb::knob(int k) {
    static const bool init = [] {
        const char* hm = std::getenv("NEB_HOST_MODE");
        g_knobs[NEB_KNOB_HOST_MODE] = (std::getenv("NEB_HOST_STAGED") || (hm && !std::strcmp(hm, "dma"))) ? 1 : 0;
        const char* sb = std::getenv("NEB_SUB_BINS_FROM");
        g_knobs[NEB_KNOB_SUB_BINS_FROM] = sb ? (int64_t)std::strtoull(sb, nullptr, 10) : (int64_t)neb::kSubBinsFrom;
        const char* mg = std::getenv("NEB_SINGLE_MAX_GRID");
        g_knobs[NEB_KNOB_SINGLE_MAX_GRID] = mg ? std::atoll(mg) : 0;
        g_knobs[NEB_KNOB_RX_STRICT] = std::getenv("NEB_RXDEV_STRICT") ? 1 : 0;
        const char* tb = std::getenv("NEB_TILE_BINS_FROM");
        g_knobs[NEB_KNOB_TILE_BINS_FROM] = tb ? (int64_t)std::strtoull(tb, nullptr, 10) : (int64_t)neb::kTileBinsFrom;
        const char* sb2 = std::getenv("NEB_SMALL_BATCH");
        g_knobs[NEB_KNOB_SMALL_BATCH] = sb2 ? (int64_t)std::strtoull(sb2, nullptr, 10) : (int64_t)neb::kSmallBatchPerWave;
        const char* fg = std::getenv("NEB_FRONT_GROUPS");
        g_knobs[NEB_KNOB_FRONT_GROUPS] = fg ? (int64_t)std::strtoull(fg, nullptr, 10) : (int64_t)neb::kSmallBatchGroups;
        return true;
    }();
    (void)init;
    return g_knobs[k].load(std::memory_order_relaxed);
}
thread_local neb::KernelTiming neb::g_kernel_timing;  // timing.hpp: armed by neb_time_next_kernel
thread_local const void* neb::g_timed_kernel = nullptr;

static void set_error(const char* where, hipError_t err) {
    std::snprintf(g_last_error, sizeof g_last_error, "%s: %s (%d)", where, hipGetErrorString(err), (int)err);
}

#define HIP_TRY(x)                                  \
    do {                                            \
        hipError_t err_ = (x);                      \
        if (err_ != hipSuccess) {                   \
            set_error(#x, err_);                    \
            return NEB_ERR_HIP;                     \
        }                                           \
    } while (0)

// Exclusive use of one slot of e's per-packet pool for the lifetime of the lease (PktPool).
class PktLease {
  public:
    explicit PktLease(PktPool& p) : p_(p) {
        std::unique_lock<std::mutex> lk(p.mu);
        p.calls.fetch_add(1, std::memory_order_relaxed);
        if (p.nfree) {
            s_ = p.free_[--p.nfree];
            return;
        }
        p.waits.fetch_add(1, std::memory_order_relaxed);
        PktWaiter w;
        p.waiters.push_back(&w);
        w.cv.wait(lk, [&] { return w.got != nullptr; });
        s_ = w.got;
    }
    ~PktLease() {
        std::lock_guard<std::mutex> g(p_.mu);
        if (p_.waiters.empty()) {
            p_.free_[p_.nfree++] = s_;
            return;
        }
        PktWaiter* w = p_.waiters.front();  // FIFO: the longest waiter gets the slot
        p_.waiters.pop_front();
        w->got = s_;
        w->cv.notify_one();
    }
    PktLease(const PktLease&) = delete;
    PktLease& operator=(const PktLease&) = delete;
    PktSlot* operator->() const { return s_; }
    // room for `bytes` of staging (the slot is exclusively ours). A per-packet call returns as soon as
    // its kernel has published the status word, so the previous lease's kernel may still be draining
    // on the slot's stream: wait for it before the buffer it writes is freed.
    bool reserve(size_t bytes) {
        if (bytes <= s_->cap) return true;
        if (s_->h) {
            const hipError_t err = hipStreamSynchronize(s_->stream);
            if (err != hipSuccess) {
                set_error("PktLease::reserve", err);
                return false;
            }
            hipHostFree(s_->h);
        }
        s_->h = nullptr;
        s_->cap = 0;
        const size_t cap = std::max(kStageMin, align_up(bytes, 1 << 16));
        hipError_t err = hipHostMalloc((void**)&s_->h, cap, hipHostMallocDefault);
        if (err != hipSuccess) {
            set_error("hipHostMalloc", err);
            s_->h = nullptr;
            return false;
        }
        s_->cap = cap;
        return true;
    }

  private:
    PktPool& p_;
    PktSlot* s_ = nullptr;
};

// After an asynchronous batch is enqueued on stream s: remember it for neb_cipher_destroy (the
// key_hint's slot, or every slot for a mixed-key batch). Events skip the system-scope cache
// flush (timing-only markers would carry it for nothing).
static void note_use(neb_engine* e, uint32_t key_hint, hipStream_t s) {
    std::lock_guard<std::mutex> g(e->use_mu);
    std::vector<KeyUse>& v = key_hint == NEB_KEYS_MIXED ? e->mixed_use : e->key_use[key_hint];
    for (KeyUse& u : v)
        if (u.s == s) {
            (void)hipEventRecord(u.ev, s);
            return;
        }
    KeyUse u{s, nullptr};
    if (hipEventCreateWithFlags(&u.ev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return;
    (void)hipEventRecord(u.ev, s);
    v.push_back(u);
}

// The key-use event of (key_hint, s), created on first use, for a batch to bind to its last
// kernel (neb_gcm_batch_single's `stop`) instead of note_use's marker after it.
static hipEvent_t use_event(neb_engine* e, uint32_t key_hint, hipStream_t s) {
    std::lock_guard<std::mutex> g(e->use_mu);
    std::vector<KeyUse>& v = key_hint == NEB_KEYS_MIXED ? e->mixed_use : e->key_use[key_hint];
    for (KeyUse& u : v)
        if (u.s == s) return u.ev;
    KeyUse u{s, nullptr};
    if (hipEventCreateWithFlags(&u.ev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) return nullptr;
    v.push_back(u);
    return u.ev;
}

extern "C" {

NEB_API const char* neb_last_error(void) { return g_last_error; }

NEB_API int neb_time_next_kernel(void* start, void* stop) {
    if ((start == nullptr) != (stop == nullptr)) return NEB_ERR_INVALID;
    neb::g_kernel_timing = {(hipEvent_t)start, (hipEvent_t)stop};
    return NEB_OK;
}

NEB_API int neb_set_knob(int knob, int64_t value) {
    if (knob < 0 || knob >= NEB_KNOB_COUNT) return NEB_ERR_INVALID;
    neb::knob(knob);  // (the environment's values first, so a later first use does not overwrite this)
    g_knobs[knob].store(value, std::memory_order_relaxed);
    return NEB_OK;
}

NEB_API int64_t neb_get_knob(int knob) { return knob < 0 || knob >= NEB_KNOB_COUNT ? -1 : neb::knob(knob); }

NEB_API const char* neb_time_last_kernel(void) {
    static thread_local std::string name;
    if (!neb::g_timed_kernel) return "";
    const char* m = hipKernelNameRefByPtr(neb::g_timed_kernel, nullptr);
    if (!m) return "";
    int st = 0;
    char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
    name = st == 0 && d ? d : m;
    std::free(d);
    return name.c_str();
}

#ifndef NEB_BUILD_ID
#define NEB_BUILD_ID "unknown"
#endif
NEB_API const char* neb_build_id(void) { return NEB_BUILD_ID; }

NEB_API const char* neb_strerror(int rc) {
    switch (rc) {
        case NEB_OK: return "ok";
        case NEB_ERR_INVALID: return "invalid argument";
        case NEB_ERR_AUTH: return "cipher: message authentication failed";
        case NEB_ERR_EXHAUSTED: return "message counter exhausted";
        case NEB_ERR_NO_CIPHER: return "no cipher state available to encrypt";
        case NEB_ERR_SHORT_BUFFER: return "output buffer too small";
        case NEB_ERR_HIP: return "HIP runtime error";
        case NEB_ERR_NO_DEVICE: return "no usable gfx950 device";
        case NEB_ERR_NO_KEY_SLOT: return "key table full";
        default: return "unknown error";
    }
}

NEB_API int neb_engine_create(int device, uint32_t max_keys, neb_engine** out) {
    if (!out || max_keys == 0 || max_keys == NEB_KEYS_MIXED) return NEB_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    hipError_t err = hipGetDeviceCount(&ndev);
    if (err != hipSuccess) {
        set_error("hipGetDeviceCount", err);
        return NEB_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= ndev) {
        std::snprintf(g_last_error, sizeof g_last_error, "device %d out of range (%d devices)", device, ndev);
        return NEB_ERR_NO_DEVICE;
    }
    int cus = 0;
    DeviceGuard dg;
    if ((err = hipSetDevice(device)) != hipSuccess ||
        (err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) {
        set_error("hipSetDevice/hipDeviceGetAttribute", err);
        return NEB_ERR_NO_DEVICE;
    }
    // the library carries gfx950 code objects only: a device they do not load on is refused
    if ((err = neb_gcm_probe()) != hipSuccess) {
        set_error("gfx950 code object not loadable on this device", err);
        return NEB_ERR_NO_DEVICE;
    }
    neb_engine* e = new (std::nothrow) neb_engine();
    if (!e) return NEB_ERR_INVALID;
    e->device = device;
    e->cu_count = cus;
    e->max_keys = max_keys;
    e->slot_alg.assign(max_keys, 0);
    e->slot_tag.assign(max_keys, 0);
    e->key_use.resize(max_keys);
    bool ok = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc((void**)&e->d_keys, (size_t)max_keys * neb::kKeyRecBytes) == hipSuccess &&
              hipMemset(e->d_keys, 0, (size_t)max_keys * neb::kKeyRecBytes) == hipSuccess &&
              hipStreamSynchronize(nullptr) == hipSuccess;  // the null-stream memset, before any stream reads keys
    // The per-packet pool's streams: high priority, which HIP gives a hardware queue of its own each.
    // Streams of the default priority share the process's 4 queues, handed out in the order
    // 1 2 3 4 4 3 2 1 (tools/native/queue_map.cpp under rocprofv3): after the null stream and the
    // engine's stream the pool's 4 landed on 2 queues, and 4 threads' calls ran 2 kernels at a time
    // (round 6 trace, profiles/r6/percall/). NEB_PKT_PRIO=0: default priority (A/B).
    static const bool prio = [] {
        const char* v = std::getenv("NEB_PKT_PRIO");
        return !(v && v[0] == '0');
    }();
    int least = 0, greatest = 0;
    if (prio) (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    for (PktSlot& sl : e->pkt.slot) {
        ok = ok &&
             (prio ? hipStreamCreateWithPriority(&sl.stream, hipStreamNonBlocking, greatest)
                   : hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking)) == hipSuccess &&
             hipHostMalloc((void**)&sl.h, kStageMin, hipHostMallocDefault) == hipSuccess;
        if (ok) {
            sl.cap = kStageMin;
            e->pkt.free_[e->pkt.nfree++] = &sl;
        }
    }
    if (!ok) {
        set_error("engine allocation", hipGetLastError());
        neb_engine_destroy(e);
        return NEB_ERR_HIP;
    }
    *out = e;
    return NEB_OK;
}

NEB_API int neb_engine_destroy(neb_engine* e) {
    if (!e) return NEB_ERR_INVALID;
    DeviceGuard dg(e->device);
    if (e->stream) hipStreamSynchronize(e->stream);
    for (hipStream_t st : {e->pipe.h2d, e->pipe.comp, e->pipe.d2h})
        if (st) { hipStreamSynchronize(st); hipStreamDestroy(st); }
    for (CombBatch* b : e->comb.all) {
        if (b->h) hipHostFree(b->h);
        delete b;
    }
    for (auto& s : e->pipe.slot) {
        for (hipEvent_t ev : {s.in_done, s.k_done, s.done})
            if (ev) hipEventDestroy(ev);
        if (s.d_buf) hipFree(s.d_buf);
        if (s.h_desc) hipHostFree(s.h_desc);
        if (s.d_desc) hipFree(s.d_desc);
        if (s.h_status) hipHostFree(s.h_status);
    }
    if (SchedSpace* sp = e->pipe.sched) {
        if (sp->done) { hipEventSynchronize(sp->done); hipEventDestroy(sp->done); }
        if (sp->mem) hipFree(sp->mem);
        delete sp;
    }
    if (e->sched.done) { hipEventSynchronize(e->sched.done); hipEventDestroy(e->sched.done); }
    if (e->sched.mem) hipFree(e->sched.mem);
    if (e->tx.done) { hipEventSynchronize(e->tx.done); hipEventDestroy(e->tx.done); }
    if (e->tx.mem) hipFree(e->tx.mem);
    if (e->tx.d_io) hipFree(e->tx.d_io);
    for (auto& r : e->rx.slot) {
        if (r.stream) { hipStreamSynchronize(r.stream); hipStreamDestroy(r.stream); }
        if (r.ev) hipEventDestroy(r.ev);
        if (r.sched) {
            if (r.sched->done) { hipEventSynchronize(r.sched->done); hipEventDestroy(r.sched->done); }
            if (r.sched->mem) hipFree(r.sched->mem);
            delete r.sched;
        }
    }
    if (e->rx.h_desc) hipHostFree(e->rx.h_desc);
    if (e->rx.h_status) hipHostFree(e->rx.h_status);
    if (e->rx.d_desc) hipFree(e->rx.d_desc);
    if (e->rx.d_status) hipFree(e->rx.d_status);
    if (e->zc_desc) hipFree(e->zc_desc);
    if (e->zc_status) hipFree(e->zc_status);
    if (e->d_keys) hipFree(e->d_keys);
    for (PktSlot& sl : e->pkt.slot) {
        if (sl.stream) { hipStreamSynchronize(sl.stream); hipStreamDestroy(sl.stream); }
        if (sl.h) hipHostFree(sl.h);
    }
    for (auto& v : e->key_use)
        for (KeyUse& u : v) hipEventDestroy(u.ev);
    for (KeyUse& u : e->mixed_use) hipEventDestroy(u.ev);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
    return NEB_OK;
}

NEB_API int neb_engine_info(const neb_engine* e, int* device, uint32_t* max_keys, uint32_t* key_record_bytes) {
    if (!e) return NEB_ERR_INVALID;
    if (device) *device = e->device;
    if (max_keys) *max_keys = e->max_keys;
    if (key_record_bytes) *key_record_bytes = neb::kKeyRecBytes;
    return NEB_OK;
}

NEB_API int neb_engine_stats(const neb_engine* e, uint64_t stats[4]) {
    if (!e || !stats) return NEB_ERR_INVALID;
    stats[0] = kPktSlots;
    stats[1] = e->pkt.calls.load(std::memory_order_relaxed);
    stats[2] = e->pkt.waits.load(std::memory_order_relaxed);
    std::lock_guard<std::mutex> g(const_cast<neb_engine*>(e)->key_mu);
    stats[3] = e->installs;
    return NEB_OK;
}

NEB_API const char* neb_cipher_name(int alg) {
    return alg == NEB_ALG_AESGCM ? "AESGCM" : alg == NEB_ALG_CHACHAPOLY ? "ChaChaPoly" : nullptr;
}

static std::atomic<uint64_t> g_key_tag{1};

// Reserve the n lowest free slots of e (caller holds e->key_mu); false if fewer are free.
static bool reserve_slots(neb_engine* e, uint32_t n, uint32_t* slots) {
    uint32_t k = 0;
    for (uint32_t s = 0; s < e->max_keys && k < n; s++)
        if (e->slot_alg[s] == 0) slots[k++] = s;
    if (k < n) return false;
    for (uint32_t i = 0; i < n; i++) e->slot_alg[slots[i]] = -1;
    return true;
}

// Key install of n keys into the reserved slots slots[0..n), one launch: the keys and slot numbers go
// through one slot of the per-packet pool (pinned, mapped: the setup kernel reads them there), each
// workgroup clears its record and installs one key, and the staged key bytes are wiped afterwards.
// On failure the records are cleared again, so no slot is left holding a half-written record
// whose algorithm tag a batch could accept.
static int install_records(neb_engine* e, int alg, const uint8_t* keys, const uint32_t* slots, uint32_t n) {
    DeviceGuard dg(e->device);
    PktLease sl(e->pkt);
    const size_t kb = align_up((size_t)n * 32u, 64);
    if (!sl.reserve(kb + (size_t)n * 4u)) return NEB_ERR_HIP;
    std::memcpy(sl->h, keys, (size_t)n * 32u);
    std::memcpy(sl->h + kb, slots, (size_t)n * 4u);
    hipError_t err = alg == NEB_ALG_AESGCM
                         ? neb_gcm_key_setup(sl->h, (const uint32_t*)(sl->h + kb), n, e->d_keys, sl->stream)
                         : neb_chacha_key_setup(sl->h, (const uint32_t*)(sl->h + kb), n, e->d_keys, sl->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(sl->stream);
    std::memset(sl->h, 0, (size_t)n * 32u);
    if (err != hipSuccess) {
        set_error("key setup", err);
        for (uint32_t i = 0; i < n; i++)
            (void)hipMemsetAsync(e->d_keys + (size_t)slots[i] * neb::kKeyRecDwords, 0, neb::kKeyRecBytes, sl->stream);
        (void)hipStreamSynchronize(sl->stream);
        return NEB_ERR_HIP;
    }
    return NEB_OK;
}

// Publish (rc == NEB_OK) or release the reserved slots; caller holds e->key_mu.
static void commit_slots(neb_engine* e, int alg, const uint32_t* slots, const uint64_t* tags, uint32_t n, bool ok) {
    for (uint32_t i = 0; i < n; i++) {
        e->slot_alg[slots[i]] = ok ? alg : 0;
        e->slot_tag[slots[i]] = ok ? tags[i] : 0;
    }
    if (ok) {
        e->installs += n;
        e->key_epoch++;
    }
}

static bool valid_alg(int alg) { return alg == NEB_ALG_AESGCM || alg == NEB_ALG_CHACHAPOLY; }

NEB_API int neb_cipher_create_batch(neb_engine* e, int alg, const uint8_t* keys, uint32_t n, neb_cipher** out) {
    if (!e || !out || !valid_alg(alg) || (n && !keys)) return NEB_ERR_INVALID;
    if (n == 0) return NEB_OK;
    for (uint32_t i = 0; i < n; i++) out[i] = nullptr;
    std::vector<uint32_t> slots(n);
    std::vector<uint64_t> tags(n);
    std::vector<neb_cipher*> cs(n, nullptr);
    for (uint32_t i = 0; i < n; i++) {
        cs[i] = new (std::nothrow) neb_cipher{e, 0, alg, 0};
        if (!cs[i]) {
            for (neb_cipher* c : cs) delete c;
            return NEB_ERR_INVALID;
        }
    }
    {
        std::lock_guard<std::mutex> g(e->key_mu);
        if (!reserve_slots(e, n, slots.data())) {
            for (neb_cipher* c : cs) delete c;
            return NEB_ERR_NO_KEY_SLOT;
        }
    }
    const int rc = install_records(e, alg, keys, slots.data(), n);
    const uint64_t t0 = g_key_tag.fetch_add(n);
    for (uint32_t i = 0; i < n; i++) tags[i] = t0 + i;
    std::lock_guard<std::mutex> g(e->key_mu);
    commit_slots(e, alg, slots.data(), tags.data(), n, rc == NEB_OK);
    for (uint32_t i = 0; i < n; i++) {
        if (rc != NEB_OK) {
            delete cs[i];
            continue;
        }
        cs[i]->key_id = slots[i];
        cs[i]->tag = tags[i];
        out[i] = cs[i];
    }
    return rc;
}

NEB_API int neb_cipher_create(neb_engine* e, int alg, const uint8_t key[32], neb_cipher** out) {
    if (!e || !key || !out || !valid_alg(alg)) return NEB_ERR_INVALID;
    *out = nullptr;
    return neb_cipher_create_batch(e, alg, key, 1, out);
}

NEB_API int neb_cipher_create_multi(neb_engine* const* engines, uint32_t m, int alg, const uint8_t key[32],
                                    neb_cipher** out) {
    if (!engines || m == 0 || !key || !out || !valid_alg(alg)) return NEB_ERR_INVALID;
    std::vector<neb_engine*> es(engines, engines + m);
    for (uint32_t k = 0; k < m; k++) {
        out[k] = nullptr;
        if (!es[k]) return NEB_ERR_INVALID;
    }
    std::vector<neb_engine*> order = es;
    std::sort(order.begin(), order.end());
    if (std::adjacent_find(order.begin(), order.end()) != order.end()) return NEB_ERR_INVALID;  // an engine twice
    std::vector<neb_cipher*> cs(m, nullptr);
    for (uint32_t k = 0; k < m; k++)
        if (!(cs[k] = new (std::nothrow) neb_cipher{es[k], 0, alg, 0})) {
            for (neb_cipher* c : cs) delete c;
            return NEB_ERR_INVALID;
        }
    // the lowest slot free on every engine, reserved on all of them at once (engines locked in
    // address order, so two concurrent multi-installs cannot deadlock)
    uint32_t slot = 0;
    {
        for (neb_engine* e : order) e->key_mu.lock();
        uint32_t lim = ~0u;
        for (neb_engine* e : es) lim = std::min(lim, e->max_keys);
        bool found = false;
        for (; slot < lim && !found; slot++) {
            found = true;
            for (neb_engine* e : es) found = found && e->slot_alg[slot] == 0;
            if (found) break;
        }
        if (found)
            for (neb_engine* e : es) e->slot_alg[slot] = -1;
        for (neb_engine* e : order) e->key_mu.unlock();
        if (!found) {
            for (neb_cipher* c : cs) delete c;
            return NEB_ERR_NO_KEY_SLOT;
        }
    }
    int rc = NEB_OK;
    std::vector<int> done(m, 0);
    for (uint32_t k = 0; k < m && rc == NEB_OK; k++) {
        rc = install_records(es[k], alg, key, &slot, 1);
        done[k] = rc == NEB_OK;
    }
    const uint64_t tag = g_key_tag.fetch_add(1);
    for (uint32_t k = 0; k < m; k++) {
        neb_engine* e = es[k];
        if (rc != NEB_OK && done[k]) {  // roll back the engines that had installed it
            DeviceGuard dg(e->device);
            PktLease sl(e->pkt);
            (void)hipMemsetAsync(e->d_keys + (size_t)slot * neb::kKeyRecDwords, 0, neb::kKeyRecBytes, sl->stream);
            (void)hipStreamSynchronize(sl->stream);
        }
        std::lock_guard<std::mutex> g(e->key_mu);
        commit_slots(e, alg, &slot, &tag, 1, rc == NEB_OK);
        if (rc == NEB_OK) {
            cs[k]->key_id = slot;
            cs[k]->tag = tag;
            out[k] = cs[k];
        } else {
            delete cs[k];
        }
    }
    return rc;
}

NEB_API int neb_cipher_destroy(neb_cipher* c) {
    if (!c) return NEB_ERR_INVALID;
    neb_engine* e = c->e;
    const uint32_t slot = c->key_id;
    DeviceGuard dg(e->device);
    // Asynchronous batches the engine enqueued that may read this record: the last single-key
    // batch with this key on each stream, the last mixed-key batch on each stream (note_use), and
    // the mixed-key AES-GCM batches of the engine's scheduler workspace. Those have no key-use
    // marker of their own (it cost ≈ 5 µs per batch): the workspace's `done` event is recorded
    // after each and every later user waits for it, so the destroy waits for the workspace's
    // latest batch — which may be another tunnel's batch enqueued after the last one that used
    // this key, so a teardown can wait behind unrelated mixed-key traffic on this engine (at most
    // the batches enqueued before the destroy; never the whole device).
    // The caller stops enqueuing with a key before destroying it.
    std::vector<hipEvent_t> wait;
    {
        std::lock_guard<std::mutex> g(e->use_mu);
        for (KeyUse& u : e->key_use[slot]) wait.push_back(u.ev);
        for (KeyUse& u : e->mixed_use) wait.push_back(u.ev);
    }
    {
        std::lock_guard<std::mutex> g(e->sched.mu);
        if (e->sched.done) wait.push_back(e->sched.done);
    }
    for (hipEvent_t ev : wait) (void)hipEventSynchronize(ev);
    int rc = NEB_OK;
    {
        PktLease sl(e->pkt);
        if (hipMemsetAsync(e->d_keys + (size_t)slot * neb::kKeyRecDwords, 0, neb::kKeyRecBytes, sl->stream) !=
                hipSuccess ||
            hipStreamSynchronize(sl->stream) != hipSuccess)
            rc = NEB_ERR_HIP;
    }
    {
        std::lock_guard<std::mutex> g(e->use_mu);
        for (KeyUse& u : e->key_use[slot]) hipEventDestroy(u.ev);
        e->key_use[slot].clear();
    }
    {
        std::lock_guard<std::mutex> g(e->key_mu);
        e->slot_alg[slot] = 0;
        e->slot_tag[slot] = 0;
        e->key_epoch++;
    }
    delete c;
    return rc;
}

NEB_API uint32_t neb_cipher_key_id(const neb_cipher* c) { return c ? c->key_id : NEB_KEYS_MIXED; }
NEB_API int neb_cipher_alg(const neb_cipher* c) { return c ? c->alg : 0; }
NEB_API int neb_overhead(const neb_cipher* c) { return c ? NEB_OVERHEAD : 0; }

static void fill_nonce(int alg, uint64_t n, uint8_t* nb) {
    if (!nb) return;
    nb[0] = nb[1] = nb[2] = nb[3] = 0;
    for (int i = 0; i < 8; i++) nb[4 + i] = alg == NEB_ALG_AESGCM ? (uint8_t)(n >> (56 - 8 * i)) : (uint8_t)(n >> (8 * i));
}

// Size the scheduler workspace for n packets (caller holds sched.mu). The counters are cleared on
// the batch's own stream: a plain hipMemset runs on the null stream, which a non-blocking stream
// does not wait for, and may still be running when the binning starts (measured: the first batches
// of a queue lost most of their packets' statuses to it).
static hipError_t sched_reserve(neb_engine* e, SchedSpace& sp, uint32_t n, hipStream_t s) {
    if (!sp.done) {
        // ordering only (the host and other streams wait for the kernels, nobody reads the
        // workspace from the host): no system-scope cache release at each record
        hipError_t err = hipEventCreateWithFlags(&sp.done, hipEventDisableTiming | hipEventDisableSystemFence);
        if (err != hipSuccess) return err;
    }
    // the tile binning's arrays (sched.hpp), only for workspaces that see batches that large: a
    // queue's small batches keep the atomic histogram and need none
    const bool tiles = (int64_t)n >= neb::knob(NEB_KNOB_TILE_BINS_FROM) || sp.ws.tcnt;
    const bool fits = n <= sp.n_cap && sp.mem && (!tiles || sp.ws.tcnt);
    if (fits && !sp.dirty) return hipSuccess;
    if (fits) {  // the bins are cleared as they are consumed, except after a failure
        hipError_t err = hipEventSynchronize(sp.done);
        if (err == hipSuccess)
            err = hipMemsetAsync(sp.ws.counters, 0, (neb::kSchedCounters + (size_t)neb::kSubBins * neb::sched_nbins(e->max_keys)) * 4u, s);
        if (err == hipSuccess) sp.dirty = false;
        return err;
    }
    const uint32_t cap = std::max<uint32_t>(n, 1u << 16);
    const uint32_t nb = neb::sched_nbins(e->max_keys);
    const uint32_t mc = neb::sched_max_chunks(cap, e->max_keys);
    const size_t b_counters = align_up((neb::kSchedCounters + (size_t)neb::kSubBins * nb) * 4u, 256);
    const size_t b_base = align_up((size_t)neb::kSubBins * nb * 4u, 256);
    const size_t b_idx = align_up((size_t)cap * 4u, 256), b_chunks = align_up((size_t)neb::kBuckets * mc * 16u, 256);
    const size_t b_tcnt = tiles ? align_up((size_t)neb::kTileMax * neb::sched_tile_words(nb) * 4u, 256) : 0;
    const size_t b_tpre = tiles ? align_up((size_t)neb::kTileMax * nb * 4u, 256) : 0;
    const size_t bytes = b_counters + b_base + 3 * b_idx + b_chunks + b_tcnt + b_tpre;
    hipError_t err = hipEventSynchronize(sp.done);  // the old buffer may still be in use
    if (err != hipSuccess) return err;
    if (sp.mem) hipFree(sp.mem);
    sp.mem = nullptr;
    sp.n_cap = 0;
    err = hipMalloc((void**)&sp.mem, bytes);
    if (err != hipSuccess) return err;
    uint8_t* m = sp.mem;
    sp.ws.counters = (uint32_t*)m;
    sp.ws.hist = sp.ws.counters + neb::kSchedCounters;
    m += b_counters;
    sp.ws.base = (uint32_t*)m;
    m += b_base;
    sp.ws.binof = (uint32_t*)m;
    m += b_idx;
    sp.ws.binpos = (uint32_t*)m;
    m += b_idx;
    sp.ws.sorted = (uint32_t*)m;
    m += b_idx;
    sp.ws.chunks = (uint4*)m;
    m += b_chunks;
    sp.ws.tcnt = tiles ? (uint32_t*)m : nullptr;
    m += b_tcnt;
    sp.ws.tpre = tiles ? (uint32_t*)m : nullptr;
    sp.ws.max_chunks = mc;
    sp.bytes = bytes;
    sp.n_cap = cap;
    err = hipMemsetAsync(sp.ws.counters, 0, b_counters, s);  // once: the binning clears its counts as it uses them
    if (err != hipSuccess) return err;
    sp.dirty = false;
    return hipSuccess;
}

// Groups per front chunk at most (sched_groups' own: up to 8) for a batch of n packets: below
// NEB_KNOB_SMALL_BATCH packets per resident wave of the chunk kernel (16 per CU) the front chunks hold
// NEB_KNOB_FRONT_GROUPS groups at most (sched.hpp kSmallBatchPerWave).
static uint32_t front_groups(const neb_engine* e, uint32_t n) {
    const int64_t below = neb::knob(NEB_KNOB_SMALL_BATCH), cap = neb::knob(NEB_KNOB_FRONT_GROUPS);
    const uint64_t waves = (uint64_t)std::max(e->cu_count, 1) * 16u;
    return below > 0 && cap > 0 && (uint64_t)n < (uint64_t)below * waves ? (uint32_t)std::min<int64_t>(cap, 8) : 8u;
}

// NEB_BIND_EVENTS=0 (read once): markers after each batch instead of events bound to its last
// kernel's dispatch (the A/B of round 4's binding for mixed-key AES-GCM and ChaCha batches)
static bool bind_events() {
    static const bool on = [] {
        const char* v = std::getenv("NEB_BIND_EVENTS");
        return !(v && v[0] == '0');
    }();
    return on;
}

// d_n (optional): the batch's real packet count in device memory, at most n (a batch whose size is
// only known on the device, e.g. the segments of a TX batch). hdr_from_dst: the TX batch's
// descriptors (tx.hip) read their first `flags` plaintext bytes from the destination.
// rx (optional, opens only): the device receive's admission mask; only packets with rx[i] != 0 are
// opened, the others keep the statuses its plan wrote (window.cpp, rxwin.hip).
// prebinned: the mixed-key binning of this batch is already in `sched` (neb_prebin, ordered before s).
static hipError_t launch_batch(neb_engine* e, int alg, int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                               int32_t* d_status, uint32_t key_hint, hipStream_t s, const uint32_t* d_n = nullptr,
                               SchedSpace* sched = nullptr, int hdr_from_dst = 0, hipEvent_t stop = nullptr,
                               const uint8_t* rx = nullptr, bool prebinned = false) {
    if (alg == NEB_ALG_AESGCM) {
        if (key_hint != NEB_KEYS_MIXED)
            return neb_gcm_batch_single(open, d_desc, n, d_arena, e->d_keys, e->max_keys, key_hint, d_status, d_n,
                                        e->cu_count, s, hdr_from_dst, stop, rx);
        // mixed keys: regroup into single-key, similar-size chunks on the device, then seal/open
        SchedSpace& sp = sched ? *sched : e->sched;
        std::lock_guard<std::mutex> g(sp.mu);
        hipError_t err = hipSuccess;
        if (!prebinned) {
            err = sched_reserve(e, sp, n, s);
            if (err == hipSuccess && !sp.last.same(s)) err = hipStreamWaitEvent(s, sp.done, 0);  // the previous batch on it
            neb::SchedWs ws = sp.ws;
            ws.max_groups = front_groups(e, n);
            if (err == hipSuccess) err = neb_sched_build(d_desc, n, d_n, e->max_keys, 4u, &ws, s);
        }
        if (err == hipSuccess)  // sp.done bound to the chunk kernel's dispatch: no marker packet between batches
            err = neb_gcm_batch_chunked(open, d_desc, n, d_arena, e->d_keys, e->max_keys, d_status, sp.ws.sorted,
                                        sp.ws.chunks, sp.ws.counters, sp.ws.max_chunks, e->cu_count,
                                        s, hdr_from_dst, bind_events() ? sp.done : nullptr,
                                        prebinned ? nullptr : rx);  // (prebinned: refused packets unlisted)
        if (err == hipSuccess && !bind_events()) err = hipEventRecord(sp.done, s);
        if (err == hipSuccess) sp.last.set(s);
        if (err != hipSuccess) {
            // binning passes of this batch may already be queued on s: let them finish before the
            // next batch clears the counters (sched_reserve's dirty path waits on sp.done only)
            (void)hipStreamSynchronize(s);
            sp.dirty = true;
        }
        return err;
    }
    return neb_chacha_batch(open, d_desc, n, d_arena, e->d_keys, e->max_keys, key_hint, d_status, d_n, e->cu_count,
                            s, hdr_from_dst, stop, rx);
}

// Poll a per-packet call's status word in pinned host memory (-1 until the kernel publishes it) for up
// to kPollUs; false when it has not come by then (the caller waits for the stream instead). A
// pinned-memory poll sees the kernel's last store within about a microsecond of it; the stream
// synchronize took ≈ 26 µs of the ≈ 36 µs call at 4 threads in round 4.
constexpr int kPollUs = 2000;
static bool poll_status(const int32_t* p, int32_t* st, int us = kPollUs) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        const int32_t v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
        if (v != -1) {
            *st = v;
            return true;
        }
        __builtin_ia32_pause();
        if ((i & 255u) == 255u &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us))
            return false;
    }
}

// A per-packet call's result from its pool slot into the caller's buffer, by status: a sealed or
// opened packet is copied; a failed open leaves zeros (the kernel's in-place zeroing, written here
// so the slot is never read); any other status (no key, exhausted counter) writes nothing, as the
// reference returns before touching out (aesgcm.go:28-30). The slot's bytes are read only when the
// kernel wrote them: slots are shared by every thread and cipher of the engine, so anything else
// there is another call's packet.
static void copy_result(int open, int32_t st, uint8_t* dst, const uint8_t* slot, size_t pay_len) {
    const size_t out_len = open ? pay_len : pay_len + 16;
    if (!out_len) return;
    if (st == NEB_STATUS_OK)
        std::memcpy(dst, slot, out_len);
    else if (open && st == NEB_STATUS_AUTH_FAILED)
        std::memset(dst, 0, out_len);
}

// One packet through the device, on a slot of the engine's per-packet pool (PktPool): the packet is
// copied into the slot's pinned, mapped buffer ([desc | status | aad | payload (+tag)]), the batch
// kernel seals or opens it there in place (zero-copy: no DMA either way) and the result is copied
// out. Up to kPktSlots calls run side by side; later ones wait their turn in FIFO order.
static int one_packet_solo(neb_cipher* c, int open, const uint8_t* ad, size_t ad_len, const uint8_t* in,
                           size_t in_len, size_t pay_len, uint64_t n, uint8_t* dst, int32_t* st_out) {
    neb_engine* e = c->e;
    const size_t o_desc = 0, o_status = 64, o_aad = 128;
    const size_t o_pay = align_up(o_aad + ad_len, 16);
    const size_t total = o_pay + pay_len + 16;
    DeviceGuard dg(e->device);
    PktLease sl(e->pkt);
    if (!sl.reserve(total)) return NEB_ERR_HIP;
    uint8_t* h = sl->h;
    // The packet's bytes travel in the kernel's arguments and only the result comes back through
    // the slot (aes_gcm.hip gcm_one_kernel, chacha_poly.hip chacha_one_kernel); NEB_ONE_KERNEL=0
    // for the A/B
    static const bool one = [] {
        const char* v = std::getenv("NEB_ONE_KERNEL");
        return !(v && v[0] == '0');
    }();
    if (one) {
        *(int32_t*)(h + o_status) = -1;
        auto* fn = c->alg == NEB_ALG_AESGCM ? neb_gcm_one : neb_chacha_one;
        hipError_t err = fn(open, ad, (uint32_t)ad_len, in, (uint32_t)in_len, (uint32_t)pay_len, n, h + o_pay,
                            (int32_t*)(h + o_status), e->d_keys, e->max_keys, c->key_id, sl->stream);
        if (err == hipSuccess) {
            // the kernel publishes the status last, behind a system-scope release of the result
            // (device_common.hpp one_publish_status): poll it, and wait for the stream only if it
            // does not come (a fault reports there)
            int32_t st = -1;
            if (!poll_status(reinterpret_cast<const int32_t*>(h + o_status), &st)) {
                err = hipStreamSynchronize(sl->stream);
                if (err != hipSuccess) {
                    set_error("one_packet", err);
                    return NEB_ERR_HIP;
                }
                st = __atomic_load_n(reinterpret_cast<const int32_t*>(h + o_status), __ATOMIC_ACQUIRE);
            }
            *st_out = st;
            copy_result(open, st, dst, h + o_pay, pay_len);
            return NEB_OK;
        }
        if (err != hipErrorInvalidValue) {  // (too large for the arguments: the batch path below)
            set_error("one_packet", err);
            return NEB_ERR_HIP;
        }
        (void)hipGetLastError();
    }
    neb_desc d{};
    d.src_off = o_pay - o_aad;
    d.dst_off = o_pay - o_aad;
    d.aad_off = 0;
    d.counter = n;
    d.len = (uint32_t)pay_len;
    d.aad_len = (uint32_t)ad_len;
    d.key_id = c->key_id;
    std::memcpy(h + o_desc, &d, sizeof d);
    *(int32_t*)(h + o_status) = -1;
    if (ad_len) std::memcpy(h + o_aad, ad, ad_len);
    if (in_len) std::memcpy(h + o_pay, in, in_len);
    hipError_t err = launch_batch(e, c->alg, open, (const neb_desc*)(h + o_desc), 1, h + o_aad,
                                  (int32_t*)(h + o_status), c->key_id, sl->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(sl->stream);
    if (err != hipSuccess) {
        set_error("one_packet", err);
        return NEB_ERR_HIP;
    }
    std::memcpy(st_out, h + o_status, 4);
    copy_result(open, *st_out, dst, h + o_pay, pay_len);
    return NEB_OK;
}

// A per-packet call through the engine's combiner (PktComb): alone while a launch slot is free
// (one_packet_solo: the packet in the kernel arguments), else as a request of the batch the next
// completed launch frees a slot for. AES-256-GCM only (the ChaCha20-Poly1305 batch kernel's statuses carry no
// release of the payload before them, so its calls stay alone).
static int one_packet(neb_cipher* c, int open, const uint8_t* ad, size_t ad_len, const uint8_t* in, size_t in_len,
                      size_t pay_len, uint64_t n, uint8_t* dst, int32_t* st_out) {
    neb_engine* e = c->e;
    static const bool comb_on = [] {  // NEB_PKT_COMBINE=0: every call alone (A/B)
        const char* v = std::getenv("NEB_PKT_COMBINE");
        return !(v && v[0] == '0');
    }();
    const size_t pay = align_up(ad_len, 16);
    if (!comb_on || c->alg != NEB_ALG_AESGCM || pay + std::max(in_len, pay_len + 16) > kCombSlot || pay + in_len > 2048)
        return one_packet_solo(c, open, ad, ad_len, in, in_len, pay_len, n, dst, st_out);
    static const uint32_t max_inflight = [] {  // NEB_PKT_INFLIGHT: launches in flight (A/B), default 4
        const char* v = std::getenv("NEB_PKT_INFLIGHT");
        const int x = v ? std::atoi(v) : (int)kPktSlots;
        return (uint32_t)std::min(std::max(x, 1), 64);
    }();
    PktComb& cb = e->comb;
    std::unique_lock<std::mutex> lk(cb.mu);
    CombBatch*& ob = cb.open[0][open ? 1 : 0];
    // Alone while a launch and a pool slot are free and no batch is gathering (each alone call
    // holds a pool slot; only these take slots here).
    if (cb.inflight < max_inflight && cb.solo < kPktSlots && !ob) {
        cb.inflight++;
        cb.solo++;
        lk.unlock();
        const int rc = one_packet_solo(c, open, ad, ad_len, in, in_len, pay_len, n, dst, st_out);
        lk.lock();
        cb.inflight--;
        cb.solo--;
        lk.unlock();
        cb.launch_cv.notify_all();
        return rc;
    }
    DeviceGuard dg(e->device);
    if (!ob) {
        if (cb.free_.empty()) {
            auto* nb = new (std::nothrow) CombBatch;
            if (!nb) return NEB_ERR_INVALID;
            if (hipHostMalloc((void**)&nb->h, kCombBytes, hipHostMallocDefault) != hipSuccess) {
                delete nb;
                set_error("hipHostMalloc (per-packet batch)", hipErrorOutOfMemory);
                return NEB_ERR_HIP;
            }
            cb.all.push_back(nb);
            cb.free_.push_back(nb);
        }
        ob = cb.free_.back();
        cb.free_.pop_back();
        ob->n = 0;
        ob->launched = false;
        ob->failed = false;
        ob->done.store(0, std::memory_order_relaxed);
        ob->alg = c->alg;
        ob->open = open;
    }
    CombBatch* b = ob;
    const uint32_t i = b->n++;
    if (b->n == kCombMax) ob = nullptr;  // full: the next call starts another
    uint8_t* slot = b->slots() + (size_t)i * kCombSlot;
    if (ad_len) std::memcpy(slot, ad, ad_len);
    if (in_len) std::memcpy(slot + pay, in, in_len);
    neb_desc& d = b->desc()[i];
    d = neb_desc{};
    d.aad_off = (uint64_t)i * kCombSlot;
    d.src_off = d.dst_off = d.aad_off + pay;  // in place in the slot
    d.counter = n;
    d.len = (uint32_t)pay_len;
    d.aad_len = (uint32_t)ad_len;
    d.key_id = c->key_id;
    __atomic_store_n(b->status() + i, -1, __ATOMIC_RELAXED);
    // The batch's first request leads it: it waits until a launch completes, launches the batch as
    // it stands then (every joined request is filled: joiners fill under the mutex), polls every
    // status and wakes the others. Under load the batch gathers for as long as the launches ahead
    // of it run, so its size follows the offered load; one thread spins per launch, the rest sleep
    // (64 threads spinning on a 16-CPU share starved the launches: p99 37 ms).
    if (i == 0) {
        cb.launch_cv.wait(lk, [&] { return cb.inflight < max_inflight; });
        cb.inflight++;
        if (ob == b) ob = nullptr;
        b->launched = true;
        b->left.store(b->n, std::memory_order_relaxed);
        b->stream = e->pkt.slot[cb.next++ % kPktSlots].stream;
        const uint32_t cnt = b->n;
        e->pkt.calls.fetch_add(cnt, std::memory_order_relaxed);  // (neb_engine_stats: per-packet calls)
        lk.unlock();
        hipError_t err = neb_gcm_one_batch(open, b->desc(), b->status(), b->slots(), cnt, e->d_keys, e->max_keys,
                                           b->stream);
        cb.launches.fetch_add(1, std::memory_order_relaxed);
        cb.combined.fetch_add(cnt, std::memory_order_relaxed);
        if (err == hipSuccess) {
            bool slow = false;
            for (uint32_t k = 0; k < cnt && !slow; k++) {
                int32_t v;
                slow = !poll_status(b->status() + k, &v);
            }
            if (slow) err = hipStreamSynchronize(b->stream);  // a slow device: the stream says when
        }
        if (err != hipSuccess) set_error("per-packet batch launch", err);
        lk.lock();
        cb.inflight--;
        lk.unlock();
        cb.launch_cv.notify_all();
        b->finish(err != hipSuccess);
    } else {
        lk.unlock();
    }
    // (the owners sleep rather than poll their own status words: 8 spinners measured 317-336 k /
    // 363-387 k calls/s at 16 / 32 threads against 338-341 k / 530-542 k sleeping)
    const bool failed = b->wait();
    const int32_t st = failed ? -1 : __atomic_load_n(b->status() + i, __ATOMIC_ACQUIRE);
    if (st != -1) copy_result(open, st, dst, slot + pay, pay_len);
    if (b->left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        lk.lock();
        cb.free_.push_back(b);
        lk.unlock();
    }
    if (st == -1) return NEB_ERR_HIP;
    *st_out = st;
    return NEB_OK;
}

// Per-packet calls combined into shared launches: {launches of combined batches, calls they carried}
NEB_API int neb_engine_pkt_combined(const neb_engine* e, uint64_t out[2]) {
    if (!e || !out) return NEB_ERR_INVALID;
    out[0] = e->comb.launches.load(std::memory_order_relaxed);
    out[1] = e->comb.combined.load(std::memory_order_relaxed);
    return NEB_OK;
}

NEB_API int neb_encrypt_danger(neb_cipher* c, uint8_t* out, size_t out_len, size_t out_cap, const uint8_t* ad,
                               size_t ad_len, const uint8_t* pt, size_t pt_len, uint64_t n, uint8_t* nb,
                               size_t* ret_len) {
    if (ret_len) *ret_len = 0;
    if (!c) return NEB_ERR_NO_CIPHER;  // aesgcm.go:25-27
    if (n >= NEB_REJECT_AFTER_MESSAGES) return NEB_ERR_EXHAUSTED;  // aesgcm.go:28-30
    if ((!out && out_cap) || (!ad && ad_len) || (!pt && pt_len) || pt_len > 0xFFFFFFF0u || ad_len > 0xFFFFFFF0u)
        return NEB_ERR_INVALID;
    if (out_cap < out_len || out_cap - out_len < pt_len + NEB_OVERHEAD) return NEB_ERR_SHORT_BUFFER;
    fill_nonce(c->alg, n, nb);
    int32_t st = -1;
    int rc = one_packet(c, 0, ad, ad_len, pt, pt_len, pt_len, n, out + out_len, &st);
    if (rc != NEB_OK) return rc;
    if (st != NEB_STATUS_OK) return st == NEB_STATUS_EXHAUSTED ? NEB_ERR_EXHAUSTED : NEB_ERR_INVALID;
    if (ret_len) *ret_len = out_len + pt_len + NEB_OVERHEAD;
    return NEB_OK;
}

NEB_API int neb_decrypt_danger(neb_cipher* c, uint8_t* out, size_t out_len, size_t out_cap, const uint8_t* ad,
                               size_t ad_len, const uint8_t* ct, size_t ct_len, uint64_t n, uint8_t* nb,
                               size_t* ret_len) {
    if (ret_len) *ret_len = 0;
    if (!c) return NEB_OK;  // aesgcm.go:40-42: ([]byte{}, nil)
    if ((!ad && ad_len) || (!ct && ct_len) || ct_len > 0xFFFFFFF0u || ad_len > 0xFFFFFFF0u) return NEB_ERR_INVALID;
    fill_nonce(c->alg, n, nb);
    if (ct_len < NEB_OVERHEAD) return NEB_ERR_AUTH;  // Open: ciphertext shorter than the tag
    const size_t pt_len = ct_len - NEB_OVERHEAD;
    if ((!out && out_cap) || out_cap < out_len || out_cap - out_len < pt_len) return NEB_ERR_SHORT_BUFFER;
    int32_t st = -1;
    int rc = one_packet(c, 1, ad, ad_len, ct, ct_len, pt_len, n, out + out_len, &st);
    if (rc != NEB_OK) return rc;
    if (st == NEB_STATUS_AUTH_FAILED) return NEB_ERR_AUTH;  // plaintext region already zeroed
    if (st != NEB_STATUS_OK) return NEB_ERR_INVALID;
    if (ret_len) *ret_len = out_len + pt_len;
    return NEB_OK;
}

static int check_batch(neb_engine* e, int alg, uint32_t key_hint) {
    if (!e || (alg != NEB_ALG_AESGCM && alg != NEB_ALG_CHACHAPOLY)) return NEB_ERR_INVALID;
    if (key_hint != NEB_KEYS_MIXED) {
        std::lock_guard<std::mutex> g(e->key_mu);
        if (key_hint >= e->max_keys || e->slot_alg[key_hint] != alg) return NEB_ERR_INVALID;
    }
    return NEB_OK;
}

static int batch_device(neb_engine* e, int alg, int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                        int32_t* d_status, uint32_t key_hint, void* stream) {
    int rc = check_batch(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    if (!d_desc || !d_arena || !d_status) return NEB_ERR_INVALID;
    DeviceGuard dg(e->device);
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream, as for any HIP launch
    // A batch binds its key-use event to its last kernel (no marker packet after it: each marker
    // between two batches cost ≈ 5 µs, C3 +3.5-5%, profiles/r3_ab/use_events.log). A mixed-key
    // AES-GCM batch runs through the engine's scheduler workspace, whose `done` event is bound to
    // its chunk kernel the same way and orders every later user of the workspace after it;
    // neb_cipher_destroy waits on that event, so it needs no key-use event of its own.
    const bool sched = alg == NEB_ALG_AESGCM && key_hint == NEB_KEYS_MIXED;
    const bool single_aes = alg == NEB_ALG_AESGCM && key_hint != NEB_KEYS_MIXED;  // bound since round 3
    hipEvent_t stop = sched || !(single_aes || bind_events()) ? nullptr : use_event(e, key_hint, s);
    hipError_t err = launch_batch(e, alg, open, d_desc, n, d_arena, d_status, key_hint, s, nullptr, nullptr, 0, stop);
    if (err != hipSuccess) {
        set_error("batch launch", err);
        return NEB_ERR_HIP;
    }
    if (!sched && !stop) note_use(e, key_hint, s);  // no event could be created: a marker
    return NEB_OK;
}

NEB_API int neb_seal_batch(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                           int32_t* d_status, uint32_t key_hint, void* stream) {
    return batch_device(e, alg, 0, d_desc, n, d_arena, d_status, key_hint, stream);
}

NEB_API int neb_open_batch(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                           int32_t* d_status, uint32_t key_hint, void* stream) {
    return batch_device(e, alg, 1, d_desc, n, d_arena, d_status, key_hint, stream);
}

// ---- for the device batched receive (window.cpp, rxwin.hip); internal ------------------------

int neb_engine_device_of(const neb_engine* e) { return e->device; }
int neb_check_batch_args(neb_engine* e, int alg, uint32_t key_hint) { return check_batch(e, alg, key_hint); }

// Open the first *d_n (a count in device memory) of at most n descriptors, on stream s.
int neb_open_batch_count(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, const uint32_t* d_n,
                         uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, hipStream_t s, const uint8_t* rx,
                         void* prebinned) {
    if (n == 0) return NEB_OK;
    hipError_t err = launch_batch(e, alg, 1, d_desc, n, d_arena, d_status, key_hint, s, d_n,
                                  static_cast<SchedSpace*>(prebinned), 0, nullptr, rx, prebinned != nullptr);
    if (err != hipSuccess) {
        set_error("batch launch", err);
        return NEB_ERR_HIP;
    }
    return NEB_OK;
}

// For the submission queue (queue.cpp): a scheduler workspace of its own, and a launch of one
// staged batch (zero-copy on pinned memory) on the queue's stream.
void* neb_sched_space_new() { return new (std::nothrow) SchedSpace; }

// The device receive (window.cpp): its mixed-key AES-GCM open is binned by extra workgroups of the
// receive's own plan launches (rxwin.hpp RxBin) into the receive's scheduler workspace `sched`,
// which this sizes for n packets and orders after its last open; the open then runs with it
// (neb_open_batch_count's `prebinned`). neb_rx_sched_abort after a failed plan (the counters are
// then in an unknown state: the next batch clears them).
int neb_rx_sched_begin(neb_engine* e, uint32_t n, void* sched, hipStream_t s, neb::SchedWs* ws, uint32_t* max_keys) {
    SchedSpace& sp = *static_cast<SchedSpace*>(sched);
    std::lock_guard<std::mutex> g(sp.mu);
    hipError_t err = sched_reserve(e, sp, n, s);
    if (err == hipSuccess && !sp.last.same(s)) err = hipStreamWaitEvent(s, sp.done, 0);  // the last open's reads
    if (err != hipSuccess) {
        sp.dirty = true;
        set_error("rx binning", err);
        return NEB_ERR_HIP;
    }
    *ws = sp.ws;
    ws->max_groups = front_groups(e, n);
    *max_keys = e->max_keys;
    return NEB_OK;
}
void neb_rx_sched_abort(void* sched) {
    SchedSpace& sp = *static_cast<SchedSpace*>(sched);
    std::lock_guard<std::mutex> g(sp.mu);
    sp.dirty = true;
}
void neb_sched_space_free(void* p) {
    auto* sp = static_cast<SchedSpace*>(p);
    if (!sp) return;
    if (sp->done) { hipEventSynchronize(sp->done); hipEventDestroy(sp->done); }
    if (sp->mem) hipFree(sp->mem);
    delete sp;
}
int neb_launch_on(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n, uint8_t* arena,
                  int32_t* status, uint32_t key_hint, hipStream_t s, void* sched) {
    if (n == 0) return NEB_OK;
    DeviceGuard dg(e->device);
    hipError_t err = launch_batch(e, alg, open, desc, n, arena, status, key_hint, s, nullptr,
                                  static_cast<SchedSpace*>(sched), 0, nullptr);
    if (err != hipSuccess) {
        set_error("queue batch launch", err);
        return NEB_ERR_HIP;
    }
    return NEB_OK;
}
bool neb_host_mapped(const void* p);
int neb_key_alg(neb_engine* e, uint32_t key) {
    std::lock_guard<std::mutex> g(e->key_mu);
    return key < e->max_keys ? e->slot_alg[key] : 0;
}

// True if p is pinned host memory the device addresses at the same pointer (hipHostMalloc).
static bool host_mapped(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer == p;
}
bool neb_host_mapped(const void* p) { return host_mapped(p); }  // queue.cpp

// Zero-copy host batch: the arena is pinned and mapped, so the kernels load and store it across
// PCIe themselves (loads = the H2D direction, stores = D2H, both at once) with no staging copies.
// Pageable descriptors / statuses go through device buffers. Every descriptor is bounds-checked
// on the host first: a kernel access outside the mapping would fault the GPU.
static int batch_host_zero_copy(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n,
                                uint8_t* arena, size_t arena_len, int32_t* status, uint32_t key_hint) {
    const bool desc_mapped = host_mapped(desc), status_mapped = host_mapped(status);
    if ((!desc_mapped || !status_mapped) && n > e->zc_cap) {
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (e->zc_desc) { hipFree(e->zc_desc); e->zc_desc = nullptr; }
        if (e->zc_status) { hipFree(e->zc_status); e->zc_status = nullptr; }
        e->zc_cap = 0;
        HIP_TRY(hipMalloc((void**)&e->zc_desc, (size_t)n * sizeof(neb_desc)));
        HIP_TRY(hipMalloc((void**)&e->zc_status, (size_t)n * sizeof(int32_t)));
        e->zc_cap = n;
    }
    const neb_desc* d_desc = desc;
    int32_t* d_status = status;
    if (!desc_mapped) {
        HIP_TRY(hipMemcpyAsync(e->zc_desc, desc, (size_t)n * sizeof(neb_desc), hipMemcpyHostToDevice, e->stream));
        d_desc = e->zc_desc;
    }
    if (!status_mapped) d_status = e->zc_status;
    HIP_TRY(launch_batch(e, alg, open, d_desc, n, arena, d_status, key_hint, e->stream));
    if (!status_mapped)
        HIP_TRY(hipMemcpyAsync(status, d_status, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return NEB_OK;
}

// Host-resident batch. A pinned, mapped arena runs zero-copy (above). Any other arena is staged in
// chunks of kPipeChunkPkts packets rotated over kPipeStreams streams: each chunk's arena span is
// copied in (hipMemcpyAsync), sealed/opened on the device and copied back, so one chunk's copy-in
// overlaps another's kernel and another's copy-back. NEB_HOST_MODE=dma forces the staging for a
// mapped arena too. Every descriptor is checked before anything is copied or launched: an invalid
// batch returns NEB_ERR_INVALID with the arena and the statuses untouched.
static int batch_host(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n, uint8_t* arena,
                      size_t arena_len, int32_t* status, uint32_t key_hint) {
    int rc = check_batch(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    if (!desc || !arena || !status) return NEB_ERR_INVALID;
    // Every descriptor is checked before the arena or the statuses are written. The staged path
    // checks the first chunk's, starts that chunk's copy-in and kernel (they write device buffers
    // only), and checks the rest while they run: ≈ 90 µs of checks per 64 Ki packets off the
    // critical path. Its first copy back waits for the whole check.
    uint32_t checked = 0;
    auto check_upto = [&](uint32_t end) {
        for (; checked < end; checked++)
            if (!neb_desc_in_arena(desc[checked], open, arena_len)) return false;
        return true;
    };
    std::lock_guard<std::mutex> g(e->pipe_mu);
    DeviceGuard dg(e->device);
    // The kernels' vector fast path tests the absolute address (arena base + offset), so a mapped
    // arena at any byte address runs zero-copy. A staged arena lands in a device buffer with the
    // same alignment modulo 16, so the kernels take the same paths either way.
    if (host_mode() == kHostZeroCopy && host_mapped(arena)) {
        if (!check_upto(n)) return NEB_ERR_INVALID;
        return batch_host_zero_copy(e, alg, open, desc, n, arena, arena_len, status, key_hint);
    }
    Pipe& P = e->pipe;
    // Each of the pipeline's streams on a hardware queue of its own: a stream with a CU mask gets
    // one (all CUs here; tools/native/queue_map.cpp), where default streams share the process's 4
    // and two of the pipeline's could land on one, so a chunk's kernel queued behind the previous
    // chunk's copy back. NEB_PIPE_QUEUES=0: default streams, 2: low-priority streams (also a queue
    // each) (A/B).
    static const int own_queues = [] {
        const char* v = std::getenv("NEB_PIPE_QUEUES");
        return v ? std::atoi(v) : 1;
    }();
    for (hipStream_t* st : {&P.h2d, &P.comp, &P.d2h}) {
        if (*st) continue;
        if (own_queues == 2) {
            int least = 0, greatest = 0;
            HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIP_TRY(hipStreamCreateWithPriority(st, hipStreamNonBlocking, least));
        } else if (own_queues == 1) {
            std::vector<uint32_t> mask(((uint32_t)e->cu_count + 31u) / 32u, 0u);
            for (int c = 0; c < e->cu_count; c++) mask[c / 32] |= 1u << (c % 32);
            HIP_TRY(hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()));
        } else {
            HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
        }
    }
    if (!P.sched && !(P.sched = new (std::nothrow) SchedSpace)) return NEB_ERR_INVALID;
    for (auto& s : P.slot) {
        if (!s.done) {
            for (hipEvent_t* ev : {&s.in_done, &s.k_done, &s.done})
                HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming));
            HIP_TRY(hipHostMalloc((void**)&s.h_desc, kPipeChunkPkts * sizeof(neb_desc), hipHostMallocDefault));
            HIP_TRY(hipMalloc((void**)&s.d_desc, kPipeChunkPkts * sizeof(neb_desc)));
            HIP_TRY(hipHostMalloc((void**)&s.h_status, kPipeChunkPkts * sizeof(int32_t), hipHostMallocDefault));
        }
        s.count = 0;
    }
    auto retire = [](PipeSlot& s) -> hipError_t {
        hipError_t err = hipEventSynchronize(s.done);
        if (err != hipSuccess) return err;
        std::memcpy(s.user_status + s.user_begin, s.h_status, s.count * sizeof(int32_t));
        s.count = 0;
        s.back_pending = false;
        return hipSuccess;
    };
    // A slot taken for the next chunk: the host waits for the previous chunk's copy back (retire).
    // In the trace each copy-in then starts as the copy back two chunks before it ends, 284 µs per
    // call idle on the copy-in stream (profiles/r6/host/final_*_trace.csv, tools/r6/
    // copy_overlap.py). Two ways of removing that wait measured no better: NEB_PIPE_GPU_WAIT=1
    // waits only for the kernel on the host and for the copy back on the device (hipStreamWaitEvent
    // before the copy-in), 27.9-29.3 against 31.7-33.4 GiB/s (ab_gpu_wait.jsonl); an empty kernel
    // after each copy back with the event after it, 30.5-32.3 against 31.3-32.9 (ab_mark.jsonl).
    static const bool gpu_wait = [] {
        const char* v = std::getenv("NEB_PIPE_GPU_WAIT");
        return v && v[0] == '1';
    }();
    auto reuse = [&](PipeSlot& s) -> hipError_t {
        if (!gpu_wait) return retire(s);
        hipError_t err = hipEventSynchronize(s.k_done);
        if (err != hipSuccess) return err;
        std::memcpy(s.user_status + s.user_begin, s.h_status, s.count * sizeof(int32_t));
        s.count = 0;
        s.back_pending = true;
        return hipSuccess;
    };
    // any failure below leaves work queued on the three streams: drain them before returning
    auto fail = [&](const char* where, hipError_t err) {
        set_error(where, err);
        for (hipStream_t st : {P.h2d, P.comp, P.d2h}) (void)hipStreamSynchronize(st);
        for (auto& s : P.slot) s.count = 0, s.back_pending = false;
        return NEB_ERR_HIP;
    };
#define PIPE_TRY(x)                                     \
    do {                                                \
        hipError_t err_ = (x);                          \
        if (err_ != hipSuccess) return fail(#x, err_);  \
    } while (0)
    const std::vector<uint32_t> plan = pipe_plan(n);
    bool arena_mapped = false;
    uint32_t begin = 0;
    for (uint32_t k = 0; k < plan.size(); begin += plan[k], k++) {
        PipeSlot& s = P.slot[k % kPipeSlots];
        if (s.count) PIPE_TRY(reuse(s));  // the slot's previous chunk's kernel is done
        const uint32_t cnt = plan[k];
        if (!check_upto(begin + cnt)) {  // (only ever the first chunk: the rest were checked after it)
            for (hipStream_t st : {P.h2d, P.comp, P.d2h}) (void)hipStreamSynchronize(st);
            for (auto& o : P.slot) o.count = 0, o.back_pending = false;
            return NEB_ERR_INVALID;
        }
        uint64_t lo = ~0ULL, hi = 0;  // every sum below stays within arena_len (checked above)
        for (uint32_t i = 0; i < cnt; i++) {
            const neb_desc& d = desc[begin + i];
            const uint64_t pay = (uint64_t)d.len + (open ? 16u : 0u), outl = (uint64_t)d.len + (open ? 0u : 16u);
            lo = std::min({lo, d.src_off, d.dst_off, d.aad_off});
            hi = std::max({hi, d.src_off + pay, d.dst_off + outl, d.aad_off + d.aad_len});
        }
        lo &= ~(uint64_t)15;
        // A chunk copies its whole span back, so spans of chunks in flight must not overlap (the
        // descriptors need not be in arena order): retire any other slot whose span intersects.
        // (A slot whose statuses are taken but whose copy back may still run: the copy-in waits for it.)
        for (auto& o : P.slot) {
            if (&o == &s || !(o.lo < hi && lo < o.hi)) continue;
            if (o.count) PIPE_TRY(retire(o));
            else if (o.back_pending) PIPE_TRY(hipStreamWaitEvent(P.h2d, o.done, 0));
        }
        s.lo = lo;
        s.hi = hi;
        const size_t span = (size_t)(hi - lo);
        if (span > s.d_cap) {  // (retired: nothing in flight uses it)
            if (s.back_pending) PIPE_TRY(hipEventSynchronize(s.done));
            s.back_pending = false;
            if (s.d_buf) { hipFree(s.d_buf); s.d_buf = nullptr; s.d_cap = 0; }
            size_t cap = align_up(span, 1 << 20);
            PIPE_TRY(hipMalloc((void**)&s.d_buf, cap));
            s.d_cap = cap;
        }
#ifndef NEB_PIPE_MODE  // A/B: 0 copies back on a stream of their own, 1 on the kernels' stream, 2 the kernels store into the arena
#define NEB_PIPE_MODE 0
#endif
        // mode 2: the outputs go straight to the host arena (a wrapping offset from the device buffer)
        const uint64_t out_rebase = NEB_PIPE_MODE == 2 ? (uint64_t)(uintptr_t)(arena + lo) - (uint64_t)(uintptr_t)s.d_buf : 0u;
        for (uint32_t i = 0; i < cnt; i++) {
            neb_desc d = desc[begin + i];
            d.src_off -= lo;
            d.aad_off -= lo;
            d.dst_off = d.dst_off - lo + out_rebase;
            s.h_desc[i] = d;
        }
        s.user_status = status;
        s.user_begin = begin;
        s.count = cnt;
        // The kernels write the chunk's statuses in the slot's pinned, mapped buffer themselves (4 B
        // per packet of posted writes). Its descriptors go to the device on the kernels' stream,
        // ahead of them: read over PCIe in place they waited behind the copies' 90 GB/s, and the
        // kernels ran 250-478 µs per 16 Ki-packet chunk instead of ≈ 25 (profiles/r6/host/); on the
        // copy-in stream the small copy's latency left that stream idle between chunks.
        static const int desc_dev = [] {  // NEB_PIPE_DESC=0: read in place, 2: hipMemcpyAsync (A/B)
            const char* v = std::getenv("NEB_PIPE_DESC");
            return v ? std::atoi(v) : 1;
        }();
        // NEB_PIPE_COPY (A/B): bit 0 copies back with a kernel of ours instead of hipMemcpyAsync, bit
        // 1 copies in with one. Only for an arena the device can address (pinned and mapped at both
        // ends: a kernel touching pageable memory faults the GPU) at the same address mod 16 as its
        // device buffer; anything else takes hipMemcpyAsync.
        static const int copy_k = [] {
            const char* v = std::getenv("NEB_PIPE_COPY");
            return v ? std::atoi(v) : 0;
        }();
        if (k == 0) arena_mapped = copy_k && arena_len && host_mapped(arena) && host_mapped(arena + arena_len - 1);
        auto copy = [&](void* dst, const void* src, hipMemcpyKind kind, hipStream_t st) {
            if (arena_mapped && (copy_k & (kind == hipMemcpyDeviceToHost ? 1 : 2)) &&
                neb_copy_span(dst, src, span, st) == hipSuccess)
                return hipSuccess;
            (void)hipGetLastError();
            return hipMemcpyAsync(dst, src, span, kind, st);
        };
        if (s.back_pending) PIPE_TRY(hipStreamWaitEvent(P.h2d, s.done, 0));
        s.back_pending = false;
        PIPE_TRY(copy(s.d_buf, arena + lo, hipMemcpyHostToDevice, P.h2d));
        PIPE_TRY(hipEventRecord(s.in_done, P.h2d));
        if (NEB_PIPE_MODE == 2 && k == 0 && !check_upto(n)) {  // (mode 2's kernels write the arena)
            for (hipStream_t st : {P.h2d, P.comp, P.d2h}) (void)hipStreamSynchronize(st);
            for (auto& o : P.slot) o.count = 0, o.back_pending = false;
            return NEB_ERR_INVALID;
        }
        PIPE_TRY(hipStreamWaitEvent(P.comp, s.in_done, 0));
        if (desc_dev == 2)
            PIPE_TRY(hipMemcpyAsync(s.d_desc, s.h_desc, cnt * sizeof(neb_desc), hipMemcpyHostToDevice, P.comp));
        else if (desc_dev)
            PIPE_TRY(neb_copy_desc(s.d_desc, s.h_desc, cnt, P.comp));
        PIPE_TRY(launch_batch(e, alg, open, desc_dev ? s.d_desc : s.h_desc, cnt, s.d_buf, s.h_status, key_hint, P.comp,
                              nullptr, P.sched));
        PIPE_TRY(hipEventRecord(s.k_done, P.comp));
        if (k == 0 && !check_upto(n)) {  // the rest of the batch, while chunk 0 is copied in and run
            for (hipStream_t st : {P.h2d, P.comp, P.d2h}) (void)hipStreamSynchronize(st);
            for (auto& o : P.slot) o.count = 0, o.back_pending = false;
            return NEB_ERR_INVALID;
        }
        if (NEB_PIPE_MODE == 2) {
            PIPE_TRY(hipEventRecord(s.done, P.comp));
        } else {
            hipStream_t back = NEB_PIPE_MODE == 1 ? P.comp : P.d2h;
            if (NEB_PIPE_MODE == 0) PIPE_TRY(hipStreamWaitEvent(P.d2h, s.k_done, 0));
            PIPE_TRY(copy(arena + lo, s.d_buf, hipMemcpyDeviceToHost, back));
            PIPE_TRY(hipEventRecord(s.done, back));
        }
    }
    for (auto& s : P.slot) {
        if (s.count) PIPE_TRY(retire(s));
        if (s.back_pending) PIPE_TRY(hipEventSynchronize(s.done));  // every copy back is in the arena
        s.back_pending = false;
    }
#undef PIPE_TRY
    return NEB_OK;
}

NEB_API int neb_seal_batch_host(neb_engine* e, int alg, const neb_desc* desc, uint32_t n, uint8_t* arena,
                                size_t arena_len, int32_t* status, uint32_t key_hint) {
    return batch_host(e, alg, 0, desc, n, arena, arena_len, status, key_hint);
}

NEB_API int neb_open_batch_host(neb_engine* e, int alg, const neb_desc* desc, uint32_t n, uint8_t* arena,
                                size_t arena_len, int32_t* status, uint32_t key_hint) {
    return batch_host(e, alg, 1, desc, n, arena, arena_len, status, key_hint);
}

// ---- pipelined receive (window.cpp) -----------------------------------------------------------
// The caller has validated every descriptor. begin: true = the arena is mapped pinned memory and
// zero-copy is the host mode; the pipeline is then reserved for the caller (e->rx.mu) until end.
// false with *rc == NEB_OK: use the synchronous neb_open_batch_host instead.

bool neb_rx_pipe_begin(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t n, uint32_t nchunks,
                       neb_desc** h_desc, int32_t** h_status, int* rc) {
    *rc = check_batch(e, alg, key_hint);
    if (*rc != NEB_OK || n == 0 || host_mode() != kHostZeroCopy || !host_mapped(arena)) return false;
    auto& r = e->rx;
    r.mu.lock();
    hipSetDevice(e->device);
    auto fail = [&] {
        r.mu.unlock();
        *rc = NEB_ERR_HIP;
        return false;
    };
    while (r.slot.size() < nchunks) {
        neb_engine::RxSlot sl;
        sl.sched = new (std::nothrow) SchedSpace;
        // the kernels' stores into the mapped arena must be visible to the host at the event
        if (!sl.sched || hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming | hipEventReleaseToSystem) != hipSuccess) {
            if (sl.stream) hipStreamDestroy(sl.stream);
            delete sl.sched;
            return fail();
        }
        r.slot.push_back(sl);
    }
    if (n > r.cap) {
        for (auto& sl : r.slot)
            if (hipStreamSynchronize(sl.stream) != hipSuccess) return fail();
        if (r.h_desc) hipHostFree(r.h_desc);
        if (r.h_status) hipHostFree(r.h_status);
        if (r.d_desc) hipFree(r.d_desc);
        if (r.d_status) hipFree(r.d_status);
        r.h_desc = nullptr;
        r.h_status = nullptr;
        r.d_desc = nullptr;
        r.d_status = nullptr;
        r.cap = 0;
        if (hipHostMalloc((void**)&r.h_desc, (size_t)n * sizeof(neb_desc), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&r.h_status, (size_t)n * sizeof(int32_t), hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void**)&r.d_desc, (size_t)n * sizeof(neb_desc)) != hipSuccess ||
            hipMalloc((void**)&r.d_status, (size_t)n * sizeof(int32_t)) != hipSuccess)
            return fail();
        r.cap = n;
    }
    *h_desc = r.h_desc;
    *h_status = r.h_status;
    return true;
}

// Queue chunk k: descriptors [c0, c0 + cnt) of the staging buffer, opened zero-copy in the arena.
int neb_rx_pipe_submit(neb_engine* e, int alg, uint32_t key_hint, uint8_t* arena, uint32_t c0, uint32_t cnt,
                       uint32_t k) {
    auto& r = e->rx;
    auto& sl = r.slot[k];
    HIP_TRY(hipMemcpyAsync(r.d_desc + c0, r.h_desc + c0, (size_t)cnt * sizeof(neb_desc), hipMemcpyHostToDevice,
                           sl.stream));
    HIP_TRY(launch_batch(e, alg, 1, r.d_desc + c0, cnt, arena, r.d_status + c0, key_hint, sl.stream, nullptr,
                         sl.sched));
    HIP_TRY(hipMemcpyAsync(r.h_status + c0, r.d_status + c0, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost,
                           sl.stream));
    HIP_TRY(hipEventRecord(sl.ev, sl.stream));
    return NEB_OK;
}

int neb_rx_pipe_wait(neb_engine* e, uint32_t k) {
    HIP_TRY(hipEventSynchronize(e->rx.slot[k].ev));
    return NEB_OK;
}

void neb_rx_pipe_end(neb_engine* e) {
    for (auto& sl : e->rx.slot) hipStreamSynchronize(sl.stream);
    e->rx.mu.unlock();
}

// ---- transmit batch (tx.hip) ------------------------------------------------------------------

static hipError_t tx_reserve(neb_engine* e, uint32_t n, uint32_t ntun, uint32_t max_wires) {
    TxSpace& tx = e->tx;
    if (!tx.done) {
        // ordering only, as SchedSpace::done: no system-scope cache release at each record
        hipError_t err = hipEventCreateWithFlags(&tx.done, hipEventDisableTiming | hipEventDisableSystemFence);
        if (err != hipSuccess) return err;
    }
    if (tx.mem && n <= tx.n_cap && ntun <= tx.tun_cap && max_wires <= tx.wire_cap) return hipSuccess;
    const uint32_t nc = std::max({n, tx.n_cap, 1024u}), tc = std::max({ntun, tx.tun_cap, 64u});
    const uint32_t wc = std::max({max_wires, tx.wire_cap, 1024u});
    size_t cub = 0;
    const size_t bytes = neb_tx_ws_bytes(nc, tc, wc, &cub);
    hipError_t err = hipEventSynchronize(tx.done);  // the old workspace may still be in use
    if (err != hipSuccess) return err;
    if (tx.mem) hipFree(tx.mem);
    tx.mem = nullptr;
    tx.n_cap = tx.tun_cap = tx.wire_cap = 0;
    err = hipMalloc((void**)&tx.mem, bytes);
    if (err != hipSuccess) return err;
    neb::tx_ws_layout(nc, tc, wc, cub, tx.mem, &tx.ws);
    tx.bytes = bytes;
    tx.n_cap = nc;
    tx.tun_cap = tc;
    tx.wire_cap = wc;
    return hipSuccess;
}

// caller holds e->tx.mu
static int tx_run(neb_engine* e, int alg, neb_tx_tunnel* d_tun, uint32_t ntun, const neb_tx_packet* d_pk, uint32_t npk,
                  const uint8_t* d_in, uint8_t* d_out, size_t out_cap, neb_tx_wire* d_wires, int32_t* d_wire_status,
                  uint32_t max_wires, uint32_t* d_nwires, int32_t* d_pk_status, uint32_t key_hint, hipStream_t s) {
    TxSpace& tx = e->tx;
    HIP_TRY(tx_reserve(e, npk, ntun, max_wires));
    if (!tx.last.same(s)) HIP_TRY(hipStreamWaitEvent(s, tx.done, 0));
    HIP_TRY(neb_tx_plan(d_pk, npk, d_in, d_tun, ntun, e->d_keys, e->max_keys, alg, &tx.ws, out_cap, max_wires,
                        d_pk_status, d_nwires, s));
    // one tunnel key with AES-GCM: the seal sums the payload into the L4 checksums itself, so the
    // segment kernel does not read the payload (aes_gcm.hip gcm_csum_fix)
    const bool cs = neb::kTxSealFromInput && NEB_TX_CSUM_SEAL && alg == NEB_ALG_AESGCM && key_hint != NEB_KEYS_MIXED;
    const uint32_t cs_slots = cs ? neb_gcm_single_slots(max_wires, e->cu_count, 0, 2) : 0u;
    HIP_TRY(neb_tx_segment(d_pk, npk, d_in, d_tun, d_out, &tx.ws, d_wires, d_nwires, max_wires, e->cu_count, cs_slots,
                           s));
    HIP_TRY(launch_batch(e, alg, 0, tx.ws.seal_desc, max_wires, d_out, d_wire_status, key_hint, s, d_nwires, nullptr,
                         cs ? 2 : (int)neb::kTxSealFromInput));
    HIP_TRY(neb_tx_finish(d_tun, npk, ntun, &tx.ws, s));
    HIP_TRY(hipEventRecord(tx.done, s));
    tx.last.set(s);
    return NEB_OK;
}

NEB_API int neb_tx_seal_batch(neb_engine* e, int alg, neb_tx_tunnel* d_tunnels, uint32_t ntunnels,
                              const neb_tx_packet* d_packets, uint32_t npackets, const uint8_t* d_in,
                              uint8_t* d_out, size_t out_cap, neb_tx_wire* d_wires, int32_t* d_wire_status,
                              uint32_t max_wires, uint32_t* d_nwires, int32_t* d_packet_status, uint32_t key_hint,
                              void* stream) {
    int rc = check_batch(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (!d_nwires || (npackets && (!d_packets || !d_in || !d_packet_status || !d_tunnels)) ||
        (max_wires && (!d_out || !d_wires || !d_wire_status)))
        return NEB_ERR_INVALID;
    DeviceGuard dg(e->device);
    hipStream_t s = (hipStream_t)stream;
    if (npackets == 0) {
        HIP_TRY(hipMemsetAsync(d_nwires, 0, sizeof(uint32_t), s));
        return NEB_OK;
    }
    std::lock_guard<std::mutex> g(e->tx.mu);
    rc = tx_run(e, alg, d_tunnels, ntunnels, d_packets, npackets, d_in, d_out, out_cap, d_wires, d_wire_status,
                max_wires, d_nwires, d_packet_status, key_hint, s);
    if (rc == NEB_OK) note_use(e, key_hint, s);
    return rc;
}

NEB_API int neb_tx_seal_batch_host(neb_engine* e, int alg, neb_tx_tunnel* tunnels, uint32_t ntunnels,
                                   const neb_tx_packet* packets, uint32_t npackets, const uint8_t* in, size_t in_len,
                                   uint8_t* out, size_t out_cap, neb_tx_wire* wires, int32_t* wire_status,
                                   uint32_t max_wires, uint32_t* nwires, int32_t* packet_status, uint32_t key_hint) {
    int rc = check_batch(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (!nwires || (npackets && (!packets || !in || !packet_status || (ntunnels && !tunnels))) ||
        (max_wires && (!out || !wires || !wire_status)))
        return NEB_ERR_INVALID;
    *nwires = 0;
    if (npackets == 0) return NEB_OK;
    // the input span the packets touch, uploaded once
    uint64_t lo = ~0ull, hi = 0;
    for (uint32_t i = 0; i < npackets; i++) {
        if (!span_in(packets[i].in_off, packets[i].len, in_len)) return NEB_ERR_INVALID;
        lo = std::min(lo, packets[i].in_off);
        hi = std::max(hi, packets[i].in_off + packets[i].len);
    }
    lo &= ~(uint64_t)15;
    const size_t span = (size_t)(hi - lo);
    const size_t o_tun = 0, o_pk = align_up((size_t)ntunnels * sizeof(neb_tx_tunnel), 256);
    const size_t o_in = o_pk + align_up((size_t)npackets * sizeof(neb_tx_packet), 256);
    const size_t o_out = o_in + align_up(span, 256);
    const size_t o_w = o_out + align_up(out_cap, 256);
    const size_t o_ws = o_w + align_up((size_t)max_wires * sizeof(neb_tx_wire), 256);
    const size_t o_ps = o_ws + align_up((size_t)max_wires * 4, 256);
    const size_t o_n = o_ps + align_up((size_t)npackets * 4, 256);
    const size_t total = o_n + 256;
    std::vector<neb_tx_packet> rebased(packets, packets + npackets);
    for (auto& p : rebased) p.in_off -= lo;
    std::lock_guard<std::mutex> g(e->tx.mu);
    DeviceGuard dg(e->device);
    TxSpace& tx = e->tx;
    hipStream_t s = e->stream;
    if (total > tx.io_cap) {
        if (tx.done) HIP_TRY(hipEventSynchronize(tx.done));
        if (tx.d_io) hipFree(tx.d_io);
        tx.d_io = nullptr;
        tx.io_cap = 0;
        const size_t cap = align_up(total, 1 << 20);
        HIP_TRY(hipMalloc((void**)&tx.d_io, cap));
        tx.io_cap = cap;
    }
    uint8_t* d = tx.d_io;
    auto* d_tun = (neb_tx_tunnel*)(d + o_tun);
    auto* d_pk = (neb_tx_packet*)(d + o_pk);
    auto* d_wires = (neb_tx_wire*)(d + o_w);
    auto* d_wst = (int32_t*)(d + o_ws);
    auto* d_pst = (int32_t*)(d + o_ps);
    auto* d_n = (uint32_t*)(d + o_n);
    if (ntunnels) HIP_TRY(hipMemcpyAsync(d_tun, tunnels, ntunnels * sizeof(neb_tx_tunnel), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_pk, rebased.data(), npackets * sizeof(neb_tx_packet), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_in, in + lo, span, hipMemcpyHostToDevice, s));
    rc = tx_run(e, alg, d_tun, ntunnels, d_pk, npackets, d + o_in, d + o_out, out_cap, d_wires, d_wst, max_wires, d_n,
                d_pst, key_hint, s);
    if (rc != NEB_OK) return rc;
    unsigned long long tot[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(tot, tx.ws.totals, sizeof tot, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(packet_status, d_pst, npackets * 4, hipMemcpyDeviceToHost, s));
    if (ntunnels) HIP_TRY(hipMemcpyAsync(tunnels, d_tun, ntunnels * sizeof(neb_tx_tunnel), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t nw = (uint32_t)tot[0];
    if (nw) {
        HIP_TRY(hipMemcpyAsync(wires, d_wires, nw * sizeof(neb_tx_wire), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(wire_status, d_wst, nw * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(out, d + o_out, (size_t)tot[1], hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *nwires = nw;
    return NEB_OK;
}

// ---- several engines --------------------------------------------------------------

// One tunnel key is one install on every engine (a tunnel has exactly one eKey / dKey,
// connection_state.go:37-49): shard k may use a key slot only if engine k holds there the same
// install (slot_tag) as engine 0, whose key table defines the batch's keys. Keys put on every
// engine by one neb_cipher_create_multi agree; anything else — a slot destroyed and reinstalled
// on one engine, keys installed engine by engine — does not, and the packets of shard k that name
// such a slot get NEB_STATUS_BAD_KEY instead of being sealed or opened with another tunnel's key.
// bad[k] flags engine k's disagreeing slots (empty when all agree; any = some engine disagrees).
struct KeyFence {
    std::vector<std::vector<uint8_t>> bad;
    bool any = false;
    bool bad_key(uint32_t k, uint32_t key) const { return key < bad[k].size() && bad[k][key]; }
};
static KeyFence key_fence(neb_engine* const* es, uint32_t m) {
    KeyFence f;
    f.bad.resize(m);
    std::vector<neb_engine*> order(es, es + m);
    std::sort(order.begin(), order.end());
    order.erase(std::unique(order.begin(), order.end()), order.end());
    if (order.size() < 2) return f;
    for (neb_engine* e : order) e->key_mu.lock();
    for (uint32_t k = 1; k < m; k++) {
        neb_engine* a = es[0];
        neb_engine* b = es[k];
        if (a == b) continue;
        const uint32_t nk = std::max(a->max_keys, b->max_keys);
        std::vector<uint8_t> v(nk, 0);
        bool anyk = false;
        for (uint32_t s = 0; s < nk; s++) {
            const uint64_t ta = s < a->max_keys ? a->slot_tag[s] : 0, tb = s < b->max_keys ? b->slot_tag[s] : 0;
            const int aa = s < a->max_keys ? a->slot_alg[s] : 0, ab = s < b->max_keys ? b->slot_alg[s] : 0;
            if (ta != tb || aa != ab) v[s] = 1, anyk = true;
        }
        if (anyk) {
            f.bad[k] = std::move(v);
            f.any = true;
        }
    }
    for (neb_engine* e : order) e->key_mu.unlock();
    if (f.any) {  // the call still returns NEB_OK (the packets carry NEB_STATUS_BAD_KEY): say why
        uint32_t first = 0, slots = 0;
        for (uint32_t k = m; k-- > 1;)
            if (!f.bad[k].empty()) first = k;
        for (uint8_t x : f.bad[first]) slots += x;
        std::snprintf(g_last_error, sizeof g_last_error,
                      "key fence: engine %u holds other installs than engine 0 in %u key slot(s); their packets get "
                      "NEB_STATUS_BAD_KEY (install a tunnel key on every engine with neb_cipher_create_multi)",
                      first, slots);
    }
    return f;
}

// Shard k of m: packets [n*k/m, n*(k+1)/m).
static inline uint32_t shard_lo(uint32_t n, uint32_t k, uint32_t m) { return (uint32_t)((uint64_t)n * k / m); }

static int batch_host_multi(neb_engine* const* engines, uint32_t m, int alg, int open, const neb_desc* desc,
                            uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status, uint32_t key_hint) {
    if (!engines || m == 0 || (n && (!desc || !arena || !status))) return NEB_ERR_INVALID;
    for (uint32_t k = 0; k < m; k++)
        if (!engines[k]) return NEB_ERR_INVALID;
    // every descriptor checked before any shard starts: an invalid batch touches nothing
    for (uint32_t i = 0; i < n; i++)
        if (!neb_desc_in_arena(desc[i], open, arena_len)) return NEB_ERR_INVALID;
    DeviceGuard dg;
    const KeyFence fence = key_fence(engines, m);
    // a shard whose engine disagrees on some keys runs on a copy of its descriptors with those
    // packets' key_id pointing past every key table (the kernels give them NEB_STATUS_BAD_KEY); a
    // single-key shard whose key disagrees is refused whole without a launch
    std::vector<std::vector<neb_desc>> fenced(m);
    std::vector<uint8_t> skip(m, 0);
    if (fence.any)
        for (uint32_t k = 1; k < m; k++) {
            if (fence.bad[k].empty()) continue;
            const uint32_t b = shard_lo(n, k, m), c = shard_lo(n, k + 1, m) - b;
            if (key_hint != NEB_KEYS_MIXED) {
                if (fence.bad_key(k, key_hint)) {
                    skip[k] = 1;
                    for (uint32_t i = 0; i < c; i++) status[b + i] = NEB_STATUS_BAD_KEY;
                }
                continue;
            }
            fenced[k].assign(desc + b, desc + b + c);
            for (neb_desc& d : fenced[k])
                if (fence.bad_key(k, d.key_id)) d.key_id = NEB_KEYS_MIXED - 1u;
        }
    auto run = [&](uint32_t k) -> int {
        const uint32_t b = shard_lo(n, k, m), c = shard_lo(n, k + 1, m) - b;
        if (skip[k]) return NEB_OK;
        const neb_desc* dk = fenced[k].empty() ? desc + b : fenced[k].data();
        return batch_host(engines[k], alg, open, dk, c, arena, arena_len, status + b, key_hint);
    };
    // A staged (not zero-copy) shard copies its whole arena span [lo & ~15, hi) in and back. Shards
    // whose spans meet (packed, unaligned or interleaved descriptors) would write stale bytes over
    // each other's results, so they run one after another; disjoint spans run side by side.
    bool serial = false;
    if (!(host_mode() == kHostZeroCopy && host_mapped(arena))) {
        std::vector<std::pair<uint64_t, uint64_t>> span;
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t b = shard_lo(n, k, m), c = shard_lo(n, k + 1, m) - b;
            if (c == 0 || skip[k]) continue;
            uint64_t lo = ~0ULL, hi = 0;
            for (uint32_t i = b; i < b + c; i++) {
                const neb_desc& d = desc[i];
                const uint64_t pay = (uint64_t)d.len + (open ? 16u : 0u), outl = (uint64_t)d.len + (open ? 0u : 16u);
                lo = std::min({lo, d.src_off, d.dst_off, d.aad_off});
                hi = std::max({hi, d.src_off + pay, d.dst_off + outl, d.aad_off + d.aad_len});
            }
            span.push_back({lo & ~(uint64_t)15, hi});
        }
        std::sort(span.begin(), span.end());
        for (size_t i = 1; i < span.size(); i++)
            if (span[i].first < span[i - 1].second) serial = true;
    }
    std::vector<int> rc(m, NEB_OK);
    if (serial) {
        for (uint32_t k = 0; k < m; k++) rc[k] = run(k);
    } else {
        std::vector<std::thread> th;
        for (uint32_t k = 1; k < m; k++) th.emplace_back([&, k] { rc[k] = run(k); });
        rc[0] = run(0);
        for (auto& t : th) t.join();
    }
    for (int r : rc)
        if (r != NEB_OK) return r;
    return NEB_OK;
}

NEB_API int neb_seal_batch_host_multi(neb_engine* const* engines, uint32_t nengines, int alg, const neb_desc* desc,
                                      uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status,
                                      uint32_t key_hint) {
    return batch_host_multi(engines, nengines, alg, 0, desc, n, arena, arena_len, status, key_hint);
}

NEB_API int neb_open_batch_host_multi(neb_engine* const* engines, uint32_t nengines, int alg, const neb_desc* desc,
                                      uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status,
                                      uint32_t key_hint) {
    return batch_host_multi(engines, nengines, alg, 1, desc, n, arena, arena_len, status, key_hint);
}

static int batch_sharded(int alg, int open, const neb_shard* sh, uint32_t m, uint32_t key_hint) {
    if (!sh || m == 0) return NEB_ERR_INVALID;
    for (uint32_t k = 0; k < m; k++)
        if (!sh[k].e) return NEB_ERR_INVALID;
    DeviceGuard dg;
    std::vector<neb_engine*> es(m);
    for (uint32_t k = 0; k < m; k++) es[k] = sh[k].e;
    const KeyFence fence = key_fence(es.data(), m);
    // device copies of a fenced shard's descriptors (KeyFence; batch_host_multi), freed at the end
    std::vector<void*> temps;
    int rc = NEB_OK;
    uint32_t launched = 0;
    for (; launched < m && rc == NEB_OK; launched++) {  // every shard queued first, then all waited for
        const neb_shard& s = sh[launched];
        const neb_desc* d_desc = s.d_desc;
        if (fence.any && !fence.bad[launched].empty() && s.n) {
            hipSetDevice(s.e->device);
            hipStream_t st = (hipStream_t)s.stream;
            if (key_hint != NEB_KEYS_MIXED) {
                if (fence.bad_key(launched, key_hint)) {
                    if (!s.d_status || hipMemsetD32Async((hipDeviceptr_t)s.d_status, NEB_STATUS_BAD_KEY, s.n, st) !=
                                           hipSuccess)
                        rc = s.d_status ? NEB_ERR_HIP : NEB_ERR_INVALID;
                    continue;
                }
            } else {
                const std::vector<uint8_t>& bad = fence.bad[launched];
                void* t = nullptr;
                const size_t db = align_up((size_t)s.n * sizeof(neb_desc), 256);
                if (!s.d_desc || hipMalloc(&t, db + bad.size()) != hipSuccess) {
                    rc = s.d_desc ? NEB_ERR_HIP : NEB_ERR_INVALID;
                    continue;
                }
                temps.push_back(t);
                uint8_t* d_bad = (uint8_t*)t + db;
                if (hipMemcpyAsync(d_bad, bad.data(), bad.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
                    neb_fence_keys(s.d_desc, (neb_desc*)t, s.n, d_bad, (uint32_t)bad.size(), st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess) {  // `bad` is pageable and local
                    rc = NEB_ERR_HIP;
                    continue;
                }
                d_desc = (const neb_desc*)t;
            }
        }
        rc = batch_device(s.e, alg, open, d_desc, s.n, s.d_arena, s.d_status, key_hint, s.stream);
    }
    for (uint32_t k = 0; k < launched; k++) {
        hipSetDevice(sh[k].e->device);
        const hipError_t err = hipStreamSynchronize((hipStream_t)sh[k].stream);
        if (err != hipSuccess && rc == NEB_OK) {
            set_error("sharded batch", err);
            rc = NEB_ERR_HIP;
        }
    }
    for (void* t : temps) hipFree(t);
    return rc;
}

NEB_API int neb_seal_batch_sharded(int alg, const neb_shard* shards, uint32_t nshards, uint32_t key_hint) {
    return batch_sharded(alg, 0, shards, nshards, key_hint);
}

NEB_API int neb_open_batch_sharded(int alg, const neb_shard* shards, uint32_t nshards, uint32_t key_hint) {
    return batch_sharded(alg, 1, shards, nshards, key_hint);
}

NEB_API int neb_host_alloc(size_t bytes, void** out) {
    if (!out || !bytes) return NEB_ERR_INVALID;
    return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? NEB_OK : NEB_ERR_HIP;
}

NEB_API int neb_host_free(void* p) {
    if (!p) return NEB_ERR_INVALID;
    return hipHostFree(p) == hipSuccess ? NEB_OK : NEB_ERR_HIP;
}

// header/header.go:102-110
NEB_API void neb_header_encode(uint8_t b[16], uint8_t version, uint8_t type, uint8_t subtype, uint32_t remote_index,
                               uint64_t counter) {
    b[0] = (uint8_t)(version << 4 | (type & 0x0f));
    b[1] = subtype;
    b[2] = 0;
    b[3] = 0;
    for (int i = 0; i < 4; i++) b[4 + i] = (uint8_t)(remote_index >> (24 - 8 * i));
    for (int i = 0; i < 8; i++) b[8 + i] = (uint8_t)(counter >> (56 - 8 * i));
}

// header/header.go:143-156
NEB_API int neb_header_parse(const uint8_t* b, size_t len, uint8_t* version, uint8_t* type, uint8_t* subtype,
                             uint16_t* reserved, uint32_t* remote_index, uint64_t* counter) {
    if (!b || len < NEB_HEADER_LEN) return NEB_ERR_INVALID;
    if (version) *version = (b[0] >> 4) & 0x0f;
    if (type) *type = b[0] & 0x0f;
    if (subtype) *subtype = b[1];
    if (reserved) *reserved = (uint16_t)(b[2] << 8 | b[3]);
    if (remote_index) *remote_index = (uint32_t)b[4] << 24 | (uint32_t)b[5] << 16 | (uint32_t)b[6] << 8 | b[7];
    if (counter) {
        uint64_t c = 0;
        for (int i = 0; i < 8; i++) c = c << 8 | b[8 + i];
        *counter = c;
    }
    return NEB_OK;
}

}  // extern "C"
