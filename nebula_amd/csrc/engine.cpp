// engine.cpp — host side of the C ABI in include/nebula_aead.h.
//
// Owns one HIP device per engine: its stream, the device key table, pinned staging for the
// per-packet CipherState calls, and the double-buffered host-resident batch pipeline. All packet
// arithmetic runs in the gfx950 kernels (aes_gcm.hip, chacha_poly.hip); there is no CPU path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/nebula_aead.h"
#include "layout.hpp"
#include "sched.hpp"
#include "tx.hpp"

extern "C" hipError_t neb_gcm_key_setup(const uint8_t* d_key, uint32_t* d_rec, hipStream_t s);
extern "C" hipError_t neb_gcm_batch_single(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                           const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                           int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                           int hdr_from_dst);
extern "C" hipError_t neb_gcm_batch_chunked(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                            const uint32_t* d_keys, uint32_t max_keys, int32_t* d_status,
                                            const uint32_t* d_sorted, const uint4* d_chunks,
                                            uint32_t* d_counters, uint32_t max_chunks, int cu_count,
                                            hipStream_t s, int hdr_from_dst);
extern "C" hipError_t neb_gcm_probe(void);
extern "C" uint32_t neb_gcm_single_slots(uint32_t n, int cu_count, int open, int hdr_from_dst);
#ifndef NEB_TX_CSUM_SEAL
#define NEB_TX_CSUM_SEAL 1  // 0: the segment kernel sums every checksum (A/B)
#endif
extern "C" hipError_t neb_chacha_key_setup(const uint8_t* d_key, uint32_t* d_rec, hipStream_t s);
extern "C" hipError_t neb_chacha_batch(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                       const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                       int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                       int hdr_from_dst);

// Device workspace of the mixed-key scheduler (sched.hpp). One per engine; a batch waits on the
// previous user's event before reusing it, so batches on different streams never overlap in it.
struct SchedSpace {
    uint8_t* mem = nullptr;
    size_t bytes = 0;
    uint32_t n_cap = 0;
    neb::SchedWs ws{};
    hipEvent_t done = nullptr;
    bool dirty = true;  // the bin counts need a clear (new buffer, or a batch that failed to launch)
    std::mutex mu;
};

namespace {

constexpr size_t kStageMin = 1 << 16;
constexpr int kPipeStreams = 3;
#ifndef NEB_PIPE_CHUNK
#define NEB_PIPE_CHUNK 8192
#endif
constexpr uint32_t kPipeChunkPkts = NEB_PIPE_CHUNK;  // packets per staged host chunk

struct PipeSlot {
    hipStream_t stream = nullptr;
    uint8_t* d_buf = nullptr;
    size_t d_cap = 0;
    neb_desc* d_desc = nullptr;
    int32_t* d_status = nullptr;
    neb_desc* h_desc = nullptr;  // pinned
    int32_t* h_status = nullptr; // pinned
    int32_t* user_status = nullptr;
    uint32_t user_begin = 0, count = 0;
    uint64_t lo = 0, hi = 0;      // arena span of the chunk in flight (count > 0)
    hipEvent_t done = nullptr;    // recorded after the chunk's span is back in the arena
    SchedSpace* sched = nullptr;  // own mixed-key workspace: the two pipeline streams never wait on each other
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// [off, off + len) lies inside [0, cap), written so that no sum can wrap around 2^64.
inline bool span_in(uint64_t off, uint64_t len, uint64_t cap) { return off <= cap && len <= cap - off; }

}  // namespace

// Every region a descriptor touches lies inside a host arena of arena_len bytes: the AAD, the
// source (payload, plus the tag when opening) and the destination (payload, plus the tag when
// sealing). Shared with window.cpp, which validates a receive batch before touching anything.
bool neb_desc_in_arena(const neb_desc& d, int open, size_t arena_len) {
    const uint64_t pay = (uint64_t)d.len + (open ? 16u : 0u), outl = (uint64_t)d.len + (open ? 0u : 16u);
    return span_in(d.src_off, pay, arena_len) && span_in(d.dst_off, outl, arena_len) &&
           span_in(d.aad_off, d.aad_len, arena_len);
}

namespace {

// Arena span copy across PCIe for the kernel-staged host path: each wave instruction moves 1 KiB of
// contiguous bytes (64 lanes x 16 B) and every lane has four loads in flight before its stores, so
// the link carries full-size requests instead of the 64-byte pieces the zero-copy kernels issue.
// dst and src are 16-byte aligned; the last nbytes % 16 bytes are copied one per lane.
__global__ __launch_bounds__(256) void span_copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                        size_t nbytes) {
    const size_t n16 = nbytes >> 4;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
        d4[i] = a;
        d4[i + stride] = b;
        d4[i + 2 * stride] = c;
        d4[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) d4[i] = s4[i];
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t < (nbytes & 15)) dst[(n16 << 4) + t] = src[(n16 << 4) + t];
}

// Two span copies in one launch, the first blocks0 workgroups on the first: a chunk's copy-in and
// the previous chunk's copy-back, so both PCIe directions carry traffic at once.
__global__ __launch_bounds__(256) void span_copy2_kernel(uint8_t* __restrict__ dst0, const uint8_t* __restrict__ src0,
                                                         size_t n0, uint32_t blocks0, uint8_t* __restrict__ dst1,
                                                         const uint8_t* __restrict__ src1, size_t n1) {
    const bool first = blockIdx.x < blocks0;
    uint8_t* dst = first ? dst0 : dst1;
    const uint8_t* src = first ? src0 : src1;
    const size_t nbytes = first ? n0 : n1;
    const size_t nblk = first ? blocks0 : gridDim.x - blocks0, blk = first ? blockIdx.x : blockIdx.x - blocks0;
    const size_t n16 = nbytes >> 4, stride = nblk * 256;
    size_t i = blk * 256 + threadIdx.x;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
        d4[i] = a;
        d4[i + stride] = b;
        d4[i + 2 * stride] = c;
        d4[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) d4[i] = s4[i];
    const size_t t = blk * 256 + threadIdx.x;
    if (t < (nbytes & 15)) dst[(n16 << 4) + t] = src[(n16 << 4) + t];
}

hipError_t span_copy2(uint8_t* dst0, const uint8_t* src0, size_t n0, uint8_t* dst1, const uint8_t* src1, size_t n1,
                      hipStream_t s) {
    const size_t b0 = std::min<size_t>(std::max<size_t>(((n0 >> 4) + 255) / 256, 1), 512);
    const size_t b1 = std::min<size_t>(std::max<size_t>(((n1 >> 4) + 255) / 256, 1), 512);
    hipLaunchKernelGGL(span_copy2_kernel, dim3((unsigned)(b0 + b1)), dim3(256), 0, s, dst0, src0, n0, (uint32_t)b0,
                       dst1, src1, n1);
    return hipGetLastError();
}

hipError_t span_copy(uint8_t* dst, const uint8_t* src, size_t nbytes, hipStream_t s) {
    if (!nbytes) return hipSuccess;
    const size_t blocks = std::min<size_t>(std::max<size_t>(((nbytes >> 4) + 255) / 256, 1), 1024);
    hipLaunchKernelGGL(span_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, nbytes);
    return hipGetLastError();
}

// Host batch path: NEB_HOST_MODE = "zc" (kernels on the mapped arena), "kcopy" (mapped arena staged
// by span_copy_kernel), "dma" (hipMemcpyAsync staging); NEB_HOST_STAGED=1 is the older name of "dma".
enum HostMode { kHostZeroCopy, kHostKernelCopy, kHostDma, kHostSplit };
// Zero-copy is the default: measured on one MI355X (C2 seal+open, 64 Ki x 1300 B) it runs at 28.4
// GiB/s against 23.9 for DMA staging and 18.1 for span-copy staging.
HostMode host_mode() {  // read per batch (a few hundred ns), so a process can switch between batches
    if (std::getenv("NEB_HOST_STAGED")) return kHostDma;
    const char* v = std::getenv("NEB_HOST_MODE");
    if (v && !std::strcmp(v, "kcopy")) return kHostKernelCopy;
    if (v && !std::strcmp(v, "dma")) return kHostDma;
    if (v && !std::strcmp(v, "split")) return kHostSplit;
    return kHostZeroCopy;
}

}  // namespace

// Device workspace of the transmit batch (tx.hpp) plus device staging for its host-memory form.
struct TxSpace {
    uint8_t* mem = nullptr;
    size_t bytes = 0;
    uint32_t n_cap = 0, tun_cap = 0, wire_cap = 0;
    neb::TxWs ws{};
    hipEvent_t done = nullptr;
    uint8_t* d_io = nullptr;  // neb_tx_seal_batch_host staging
    size_t io_cap = 0;
    std::mutex mu;
};

struct neb_engine {
    int device = 0;
    int cu_count = 0;
    hipStream_t stream = nullptr;
    uint32_t max_keys = 0;
    uint32_t* d_keys = nullptr;
    std::vector<int> slot_alg;  // 0 = free
    std::mutex key_mu;

    std::mutex io_mu;  // per-packet staging
    uint8_t* h_stage = nullptr;
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;

    std::mutex pipe_mu;
    PipeSlot pipe[kPipeStreams];
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
};

static thread_local char g_last_error[256] = "";

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

static int ensure_stage(neb_engine* e, size_t bytes) {
    if (bytes <= e->stage_cap) return NEB_OK;
    size_t cap = std::max(kStageMin, align_up(bytes, 1 << 16));
    if (e->h_stage) hipHostFree(e->h_stage);
    if (e->d_stage) hipFree(e->d_stage);
    e->h_stage = nullptr;
    e->d_stage = nullptr;
    e->stage_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&e->h_stage, cap, hipHostMallocDefault));
    HIP_TRY(hipMalloc((void**)&e->d_stage, cap));
    e->stage_cap = cap;
    return NEB_OK;
}

extern "C" {

NEB_API const char* neb_last_error(void) { return g_last_error; }

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
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void**)&e->d_keys, (size_t)max_keys * neb::kKeyRecBytes) != hipSuccess ||
        hipMemset(e->d_keys, 0, (size_t)max_keys * neb::kKeyRecBytes) != hipSuccess) {
        set_error("engine allocation", hipGetLastError());
        neb_engine_destroy(e);
        return NEB_ERR_HIP;
    }
    *out = e;
    return NEB_OK;
}

NEB_API int neb_engine_destroy(neb_engine* e) {
    if (!e) return NEB_ERR_INVALID;
    hipSetDevice(e->device);
    if (e->stream) hipStreamSynchronize(e->stream);
    for (auto& s : e->pipe) {
        if (s.stream) { hipStreamSynchronize(s.stream); hipStreamDestroy(s.stream); }
        if (s.done) hipEventDestroy(s.done);
        if (s.d_buf) hipFree(s.d_buf);
        if (s.d_desc) hipFree(s.d_desc);
        if (s.d_status) hipFree(s.d_status);
        if (s.h_desc) hipHostFree(s.h_desc);
        if (s.h_status) hipHostFree(s.h_status);
        if (s.sched) {
            if (s.sched->done) { hipEventSynchronize(s.sched->done); hipEventDestroy(s.sched->done); }
            if (s.sched->mem) hipFree(s.sched->mem);
            delete s.sched;
        }
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
    if (e->h_stage) hipHostFree(e->h_stage);
    if (e->d_stage) hipFree(e->d_stage);
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

NEB_API const char* neb_cipher_name(int alg) {
    return alg == NEB_ALG_AESGCM ? "AESGCM" : alg == NEB_ALG_CHACHAPOLY ? "ChaChaPoly" : nullptr;
}

NEB_API int neb_cipher_create(neb_engine* e, int alg, const uint8_t key[32], neb_cipher** out) {
    if (!e || !key || !out || (alg != NEB_ALG_AESGCM && alg != NEB_ALG_CHACHAPOLY)) return NEB_ERR_INVALID;
    *out = nullptr;
    uint32_t slot;
    {
        std::lock_guard<std::mutex> g(e->key_mu);
        auto it = std::find(e->slot_alg.begin(), e->slot_alg.end(), 0);
        if (it == e->slot_alg.end()) return NEB_ERR_NO_KEY_SLOT;
        slot = (uint32_t)(it - e->slot_alg.begin());
        *it = -1;  // reserved
    }
    int rc = NEB_OK;
    {
        std::lock_guard<std::mutex> g(e->io_mu);
        hipSetDevice(e->device);
        rc = ensure_stage(e, 64);
        if (rc == NEB_OK) {
            std::memcpy(e->h_stage, key, 32);
            uint32_t* rec = e->d_keys + (size_t)slot * neb::kKeyRecDwords;
            hipError_t err = hipMemcpyAsync(e->d_stage, e->h_stage, 32, hipMemcpyHostToDevice, e->stream);
            if (err == hipSuccess) err = hipMemsetAsync(rec, 0, neb::kKeyRecBytes, e->stream);
            if (err == hipSuccess)
                err = alg == NEB_ALG_AESGCM ? neb_gcm_key_setup(e->d_stage, rec, e->stream)
                                            : neb_chacha_key_setup(e->d_stage, rec, e->stream);
            if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
            std::memset(e->h_stage, 0, 32);
            if (err != hipSuccess) rc = NEB_ERR_HIP;
        }
    }
    std::lock_guard<std::mutex> g(e->key_mu);
    if (rc != NEB_OK) {
        e->slot_alg[slot] = 0;
        return rc;
    }
    neb_cipher* c = new (std::nothrow) neb_cipher{e, slot, alg};
    if (!c) {
        e->slot_alg[slot] = 0;
        return NEB_ERR_INVALID;
    }
    e->slot_alg[slot] = alg;
    *out = c;
    return NEB_OK;
}

NEB_API int neb_cipher_destroy(neb_cipher* c) {
    if (!c) return NEB_ERR_INVALID;
    neb_engine* e = c->e;
    hipSetDevice(e->device);
    // Asynchronous batches (neb_seal_batch / neb_open_batch / neb_tx_seal_batch / neb_rx_open_batch)
    // still queued on caller streams may read this record: the whole device drains first. A
    // destroy is rare; an event recorded after every launch instead cost 2-4 µs per kernel
    // (profiles/r2_micro/ab_inflight_events.log).
    hipDeviceSynchronize();
    {
        std::lock_guard<std::mutex> g(e->io_mu);
        hipMemsetAsync(e->d_keys + (size_t)c->key_id * neb::kKeyRecDwords, 0, neb::kKeyRecBytes, e->stream);
        hipStreamSynchronize(e->stream);
    }
    {
        std::lock_guard<std::mutex> g(e->key_mu);
        e->slot_alg[c->key_id] = 0;
    }
    delete c;
    return NEB_OK;
}

NEB_API uint32_t neb_cipher_key_id(const neb_cipher* c) { return c ? c->key_id : NEB_KEYS_MIXED; }
NEB_API int neb_cipher_alg(const neb_cipher* c) { return c ? c->alg : 0; }
NEB_API int neb_overhead(const neb_cipher* c) { return c ? NEB_OVERHEAD : 0; }

static void fill_nonce(int alg, uint64_t n, uint8_t* nb) {
    if (!nb) return;
    nb[0] = nb[1] = nb[2] = nb[3] = 0;
    for (int i = 0; i < 8; i++) nb[4 + i] = alg == NEB_ALG_AESGCM ? (uint8_t)(n >> (56 - 8 * i)) : (uint8_t)(n >> (8 * i));
}

// Size the scheduler workspace for n packets (caller holds sched.mu).
static hipError_t sched_reserve(neb_engine* e, SchedSpace& sp, uint32_t n) {
    if (!sp.done) {
        hipError_t err = hipEventCreateWithFlags(&sp.done, hipEventDisableTiming);
        if (err != hipSuccess) return err;
    }
    if (n <= sp.n_cap && sp.mem && !sp.dirty) return hipSuccess;
    if (n <= sp.n_cap && sp.mem) {  // the bins are cleared as they are consumed, except after a failure
        hipError_t err = hipEventSynchronize(sp.done);
        if (err == hipSuccess) err = hipMemset(sp.ws.counters, 0, (neb::kSchedCounters + 2u * neb::sched_nbins(e->max_keys)) * 4u);
        if (err == hipSuccess) sp.dirty = false;
        return err;
    }
    const uint32_t cap = std::max<uint32_t>(n, 1u << 16);
    const uint32_t nb = neb::sched_nbins(e->max_keys);
    const uint32_t mc = neb::sched_max_chunks(cap, e->max_keys);
    const size_t b_counters = align_up((neb::kSchedCounters + 2u * (size_t)nb) * 4u, 256);
    const size_t b_base = align_up((size_t)nb * 4u, 256);
    const size_t b_idx = align_up((size_t)cap * 4u, 256), b_chunks = (size_t)mc * 16u;
    const size_t bytes = b_counters + b_base + 3 * b_idx + b_chunks;
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
    sp.ws.fill = sp.ws.hist + nb;
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
    sp.ws.max_chunks = mc;
    sp.bytes = bytes;
    sp.n_cap = cap;
    err = hipMemset(sp.ws.counters, 0, b_counters);  // once: the binning clears its counts as it uses them
    if (err != hipSuccess) return err;
    sp.dirty = false;
    return hipSuccess;
}

// d_n (optional): the batch's real packet count in device memory, at most n (a batch whose size is
// only known on the device, e.g. the segments of a TX batch). hdr_from_dst: the TX batch's
// descriptors (tx.hip) read their first `flags` plaintext bytes from the destination.
static hipError_t launch_batch(neb_engine* e, int alg, int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                               int32_t* d_status, uint32_t key_hint, hipStream_t s, const uint32_t* d_n = nullptr,
                               SchedSpace* sched = nullptr, int hdr_from_dst = 0) {
    if (alg == NEB_ALG_AESGCM) {
        if (key_hint != NEB_KEYS_MIXED)
            return neb_gcm_batch_single(open, d_desc, n, d_arena, e->d_keys, e->max_keys, key_hint, d_status, d_n,
                                        e->cu_count, s, hdr_from_dst);
        // mixed keys: regroup into single-key, similar-size chunks on the device, then seal/open
        SchedSpace& sp = sched ? *sched : e->sched;
        std::lock_guard<std::mutex> g(sp.mu);
        hipError_t err = sched_reserve(e, sp, n);
        if (err == hipSuccess) err = hipStreamWaitEvent(s, sp.done, 0);
        if (err == hipSuccess) err = neb_sched_build(d_desc, n, d_n, e->max_keys, 4u, &sp.ws, s);
        if (err == hipSuccess)
            err = neb_gcm_batch_chunked(open, d_desc, n, d_arena, e->d_keys, e->max_keys, d_status, sp.ws.sorted,
                                        sp.ws.chunks, sp.ws.counters, sp.ws.max_chunks, e->cu_count, s, hdr_from_dst);
        if (err == hipSuccess) err = hipEventRecord(sp.done, s);
        if (err != hipSuccess) sp.dirty = true;
        return err;
    }
    return neb_chacha_batch(open, d_desc, n, d_arena, e->d_keys, e->max_keys, key_hint, d_status, d_n, e->cu_count,
                            s, hdr_from_dst);
}

// One packet through the device: [desc | status | aad | payload (+tag)] in one staging buffer.
static int one_packet(neb_cipher* c, int open, const uint8_t* ad, size_t ad_len, const uint8_t* in, size_t in_len,
                      size_t pay_len, uint64_t n, uint8_t* dst, int32_t* st_out) {
    neb_engine* e = c->e;
    const size_t o_desc = 0, o_status = 64, o_aad = 128;
    const size_t o_pay = align_up(o_aad + ad_len, 16);
    const size_t total = o_pay + pay_len + 16;
    std::lock_guard<std::mutex> g(e->io_mu);
    hipSetDevice(e->device);
    int rc = ensure_stage(e, total);
    if (rc != NEB_OK) return rc;
    uint8_t* h = e->h_stage;
    neb_desc d{};
    d.src_off = o_pay - o_aad;
    d.dst_off = o_pay - o_aad;
    d.aad_off = 0;
    d.counter = n;
    d.len = (uint32_t)pay_len;
    d.aad_len = (uint32_t)ad_len;
    d.key_id = c->key_id;
    std::memcpy(h + o_desc, &d, sizeof d);
    if (ad_len) std::memcpy(h + o_aad, ad, ad_len);
    if (in_len) std::memcpy(h + o_pay, in, in_len);
    hipError_t err = hipMemcpyAsync(e->d_stage, h, o_pay + in_len, hipMemcpyHostToDevice, e->stream);
    if (err == hipSuccess)
        err = launch_batch(e, c->alg, open, (const neb_desc*)(e->d_stage + o_desc), 1, e->d_stage + o_aad,
                           (int32_t*)(e->d_stage + o_status), c->key_id, e->stream);
    if (err != hipSuccess) set_error("one_packet", err);
    const size_t out_len = open ? pay_len : pay_len + 16;
    if (err == hipSuccess) err = hipMemcpyAsync(h + o_status, e->d_stage + o_status, 4, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess && out_len)
        err = hipMemcpyAsync(h + o_pay, e->d_stage + o_pay, out_len, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return NEB_ERR_HIP;
    std::memcpy(st_out, h + o_status, 4);
    if (out_len) std::memcpy(dst, h + o_pay, out_len);
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
    hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream, as for any HIP launch
    hipError_t err = launch_batch(e, alg, open, d_desc, n, d_arena, d_status, key_hint, s);
    if (err != hipSuccess) {
        set_error("batch launch", err);
        return NEB_ERR_HIP;
    }
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
                         uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, hipStream_t s) {
    if (n == 0) return NEB_OK;
    hipError_t err = launch_batch(e, alg, 1, d_desc, n, d_arena, d_status, key_hint, s, d_n);
    if (err != hipSuccess) {
        set_error("batch launch", err);
        return NEB_ERR_HIP;
    }
    return NEB_OK;
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
// overlaps another's kernel and another's copy-back. NEB_HOST_MODE=kcopy stages a mapped arena with
// span_copy_kernel instead (measured slower, kept for the A/B); =dma forces hipMemcpyAsync staging.
// Every descriptor is checked before anything is copied or launched, in every mode: an invalid batch
// returns NEB_ERR_INVALID with the arena and the statuses untouched.
static int batch_host(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n, uint8_t* arena,
                      size_t arena_len, int32_t* status, uint32_t key_hint) {
    int rc = check_batch(e, alg, key_hint);
    if (rc != NEB_OK) return rc;
    if (n == 0) return NEB_OK;
    if (!desc || !arena || !status) return NEB_ERR_INVALID;
    for (uint32_t i = 0; i < n; i++)
        if (!neb_desc_in_arena(desc[i], open, arena_len)) return NEB_ERR_INVALID;
    std::lock_guard<std::mutex> g(e->pipe_mu);
    hipSetDevice(e->device);
    const HostMode mode = host_mode();
    // The kernels' vector fast path tests the absolute address (arena base + offset), so a mapped
    // arena at any byte address runs zero-copy. A staged arena lands in a device buffer with the
    // same alignment modulo 16, so the kernels take the same paths either way.
    const bool mapped = mode != kHostDma && host_mapped(arena);
    if (mapped && mode == kHostZeroCopy)
        return batch_host_zero_copy(e, alg, open, desc, n, arena, arena_len, status, key_hint);
    // mapped arena: copies by span_copy_kernel, whose 16-byte vector copies need an aligned base
    // (an unaligned one is DMA-staged)
    const bool kcopy = mapped && mode == kHostKernelCopy && ((uintptr_t)arena & 15) == 0;
    // split (mapped arena): each chunk's sources (payload, AAD) are DMA-staged into a device buffer
    // while the kernel stores its outputs straight into the mapped arena, so the copy engine carries
    // the H2D direction and the kernel's stores the D2H one, and nothing is copied back.
    const bool split = mapped && mode == kHostSplit;
    for (auto& s : e->pipe) {
        if (!s.stream) {
            HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
            // system-scope release: a split chunk's kernel stores into the mapped arena, which is
            // non-coherent (L2-cached) host memory by default; the event must make them visible
            HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming | hipEventReleaseToSystem));
            HIP_TRY(hipMalloc((void**)&s.d_desc, kPipeChunkPkts * sizeof(neb_desc)));
            HIP_TRY(hipMalloc((void**)&s.d_status, kPipeChunkPkts * sizeof(int32_t)));
            HIP_TRY(hipHostMalloc((void**)&s.h_desc, kPipeChunkPkts * sizeof(neb_desc), hipHostMallocDefault));
            HIP_TRY(hipHostMalloc((void**)&s.h_status, kPipeChunkPkts * sizeof(int32_t), hipHostMallocDefault));
        }
        if (!s.sched) {
            s.sched = new (std::nothrow) SchedSpace;
            if (!s.sched) return NEB_ERR_INVALID;
        }
        s.count = 0;
    }
    // kcopy: every chunk runs on pipe[0]'s stream and chunk k's copy-in shares one launch with chunk
    // k-1's copy-back (span_copy2), unless their spans overlap; `pend` is the slot whose copy-back
    // has not been issued yet. DMA staging: one stream per slot, chunks overlap across streams.
    hipStream_t ks = e->pipe[0].stream;
    int slot = 0, pend = -1;
    auto retire = [](PipeSlot& s) -> hipError_t {
        hipError_t err = hipEventSynchronize(s.done);
        if (err != hipSuccess) return err;
        std::memcpy(s.user_status + s.user_begin, s.h_status, s.count * sizeof(int32_t));
        s.count = 0;
        return hipSuccess;
    };
    for (uint32_t begin = 0; begin < n; begin += kPipeChunkPkts, slot = (slot + 1) % kPipeStreams) {
        PipeSlot& s = e->pipe[slot];
        if (s.count) HIP_TRY(retire(s));  // retire this slot's previous chunk before reusing its buffers
        const uint32_t cnt = std::min(kPipeChunkPkts, n - begin);
        uint64_t lo = ~0ULL, hi = 0;  // every sum below stays within arena_len (checked above)
        for (uint32_t i = 0; i < cnt; i++) {
            const neb_desc& d = desc[begin + i];
            const uint64_t pay = (uint64_t)d.len + (open ? 16u : 0u), outl = (uint64_t)d.len + (open ? 0u : 16u);
            if (split) {  // only what the kernel reads is staged
                lo = std::min({lo, d.src_off, d.aad_off});
                hi = std::max({hi, d.src_off + pay, d.aad_off + d.aad_len});
            } else {
                lo = std::min({lo, d.src_off, d.dst_off, d.aad_off});
                hi = std::max({hi, d.src_off + pay, d.dst_off + outl, d.aad_off + d.aad_len});
            }
        }
        lo &= ~(uint64_t)15;
        // A chunk copies its whole span back, so spans of chunks in flight must not overlap (the
        // descriptors need not be in arena order): retire any other slot whose span intersects.
        // (kcopy chunks are ordered by their one stream; only the launch shared with `pend` races.)
        if (!kcopy && !split)
            for (auto& o : e->pipe)
                if (&o != &s && o.count && o.lo < hi && lo < o.hi) HIP_TRY(retire(o));
        s.lo = lo;
        s.hi = hi;
        const size_t span = (size_t)(hi - lo);
        if (span > s.d_cap) {
            if (s.d_buf) { HIP_TRY(hipStreamSynchronize(s.stream)); hipFree(s.d_buf); s.d_buf = nullptr; s.d_cap = 0; }
            size_t cap = align_up(span, 1 << 20);
            HIP_TRY(hipMalloc((void**)&s.d_buf, cap));
            s.d_cap = cap;
        }
        for (uint32_t i = 0; i < cnt; i++) {
            neb_desc d = desc[begin + i];
            d.src_off -= lo;
            d.aad_off -= lo;
            // split: the kernel's d_buf + dst_off must land on the mapped arena (64-bit wrap-around)
            d.dst_off = split ? (uint64_t)(uintptr_t)(arena + d.dst_off) - (uint64_t)(uintptr_t)s.d_buf : d.dst_off - lo;
            s.h_desc[i] = d;
        }
        s.user_status = status;
        s.user_begin = begin;
        s.count = cnt;
        if (kcopy) {
            HIP_TRY(hipMemcpyAsync(s.d_desc, s.h_desc, cnt * sizeof(neb_desc), hipMemcpyHostToDevice, ks));
            if (pend >= 0) {
                PipeSlot& p = e->pipe[pend];
                const size_t pspan = (size_t)(p.hi - p.lo);
                if (p.lo < hi && lo < p.hi) {  // overlapping spans: copy back first, then copy in
                    HIP_TRY(span_copy(arena + p.lo, p.d_buf, pspan, ks));
                    HIP_TRY(span_copy(s.d_buf, arena + lo, span, ks));
                } else {
                    HIP_TRY(span_copy2(s.d_buf, arena + lo, span, arena + p.lo, p.d_buf, pspan, ks));
                }
                HIP_TRY(hipEventRecord(p.done, ks));
            } else {
                HIP_TRY(span_copy(s.d_buf, arena + lo, span, ks));
            }
            HIP_TRY(launch_batch(e, alg, open, s.d_desc, cnt, s.d_buf, s.d_status, key_hint, ks, nullptr, s.sched));
            HIP_TRY(hipMemcpyAsync(s.h_status, s.d_status, cnt * sizeof(int32_t), hipMemcpyDeviceToHost, ks));
            pend = slot;
            continue;
        }
        HIP_TRY(hipMemcpyAsync(s.d_desc, s.h_desc, cnt * sizeof(neb_desc), hipMemcpyHostToDevice, s.stream));
        HIP_TRY(hipMemcpyAsync(s.d_buf, arena + lo, span, hipMemcpyHostToDevice, s.stream));
        HIP_TRY(launch_batch(e, alg, open, s.d_desc, cnt, s.d_buf, s.d_status, key_hint, s.stream, nullptr, s.sched));
        if (split) {
            HIP_TRY(hipMemcpyAsync(s.h_status, s.d_status, cnt * sizeof(int32_t), hipMemcpyDeviceToHost, s.stream));
            HIP_TRY(hipEventRecord(s.done, s.stream));
            continue;
        }
        HIP_TRY(hipMemcpyAsync(arena + lo, s.d_buf, span, hipMemcpyDeviceToHost, s.stream));
        HIP_TRY(hipMemcpyAsync(s.h_status, s.d_status, cnt * sizeof(int32_t), hipMemcpyDeviceToHost, s.stream));
        HIP_TRY(hipEventRecord(s.done, s.stream));
    }
    if (pend >= 0) {
        PipeSlot& p = e->pipe[pend];
        HIP_TRY(span_copy(arena + p.lo, p.d_buf, (size_t)(p.hi - p.lo), ks));
        HIP_TRY(hipEventRecord(p.done, ks));
    }
    for (auto& s : e->pipe)
        if (s.count) HIP_TRY(retire(s));
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
        hipError_t err = hipEventCreateWithFlags(&tx.done, hipEventDisableTiming);
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
    HIP_TRY(hipStreamWaitEvent(s, tx.done, 0));
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
    hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;
    if (npackets == 0) {
        HIP_TRY(hipMemsetAsync(d_nwires, 0, sizeof(uint32_t), s));
        return NEB_OK;
    }
    std::lock_guard<std::mutex> g(e->tx.mu);
    rc = tx_run(e, alg, d_tunnels, ntunnels, d_packets, npackets, d_in, d_out, out_cap, d_wires, d_wire_status,
                max_wires, d_nwires, d_packet_status, key_hint, s);
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
    hipSetDevice(e->device);
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
