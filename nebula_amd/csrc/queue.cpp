// queue.cpp — the C ABI of the submission queue (include/nebula_aead.h): queue_core.hpp's state
// machine over the engine. Staging is pinned, mapped host memory, each batch is one zero-copy
// kernel launch on the queue's stream (its own mixed-key scheduler workspace), and a HIP event with
// a system-scope release marks it done.
#include <hip/hip_runtime.h>

#include <new>

#include "queue_core.hpp"

extern "C" {  // engine.cpp, internal
void* neb_sched_space_new();
void neb_sched_space_free(void* p);
int neb_launch_on(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n, uint8_t* arena,
                  int32_t* status, uint32_t key_hint, hipStream_t s, void* sched);
int neb_key_alg(neb_engine* e, uint32_t key);
int neb_engine_device_of(const neb_engine* e);
}

namespace {

struct HipDev {
    using Token = hipEvent_t;
    neb_engine* e = nullptr;
    int alg = 0, open = 0;
    hipStream_t stream = nullptr;
    void* sched = nullptr;
    int launch(neb_desc* desc, uint32_t n, uint8_t* arena, int32_t* status, uint32_t hint, Token& ev) {
        int rc = neb_launch_on(e, alg, open, desc, n, arena, status, hint, stream, sched);
        if (rc == NEB_OK && hipEventRecord(ev, stream) != hipSuccess) rc = NEB_ERR_HIP;
        return rc;
    }
    int wait(Token& ev) { return hipEventSynchronize(ev) == hipSuccess ? NEB_OK : NEB_ERR_HIP; }
    bool key_ok(uint32_t key) { return neb_key_alg(e, key) == alg; }
};

}  // namespace

struct neb_queue : neb_q::Queue<HipDev> {};

extern "C" {

NEB_API int neb_queue_create(neb_engine* e, int alg, int open, const neb_queue_config* cfg, neb_queue** out) {
    if (!e || !out || (alg != NEB_ALG_AESGCM && alg != NEB_ALG_CHACHAPOLY) || (open != 0 && open != 1))
        return NEB_ERR_INVALID;
    *out = nullptr;
    neb_queue_config c = cfg ? *cfg : neb_queue_config{};
    if (!neb_q::normalize(c)) return NEB_ERR_INVALID;
    neb_queue* q = new (std::nothrow) neb_queue;
    if (!q) return NEB_ERR_INVALID;
    q->dev.e = e;
    q->dev.alg = alg;
    q->dev.open = open;
    q->open = open;
    q->cfg = c;
    hipSetDevice(neb_engine_device_of(e));
    q->b.resize(c.depth);
    bool ok = hipStreamCreateWithFlags(&q->dev.stream, hipStreamNonBlocking) == hipSuccess;
    q->dev.sched = ok ? neb_sched_space_new() : nullptr;
    ok = ok && q->dev.sched;
    for (auto& x : q->b) {
        ok = ok && hipHostMalloc((void**)&x.arena, c.arena_bytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&x.desc, (size_t)c.max_packets * sizeof(neb_desc), hipHostMallocDefault) ==
                       hipSuccess;
        ok = ok && hipHostMalloc((void**)&x.status, (size_t)c.max_packets * 4, hipHostMallocDefault) == hipSuccess;
        // release-to-system: the kernel's stores into the mapped staging are visible to the host
        // once the event completes
        ok = ok && hipEventCreateWithFlags(&x.tok, hipEventDisableTiming | hipEventReleaseToSystem) == hipSuccess;
    }
    if (!ok) {
        neb_queue_destroy(q);
        return NEB_ERR_HIP;
    }
    q->start();
    *out = q;
    return NEB_OK;
}

NEB_API int neb_queue_destroy(neb_queue* q) {
    if (!q) return NEB_ERR_INVALID;
    q->shutdown();
    hipSetDevice(neb_engine_device_of(q->dev.e));
    if (q->dev.stream) hipStreamSynchronize(q->dev.stream);
    for (auto& x : q->b) {
        if (x.arena) hipHostFree(x.arena);
        if (x.desc) hipHostFree(x.desc);
        if (x.status) hipHostFree(x.status);
        if (x.tok) hipEventDestroy(x.tok);
    }
    neb_sched_space_free(q->dev.sched);
    if (q->dev.stream) hipStreamDestroy(q->dev.stream);
    delete q;
    return NEB_OK;
}

NEB_API int neb_queue_flush(neb_queue* q) { return q ? q->flush() : NEB_ERR_INVALID; }

NEB_API int neb_queue_stats(neb_queue* q, uint64_t stats[4]) {
    if (!q || !stats) return NEB_ERR_INVALID;
    q->stats(stats);
    return NEB_OK;
}

NEB_API int neb_queue_submit(neb_queue* q, const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len,
                             int32_t* status) {
    return q ? q->submit(desc, n, arena, arena_len, status) : NEB_ERR_INVALID;
}

}  // extern "C"
