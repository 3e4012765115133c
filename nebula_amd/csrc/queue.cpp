// queue.cpp — the C ABI of the submission queue (include/nebula_aead.h): queue_core.hpp's state
// machine over the engine. Staging is pinned, mapped host memory; each batch is one zero-copy
// kernel launch on its own stream (and mixed-key scheduler workspace).
#include <hip/hip_runtime.h>

#include <new>
#include <vector>

#include "hip_guard.hpp"
#include "queue_core.hpp"

extern "C" {  // engine.cpp, internal
void* neb_sched_space_new();
void neb_sched_space_free(void* p);
int neb_launch_on(neb_engine* e, int alg, int open, const neb_desc* desc, uint32_t n, uint8_t* arena,
                  int32_t* status, uint32_t key_hint, hipStream_t s, void* sched);
int neb_key_alg(neb_engine* e, uint32_t key);
int neb_engine_device_of(const neb_engine* e);
bool neb_host_mapped(const void* p);
}

namespace {

// One stream and mixed-key scheduler workspace per staging batch: consecutive batches run
// concurrently on the device (a small zero-copy batch is PCIe latency, not bandwidth). A batch is
// done when its stream has drained: only that batch is ever on it (a staging batch is relaunched
// only after every submitter has copied its results out), and the stream synchronize makes the
// kernel's stores into the mapped staging visible to the host, as for the zero-copy host batch.
struct HipDev {
    using Token = uint32_t;  // the staging batch's index (its stream)
    neb_engine* e = nullptr;
    int alg = 0, open = 0;
    std::vector<hipStream_t> stream;
    std::vector<void*> sched;
    int launch(uint32_t i, neb_desc* desc, uint32_t n, uint8_t* arena, int32_t* status, uint32_t hint, Token& tok) {
        tok = i;
        return neb_launch_on(e, alg, open, desc, n, arena, status, hint, stream[i], sched[i]);
    }
    int wait(Token& tok) { return hipStreamSynchronize(stream[tok]) == hipSuccess ? NEB_OK : NEB_ERR_HIP; }
    bool key_ok(uint32_t key) { return neb_key_alg(e, key) == alg; }
    bool mapped(const uint8_t* arena) { return neb_host_mapped(arena); }
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
    DeviceGuard dg(neb_engine_device_of(e));
    q->b.resize(c.depth);
    q->dev.stream.assign(c.depth, nullptr);
    q->dev.sched.assign(c.depth, nullptr);
    bool ok = true;
    for (uint32_t i = 0; i < c.depth; i++) {
        ok = ok && hipStreamCreateWithFlags(&q->dev.stream[i], hipStreamNonBlocking) == hipSuccess;
        q->dev.sched[i] = ok ? neb_sched_space_new() : nullptr;
        ok = ok && q->dev.sched[i];
    }
    for (auto& x : q->b) {
        ok = ok && hipHostMalloc((void**)&x.arena, c.arena_bytes, hipHostMallocDefault) == hipSuccess;
        ok = ok && hipHostMalloc((void**)&x.desc, (size_t)c.max_packets * sizeof(neb_desc), hipHostMallocDefault) ==
                       hipSuccess;
        ok = ok && hipHostMalloc((void**)&x.status, (size_t)c.max_packets * 4, hipHostMallocDefault) == hipSuccess;
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
    DeviceGuard dg(neb_engine_device_of(q->dev.e));
    for (hipStream_t st : q->dev.stream)
        if (st) hipStreamSynchronize(st);
    for (auto& x : q->b) {
        if (x.arena) hipHostFree(x.arena);
        if (x.desc) hipHostFree(x.desc);
        if (x.status) hipHostFree(x.status);
    }
    for (void* sp : q->dev.sched) neb_sched_space_free(sp);
    for (hipStream_t st : q->dev.stream)
        if (st) hipStreamDestroy(st);
    delete q;
    return NEB_OK;
}

NEB_API int neb_queue_flush(neb_queue* q) { return q ? q->flush() : NEB_ERR_INVALID; }

NEB_API int neb_queue_stats(neb_queue* q, uint64_t stats[4]) {
    if (!q || !stats) return NEB_ERR_INVALID;
    q->stats(stats);
    return NEB_OK;
}

NEB_API int neb_queue_phases(neb_queue* q, uint64_t ns[6]) {
    if (!q || !ns) return NEB_ERR_INVALID;
    q->phases(ns);
    return NEB_OK;
}

NEB_API int neb_queue_submit(neb_queue* q, const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len,
                             int32_t* status) {
    return q ? q->submit(desc, n, arena, arena_len, status) : NEB_ERR_INVALID;
}

}  // extern "C"
