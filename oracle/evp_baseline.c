/*
 * evp_baseline.c — TEST/BENCH INFRASTRUCTURE ONLY (the `cpu_baseline` leg of bench.py, and a
 * second independent checker for tests/).
 *
 * A CPU port of the reference's per-packet seal/open loop (noiseutil/aesgcm.go:24-49,
 * noiseutil/chachapoly.go:23-48 driven as inside.go:123-146 / connection_state.go:99-119 drive
 * them) on OpenSSL libcrypto EVP. The Go reference cannot be built here (no Go toolchain); its
 * arithmetic runs in the Go stdlib's AES-NI + PCLMULQDQ assembly, and EVP's AES-GCM /
 * ChaCha20-Poly1305 are the same class of implementation (AES-NI/VAES + PCLMULQDQ, AVX2/AVX-512
 * ChaCha). Like Go's cipher.AEAD, one context per tunnel key holds the expanded key; each packet
 * only sets the 12-byte nonce.
 *
 * Threads: each thread takes a contiguous slice of the packet list, pinned to core (tid % ncpu).
 */
#define _GNU_SOURCE
#include <openssl/evp.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define EVB_API __attribute__((visibility("default")))

typedef struct {
    uint64_t src_off, dst_off, aad_off, counter;
    uint32_t len, aad_len, key_id, flags;
} evb_desc;

typedef struct {
    int alg, open, tid, pin;
    const uint8_t* keys;
    uint32_t nkeys;
    const evb_desc* d;
    size_t begin, end;
    uint8_t* arena;
    int32_t* status;
    int iters;
    long failures;
} evb_job;

static void mk_nonce(int alg, uint64_t n, uint8_t nb[12]) {
    nb[0] = nb[1] = nb[2] = nb[3] = 0;
    for (int i = 0; i < 8; i++) nb[4 + i] = alg == 1 ? (uint8_t)(n >> (56 - 8 * i)) : (uint8_t)(n >> (8 * i));
}

static void* evb_worker(void* arg) {
    evb_job* j = (evb_job*)arg;
    if (j->pin >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->pin, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const EVP_CIPHER* ciph = j->alg == 1 ? EVP_aes_256_gcm() : EVP_chacha20_poly1305();
    EVP_CIPHER_CTX** ctx = (EVP_CIPHER_CTX**)calloc(j->nkeys, sizeof(*ctx));
    for (int it = 0; it < j->iters; it++) {
        for (size_t i = j->begin; i < j->end; i++) {
            const evb_desc* d = &j->d[i];
            EVP_CIPHER_CTX* c = ctx[d->key_id];
            if (!c) {
                c = ctx[d->key_id] = EVP_CIPHER_CTX_new();
                if (j->open) EVP_DecryptInit_ex(c, ciph, NULL, j->keys + 32 * (size_t)d->key_id, NULL);
                else EVP_EncryptInit_ex(c, ciph, NULL, j->keys + 32 * (size_t)d->key_id, NULL);
            }
            uint8_t nb[12];
            int outl = 0, finl = 0;
            mk_nonce(j->alg, d->counter, nb);
            uint8_t* aad = j->arena + d->aad_off;
            uint8_t* src = j->arena + d->src_off;
            uint8_t* dst = j->arena + d->dst_off;
            if (!j->open) {
                EVP_EncryptInit_ex(c, NULL, NULL, NULL, nb);
                EVP_EncryptUpdate(c, NULL, &outl, aad, (int)d->aad_len);
                EVP_EncryptUpdate(c, dst, &outl, src, (int)d->len);
                EVP_EncryptFinal_ex(c, dst + outl, &finl);
                EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, dst + d->len);
                if (j->status) j->status[i] = 0;
            } else {
                uint8_t tag[16];
                memcpy(tag, src + d->len, 16);
                EVP_DecryptInit_ex(c, NULL, NULL, NULL, nb);
                EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, tag);
                EVP_DecryptUpdate(c, NULL, &outl, aad, (int)d->aad_len);
                EVP_DecryptUpdate(c, dst, &outl, src, (int)d->len);
                int ok = EVP_DecryptFinal_ex(c, dst + outl, &finl) > 0;
                if (!ok) {
                    memset(dst, 0, d->len);
                    j->failures++;
                }
                if (j->status) j->status[i] = ok ? 0 : 1;
            }
        }
    }
    for (uint32_t k = 0; k < j->nkeys; k++)
        if (ctx[k]) EVP_CIPHER_CTX_free(ctx[k]);
    free(ctx);
    return NULL;
}

/* Seal (open=0) or open (open=1) desc[0..n) `iters` times over `threads` pinned threads.
 * Returns wall seconds; *failures = auth failures counted in the last pass type. */
EVB_API double evb_run(int alg, int open, const uint8_t* keys, uint32_t nkeys, const evb_desc* d, size_t n,
                       uint8_t* arena, int32_t* status, int threads, int iters, int pin, long* failures) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    evb_job* jobs = (evb_job*)calloc((size_t)threads, sizeof(evb_job));
    /* pin only to CPUs this process may use (a GPU box grants a share of a larger machine) */
    cpu_set_t allowed;
    int cpus[CPU_SETSIZE], ncpu = 0;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
    if (ncpu == 0) { cpus[0] = 0; ncpu = 1; pin = 0; }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (evb_job){alg, open, t, pin ? cpus[t % ncpu] : -1, keys, nkeys, d,
                            n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads,
                            arena, status, iters, 0};
        pthread_create(&th[t], NULL, evb_worker, &jobs[t]);
    }
    long fails = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        fails += jobs[t].failures;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (failures) *failures = fails;
    free(th);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
