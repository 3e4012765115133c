/*
 * nebula_aead.h — C ABI of the MI355X (gfx950) AEAD engine for Nebula's per-packet data plane.
 *
 * Plain C: pointers, sizes and integers only; no torch or HIP types cross this boundary
 * (streams are passed as `void*` = hipStream_t). Every entry point returns an int status
 * (NEB_OK = 0, negative = error); nothing throws across the ABI.
 *
 * Reference interfaces replaced (slackhq/nebula, /root/reference):
 *   neb_cipher_create        noise.CipherFunc.Cipher(k [32]byte) — flynn/noise v1.1.0 [ext]; the
 *                            reference's own CipherFunc pattern is noiseutil/fips140.go:31-40,
 *                            selected at pki.go:263-269; wrapped by noiseutil.NewCipherState
 *                            (noiseutil/cipher_state.go:42-54, plugin hook :43-45)
 *   neb_cipher_name          noise.CipherFunc.CipherName() ("AESGCM" / "ChaChaPoly")
 *   neb_encrypt_danger       CipherState.EncryptDanger  noiseutil/cipher_state.go:32,
 *                            noiseutil/aesgcm.go:24-37, noiseutil/chachapoly.go:23-36
 *   neb_decrypt_danger       CipherState.DecryptDanger  noiseutil/cipher_state.go:35,
 *                            noiseutil/aesgcm.go:39-49, noiseutil/chachapoly.go:38-48
 *   neb_overhead             CipherState.Overhead       noiseutil/aesgcm.go:51-56, chachapoly.go:50-55
 *   neb_seal_batch           the per-segment EncryptDanger loop of inside.go:123-146 / :225-236,
 *                            batched at the TX flush point interface.go:465-469,478-487
 *   neb_open_batch           the per-packet ConnectionState.Decrypt → DecryptDanger of
 *                            connection_state.go:99-119 / outside.go:133, batched at the RX flush
 *                            point interface.go:395-400; GMAC-only VerifyRelay
 *                            (connection_state.go:121-148) is an open with len = 0
 *   neb_header_encode/parse  header.Encode header/header.go:102-110, (*H).Parse :143-156
 *   NEB_REJECT_AFTER_MESSAGES noiseutil/cipher_state.go:11-15
 *   neb_window_*             nebula.Bits, the anti-replay window: NewBits bits.go:28-50,
 *                            Check :134-150, Update :152-262, its lost / duplicate / out-of-window
 *                            counters (:23-25, network.packets.{lost,duplicate,out_of_window})
 *   neb_tx_seal_batch        sendInsideMessage (inside.go:154-240) over a batch of TUN reads:
 *                            decodeRead (overlay/tio/tio_gso_linux.go:231-280), SegmentSuperpacket
 *                            (overlay/tio/tun_linux_offload.go:46-60, virtio/segment_linux.go),
 *                            sendInsideEncrypt (inside.go:123-146) into SendBatch slots
 *                            (overlay/batch/tx_batch.go:15-59)
 *   neb_rx_open_batch_host   ConnectionState.Decrypt (connection_state.go:99-119) over a whole
 *                            receive batch (the recvmmsg flush, interface.go:381-413): window
 *                            Check → DecryptDanger → window Update, results identical to the
 *                            per-packet loop in arrival order
 *   neb_queue_*              the flush points themselves (flushSendBatch interface.go:478-487,
 *                            listenOut's flush :395-400) of every routine (interface.go:320-335),
 *                            gathered into shared device batches
 */
#ifndef NEBULA_AEAD_H
#define NEBULA_AEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NEB_API __attribute__((visibility("default")))

/* Cipher identifiers; the names are the Noise CipherName strings hashed into the handshake. */
#define NEB_ALG_AESGCM 1     /* "AESGCM": AES-256-GCM, nonce 00000000 || BE64(n) (aesgcm.go:31-35) */
#define NEB_ALG_CHACHAPOLY 2 /* "ChaChaPoly": ChaCha20-Poly1305, nonce 00000000 || LE64(n) (chachapoly.go:30-34) */

/* Return codes. */
#define NEB_OK 0
#define NEB_ERR_INVALID (-1)      /* bad argument */
#define NEB_ERR_AUTH (-2)         /* Open: "cipher: message authentication failed"; plaintext region zeroed */
#define NEB_ERR_EXHAUSTED (-3)    /* ErrMessageCounterExhausted (cipher_state.go:18) */
#define NEB_ERR_NO_CIPHER (-4)    /* nil receiver on Encrypt: "no cipher state available to encrypt" */
#define NEB_ERR_SHORT_BUFFER (-5) /* out capacity too small for the appended output */
#define NEB_ERR_HIP (-6)          /* HIP runtime failure */
#define NEB_ERR_NO_DEVICE (-7)    /* no gfx950 device / kernels not loadable */
#define NEB_ERR_NO_KEY_SLOT (-8)  /* key table full */

#define NEB_OVERHEAD 16 /* AEAD tag size (Overhead()) */
#define NEB_HEADER_LEN 16
#define NEB_REJECT_HEADROOM (1ULL << 40)
#define NEB_REJECT_AFTER_MESSAGES (UINT64_MAX - NEB_REJECT_HEADROOM)

/* Per-packet status written by the batch calls. */
#define NEB_STATUS_OK 0
#define NEB_STATUS_AUTH_FAILED 1 /* open: tag mismatch, payload destination zeroed */
#define NEB_STATUS_EXHAUSTED 2   /* seal: counter >= NEB_REJECT_AFTER_MESSAGES, nothing written */
#define NEB_STATUS_BAD_KEY 3     /* key_id not installed / wrong algorithm / violates the uniform-key hint */
#define NEB_STATUS_REPLAY 4      /* receive: the replay window refused the counter — ErrAlreadySeen
                                    (connection_state.go:103-105,114-116); nothing decrypted when
                                    refused before decryption */

typedef struct neb_engine neb_engine; /* one per GPU: stream, key table, staging */
typedef struct neb_cipher neb_cipher; /* one installed tunnel key (a CipherState) */

/* One packet of a batch. Offsets index the batch arena (device memory for neb_*_batch, pinned host
 * memory for neb_*_batch_host).
 *   seal: reads aad[aad_len] at aad_off and pt[len] at src_off; writes ct[len] || tag[16] at dst_off.
 *   open: reads aad at aad_off and ct[len] || tag[16] at src_off; writes pt[len] at dst_off.
 * dst_off == src_off is the in-place form used by Nebula (connection_state.go:107). Any other
 * overlap between one packet's regions, or between packets, is undefined. `counter` is the nonce n
 * (= the header's message counter). */
typedef struct neb_desc {
    uint64_t src_off;
    uint64_t dst_off;
    uint64_t aad_off;
    uint64_t counter;
    uint32_t len;
    uint32_t aad_len;
    uint32_t key_id;
    uint32_t flags; /* reserved, 0 */
} neb_desc;

/* ---- engine ------------------------------------------------------------------------------- */

/* Create an engine on HIP device `device` with room for `max_keys` installed keys. */
NEB_API int neb_engine_create(int device, uint32_t max_keys, neb_engine** out);
NEB_API int neb_engine_destroy(neb_engine* e);
/* Device pointer to the engine's key table and the bytes per key record (for diagnostics). */
NEB_API int neb_engine_info(const neb_engine* e, int* device, uint32_t* max_keys, uint32_t* key_record_bytes);
/* stats[0..3]: slots of the per-packet pool (fixed, 4: streams + pinned staging shared by every
 * thread's neb_encrypt_danger / neb_decrypt_danger), per-packet calls, calls that waited for a
 * slot, keys installed (since creation). */
NEB_API int neb_engine_stats(const neb_engine* e, uint64_t stats[4]);
/* Per-packet AES-256-GCM calls that arrived while every launch slot was busy ride together in one
 * launch (round 6): {such combined launches, calls they carried} since creation. */
NEB_API int neb_engine_pkt_combined(const neb_engine* e, uint64_t out[2]);
/* Every entry point restores the calling thread's current HIP device before it returns. Streams
 * passed to the batch calls must stay alive until the work enqueued on them has completed. */
/* Human-readable text of a return code. */
NEB_API const char* neb_strerror(int rc);
/* Detail of the last NEB_ERR_HIP / NEB_ERR_NO_DEVICE on the calling thread (HIP error string), or of
 * the last multi-engine batch call that fenced key slots (it returns NEB_OK; the fenced packets get
 * NEB_STATUS_BAD_KEY — see neb_cipher_create_multi). */
NEB_API const char* neb_last_error(void);
/* The first 16 hex digits of the SHA-256 of the library's sources (nebula_amd/Makefile SRC then
 * HDR, concatenated) it was built from: a test compares it with the sources beside it. */
NEB_API const char* neb_build_id(void);
/* Measurement: the next device batch this thread launches binds its dominant kernel's begin and end
 * to these two HIP events (hipEvent_t, created with timing enabled) instead of recording markers
 * around it — the single-key kernel, the mixed-key chunk kernel or the ChaCha kernel (a small batch:
 * its one kernel). NULL, NULL disarms. */
NEB_API int neb_time_next_kernel(void* start, void* stop);
/* Process-wide knobs for A/B measurements and tests. Each starts from the environment variable named
 * beside it (read once, at the first use of any knob) and can be changed between batches; batches
 * read them with one atomic load (no getenv on the batch path). */
enum {
    NEB_KNOB_HOST_MODE = 0,       /* NEB_HOST_MODE: 0 zero-copy for mapped arenas (default), 1 "dma" staging */
    NEB_KNOB_SUB_BINS_FROM = 1,   /* NEB_SUB_BINS_FROM: mixed-key batches of at least this many packets
                                   * count their bins in sub-bins (default 262144) */
    NEB_KNOB_SINGLE_MAX_GRID = 2, /* NEB_SINGLE_MAX_GRID: cap on the single-key kernel's workgroups (0: none;
                                   * tests use it to force a partial last pass) */
    NEB_KNOB_RX_STRICT = 3,       /* NEB_RXDEV_STRICT: a device receive whose windows need the sequential host
                                   * finish fails with NEB_ERR_INVALID instead (tests: the parallel form ran) */
    NEB_KNOB_TILE_BINS_FROM = 4,  /* NEB_TILE_BINS_FROM: mixed-key batches of at least this many packets bin
                                   * through per-workgroup LDS histograms (sched.hpp: no per-packet global
                                   * atomic); smaller ones through the atomic histogram */
    NEB_KNOB_SMALL_BATCH = 5,     /* NEB_SMALL_BATCH: a mixed-key AES-GCM batch with fewer packets than this
                                   * per resident wave of the chunk kernel (16 per CU) is chunked finer, up to
                                   * NEB_KNOB_FRONT_GROUPS groups per chunk (default 48; 0: never) */
    NEB_KNOB_FRONT_GROUPS = 6,    /* NEB_FRONT_GROUPS: the 16-packet groups per front chunk of the short size
                                   * classes in such a batch at most (default 1; the classes' own: up to 8) */
    NEB_KNOB_COUNT = 7
};
NEB_API int neb_set_knob(int knob, int64_t value);
NEB_API int64_t neb_get_knob(int knob); /* -1 for an unknown knob */
/* The (demangled) name of the kernel the last armed pair was bound to on this thread, or "" when
 * none has been bound yet: what a benchmark's kernel time is the time of. */
NEB_API const char* neb_time_last_kernel(void);

/* ---- key install: noise.CipherFunc.Cipher(k) ----------------------------------------------- */

/* Install a 32-byte key: AES-256 key schedule + H = E_K(0^128) + H^1..H^16 (AESGCM), or the raw
 * ChaCha20 key (ChaChaPoly), computed on the device into the engine's key table. */
NEB_API int neb_cipher_create(neb_engine* e, int alg, const uint8_t key[32], neb_cipher** out);
/* Install n keys at once (keys = n x 32 bytes; out[n]): the tunnel keys a lighthouse or a rekey
 * storm completes in one go (handshake_manager.go:752,877 -> connection_state.go:55-75 per tunnel).
 * One launch of n workgroups and one synchronize instead of n; each key gets the lowest free
 * slot in turn, as n calls of neb_cipher_create would. NEB_ERR_NO_KEY_SLOT (nothing installed)
 * when fewer than n slots are free. */
NEB_API int neb_cipher_create_batch(neb_engine* e, int alg, const uint8_t* keys, uint32_t n, neb_cipher** out);
/* Install ONE tunnel key on every engine of a set (one per GPU; the engines used together by
 * neb_*_batch_host_multi / neb_*_batch_sharded): the same key_id on all of them — the lowest slot
 * free on every engine, reserved on all at once — or on none (NEB_ERR_NO_KEY_SLOT, or the error of
 * the failing engine with the others rolled back). out[k] is the key's cipher on engines[k]; each
 * is destroyed on its own. The installs share one identity that the multi-engine batch calls
 * check (below). A tunnel has exactly one eKey / dKey (connection_state.go:37-49, 55-75). */
NEB_API int neb_cipher_create_multi(neb_engine* const* engines, uint32_t nengines, int alg, const uint8_t key[32],
                                    neb_cipher** out);
/* Waits for the asynchronous batches this engine enqueued that may read the key — the last
 * single-key batch with it on each stream and the last mixed-key batch on each stream — then
 * clears the key record and frees its slot. Other work on the device is not waited for. The caller
 * stops enqueuing batches with the key before destroying it (as Go code stops using a
 * CipherState it drops); a batch enqueued after the destroy gets NEB_STATUS_BAD_KEY for its
 * packets (the kernels check the slot's algorithm tag) or, once the slot is reused, the new key. */
NEB_API int neb_cipher_destroy(neb_cipher* c);
NEB_API uint32_t neb_cipher_key_id(const neb_cipher* c);
NEB_API int neb_cipher_alg(const neb_cipher* c);
NEB_API const char* neb_cipher_name(int alg); /* "AESGCM", "ChaChaPoly", NULL if unknown */

/* ---- per-packet CipherState surface (host buffers; exact Go slice semantics) ---------------- */

/* Overhead(): 16, or 0 when c == NULL. */
NEB_API int neb_overhead(const neb_cipher* c);

/* EncryptDanger(out, ad, plaintext, n, nb): keeps out[0:out_len], appends ct || tag, sets
 * *ret_len = out_len + pt_len + 16. `ad` may alias out[0:out_len] (inside.go:131). `nb` (12 bytes,
 * may be NULL) receives the nonce exactly as the Go code assembles it.
 * Errors: NEB_ERR_NO_CIPHER (c == NULL), NEB_ERR_EXHAUSTED (n >= NEB_REJECT_AFTER_MESSAGES; out
 * untouched), NEB_ERR_SHORT_BUFFER (out_cap < out_len + pt_len + 16). */
NEB_API int neb_encrypt_danger(neb_cipher* c, uint8_t* out, size_t out_len, size_t out_cap, const uint8_t* ad,
                               size_t ad_len, const uint8_t* pt, size_t pt_len, uint64_t n, uint8_t* nb,
                               size_t* ret_len);

/* DecryptDanger(out, ad, ciphertext, n, nb): ciphertext = ct || tag. Keeps out[0:out_len], writes
 * the plaintext after it, *ret_len = out_len + ct_len - 16. In place when out + out_len == ct
 * (connection_state.go:107). On tag mismatch returns NEB_ERR_AUTH, zeroes the would-be plaintext
 * region and touches nothing else (cipher_state_test.go:194-237). c == NULL: returns NEB_OK with
 * *ret_len = 0 (Go returns []byte{}, nil). ct_len < 16 is an auth failure. */
NEB_API int neb_decrypt_danger(neb_cipher* c, uint8_t* out, size_t out_len, size_t out_cap, const uint8_t* ad,
                               size_t ad_len, const uint8_t* ct, size_t ct_len, uint64_t n, uint8_t* nb,
                               size_t* ret_len);

/* ---- batched data plane: device-resident arena ----------------------------------------------- */

/* Key hint for the batch calls: NEB_KEYS_MIXED, or a key_id every descriptor uses (one tunnel's
 * batch) — the engine then keeps that key's round keys in scalar registers and its GHASH tables
 * shared per workgroup. Descriptors whose key_id differs from the hint get NEB_STATUS_BAD_KEY. */
#define NEB_KEYS_MIXED 0xFFFFFFFFu

/* Seal/open n packets. d_desc, d_arena, d_status are device pointers; `stream` is a hipStream_t
 * (NULL = the HIP default stream). Asynchronous: returns after enqueueing. Every descriptor's key must
 * have algorithm `alg`. */
NEB_API int neb_seal_batch(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                           int32_t* d_status, uint32_t key_hint, void* stream);
NEB_API int neb_open_batch(neb_engine* e, int alg, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                           int32_t* d_status, uint32_t key_hint, void* stream);

/* ---- batched data plane: host-resident arena (the TUN / UDP side) ---------------------------- */

/* Same as above but desc/arena/status live in host memory. Synchronous.
 * Every descriptor is first bounds-checked against arena_len, in every mode: an invalid batch
 * returns NEB_ERR_INVALID with the arena and the statuses untouched.
 * - arena pinned and mapped (neb_host_alloc, at any byte address): zero-copy — the kernels load
 *   and store the arena across PCIe directly; desc/status may be pinned or ordinary.
 * - any other arena: the range the descriptors touch is streamed through the device in chunks of
 *   8192 packets, H2D -> kernel -> D2H, rotated over three streams; chunks whose arena ranges
 *   overlap are serialised (each copies its whole range back).
 * Environment, read per call: NEB_HOST_MODE=dma (or NEB_HOST_STAGED=1) stages every arena. */
NEB_API int neb_seal_batch_host(neb_engine* e, int alg, const neb_desc* desc, uint32_t n, uint8_t* arena,
                                size_t arena_len, int32_t* status, uint32_t key_hint);
NEB_API int neb_open_batch_host(neb_engine* e, int alg, const neb_desc* desc, uint32_t n, uint8_t* arena,
                                size_t arena_len, int32_t* status, uint32_t key_hint);

/* ---- several GPUs in one process: contiguous shards, no collective ------------ */
/* Packets are independent, so a batch shards by contiguous packet range over engines (one per GPU,
 * or several on one GPU): shard k takes packets [n*k/m, n*(k+1)/m) of m engines. A batch's keys
 * are engine 0's: install each tunnel key on the set with neb_cipher_create_multi. A packet of
 * shard k whose key_id names a slot where engine k does not hold the same install as engine 0
 * (not installed there, destroyed and reinstalled on one engine, keys installed engine by engine)
 * gets NEB_STATUS_BAD_KEY and is not touched — never sealed or opened with another key. */
/* Host-resident batch (the arena in host memory, pinned or not): one host thread per engine runs
 * neb_seal_batch_host / neb_open_batch_host on its shard; returns when every shard is done, with
 * the first failing shard's return code (the other shards still complete). A staged (not pinned)
 * arena whose shards' byte spans overlap runs the shards one after another. */
NEB_API int neb_seal_batch_host_multi(neb_engine* const* engines, uint32_t nengines, int alg, const neb_desc* desc,
                                      uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status,
                                      uint32_t key_hint);
NEB_API int neb_open_batch_host_multi(neb_engine* const* engines, uint32_t nengines, int alg, const neb_desc* desc,
                                      uint32_t n, uint8_t* arena, size_t arena_len, int32_t* status,
                                      uint32_t key_hint);
/* Device-resident shards: shard k's descriptors, arena and statuses live on engine k's device
 * (each shard's descriptors index its own arena); each is enqueued on its stream (NULL: the
 * device's default stream) and the call returns once every shard is done. */
typedef struct neb_shard {
    neb_engine* e;
    const neb_desc* d_desc;
    uint32_t n;
    uint8_t* d_arena;
    int32_t* d_status;
    void* stream;
} neb_shard;
NEB_API int neb_seal_batch_sharded(int alg, const neb_shard* shards, uint32_t nshards, uint32_t key_hint);
NEB_API int neb_open_batch_sharded(int alg, const neb_shard* shards, uint32_t nshards, uint32_t key_hint);

/* Pinned host memory (hipHostMalloc) for arenas that back the reference's batch.Arena
 * (overlay/batch/coalesce_core.go:142-169) so the batch path needs no bounce copy. */
NEB_API int neb_host_alloc(size_t bytes, void** out);
NEB_API int neb_host_free(void* p);

/* ---- replay window + batched receive ---------------------------------------------------------- */
typedef struct neb_window neb_window; /* one per tunnel (ConnectionState.window, ReplayWindow = 8192) */
/* NewBits(length): length must be a power of two (NEB_ERR_INVALID otherwise; Go panics). */
NEB_API int neb_window_create(uint64_t length, neb_window** out);
NEB_API int neb_window_destroy(neb_window* w);
/* Check(i) / Update(i): 1 = accepted, 0 = refused, < 0 = error. Each call is atomic (the window
 * carries its own lock, ConnectionState.decryptLock). */
NEB_API int neb_window_check(neb_window* w, uint64_t counter);
NEB_API int neb_window_update(neb_window* w, uint64_t counter);
/* current counter and {lost, duplicate, out_of_window} counts since creation / the last reset. */
NEB_API int neb_window_state(const neb_window* w, uint64_t* current, int64_t counters[3]);
NEB_API int neb_window_slot(const neb_window* w, uint64_t slot); /* bit of slot (slot mod length) */
NEB_API int neb_window_reset_counters(neb_window* w);
/* Receive a batch in arrival order: for every packet, windows[desc.key_id] (NULL or key_id >=
 * nwindows → NEB_STATUS_BAD_KEY) is checked, the packet opened in place (host arena, as
 * neb_open_batch_host) and the window updated — statuses OK / AUTH_FAILED / BAD_KEY / REPLAY,
 * window contents and counters identical to calling Decrypt packet by packet. All packets that
 * pass go to the GPU as one batch; a packet refused by its window is not decrypted. */
NEB_API int neb_rx_open_batch_host(neb_engine* e, int alg, neb_window* const* windows, uint32_t nwindows,
                                   const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len,
                                   int32_t* status, uint32_t key_hint);
/* Replay windows in device memory, for receive batches that stay on the device (neb_rx_open_batch).
 * A set holds `count` windows of one power-of-two length, all absent at creation. load copies a
 * host window's state into slot idx (NULL: the slot becomes absent); store copies slot idx back
 * into a host window of the same length (NEB_ERR_INVALID for an absent slot). Synchronous. */
typedef struct neb_dwindows neb_dwindows;
NEB_API int neb_dwindows_create(neb_engine* e, uint32_t count, uint64_t length, neb_dwindows** out);
NEB_API int neb_dwindows_destroy(neb_dwindows* d);
NEB_API int neb_dwindows_load(neb_dwindows* d, uint32_t idx, const neb_window* w);
NEB_API int neb_dwindows_store(neb_dwindows* d, uint32_t idx, neb_window* w);
/* Fault injection for tests: the polls a device receive's scan may spend waiting for an earlier
 * workgroup before the batch fails with NEB_ERR_HIP (default 2^20, about 0.1 s; 0 fails every scan
 * that has to wait). A failed batch moves no window. */
NEB_API int neb_dwindows_set_spin_limit(neb_dwindows* d, uint32_t limit);
/* neb_rx_open_batch_host over a device-resident batch (device descriptors, arena and statuses),
 * with the windows of `d` (slot desc.key_id; absent or out of range → NEB_STATUS_BAD_KEY): the
 * same statuses, arena bytes, window contents and counters as Decrypt packet by packet. Runs on
 * `stream` and returns when the batch is done (it reads back which windows need the exact
 * sequential finish: those where a tag failed, or counters within 2^62 of wrapping). */
NEB_API int neb_rx_open_batch(neb_engine* e, int alg, neb_dwindows* d, const neb_desc* d_desc, uint32_t n,
                              uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream);
/* ---- receive from the wire: readOutsidePackets' gate in front of Decrypt / VerifyRelay ---------- */
/* One received UDP datagram (or GRO segment) of a receive batch, as readOutsidePackets gets it
 * (outside.go:30): the wire packet header(16) || ct || tag(16) at off of the arena, len bytes, and
 * the tunnel (window / key slot) the caller's hostmap lookup resolved from the header's remote
 * index (outside.go:94-100), NEB_KEYS_MIXED when it found none. */
typedef struct neb_rx_packet {
    uint64_t off;
    uint32_t len;
    uint32_t key_id;
} neb_rx_packet;
#define NEB_STATUS_NOT_MESSAGE 7 /* a valid header of an unencrypted type (handshake, recv error,
                                    outside.go:83-89): left to the control plane, untouched */
/* Or-ed into neb_rx_packet.len by the caller for a datagram that readOutsidePackets' double-
 * encryption check refuses (outside.go:66-74: not relayed, and the UDP source address is inside the
 * node's own VPN networks, f.myVpnNetworksTable). The batch does not carry source addresses, so the
 * caller makes that lookup; the gate then drops the packet as the reference does, right after
 * IsValidSubType and before the handshake hand-off: NEB_STATUS_INVALID, nothing touched. */
#define NEB_RX_OWN_SOURCE 0x80000000u
/* Per packet, readOutsidePackets up to the decrypt, then Decrypt or VerifyRelay: h.Parse (len < 16:
 * NEB_STATUS_INVALID, header.go:143-146); version 1 and IsValidSubType (header.go:192-205), else
 * NEB_STATUS_INVALID (outside.go:49-64); Handshake / RecvError types -> NEB_STATUS_NOT_MESSAGE; no
 * tunnel -> NEB_STATUS_BAD_KEY (outside.go:100-106); len < 16 + 16 -> NEB_STATUS_INVALID
 * (outside.go:108-114); the nonce is the header's counter (bytes 8:16, big-endian). Message/Relay
 * packets are verified GMAC-only over packet[:len-16] (VerifyRelay, connection_state.go:121-148),
 * every other type is opened in place with the header as AAD (Decrypt, connection_state.go:99-119),
 * both through the replay window of their tunnel: statuses, arena bytes and windows as
 * neb_rx_open_batch_host / neb_rx_open_batch give for the descriptors the gate builds. Packets the
 * gate refuses are not touched. The host form checks every packet against arena_len first. */
NEB_API int neb_rx_open_wire_batch_host(neb_engine* e, int alg, neb_window* const* windows, uint32_t nwindows,
                                        const neb_rx_packet* pk, uint32_t n, uint8_t* arena, size_t arena_len,
                                        int32_t* status, uint32_t key_hint);
NEB_API int neb_rx_open_wire_batch(neb_engine* e, int alg, neb_dwindows* d, const neb_rx_packet* d_pk, uint32_t n,
                                   uint8_t* d_arena, int32_t* d_status, uint32_t key_hint, void* stream);
/* ---- transmit: TUN reads (IP packets, TSO/USO superpackets) -> sealed wire packets ------------ */
/* virtio_net_hdr values (linux/virtio_net.h), as the TUN hands them over (overlay/tio/virtio/header_linux.go) */
#define NEB_VNET_F_NEEDS_CSUM 1
#define NEB_VNET_F_RSC_INFO 4
#define NEB_GSO_NONE 0
#define NEB_GSO_TCPV4 1
#define NEB_GSO_TCPV6 4
#define NEB_GSO_UDP_L4 5
#define NEB_GSO_ECN 0x80
/* Per-packet status of a TX batch (besides NEB_STATUS_OK / NEB_STATUS_BAD_KEY = the tunnel has no
 * key, `if ci.eKey == nil { return }`, inside.go:155-158). */
#define NEB_STATUS_INVALID 5  /* virtio / IP header rejected (decodeRead, CheckValid, CorrectHdrLen,
                                 SegmentTCP/UDP, FinishChecksum errors): dropped, no counter used */
#define NEB_STATUS_NO_SPACE 6 /* the output arena or the wire array is full: dropped */
/* One TUN read: an IP packet at in_off of the input arena with its virtio_net_hdr, bound for a tunnel. */
typedef struct neb_tx_packet {
    uint64_t in_off;
    uint32_t len;
    uint32_t tunnel;     /* index into the tunnel array */
    uint8_t vnet_flags;  /* virtio_net_hdr.flags */
    uint8_t gso_type;    /* virtio_net_hdr.gso_type (the ECN qualifier allowed) */
    uint16_t hdr_len;    /* virtio_net_hdr.hdr_len (re-derived from the TCP header, CorrectHdrLen) */
    uint16_t gso_size;
    uint16_t csum_start;
    uint16_t csum_offset;
    uint16_t reserved;
} neb_tx_packet;
/* The sending side of one tunnel (ConnectionState + HostInfo fields the TX path reads). */
typedef struct neb_tx_tunnel {
    uint64_t message_counter; /* ConnectionState.messageCounter: the last counter used; the batch
                                 advances it by one per segment, as inside.go:127 does */
    uint32_t key_id;          /* the eKey's key_id (neb_cipher_key_id); NEB_KEYS_MIXED = no eKey */
    uint32_t remote_index;    /* hostinfo.remoteIndexId, written into every header */
} neb_tx_tunnel;
/* One wire packet: header(16) || ct || tag(16) at out_off (16-byte aligned) of the output arena. */
typedef struct neb_tx_wire {
    uint64_t out_off;
    uint64_t counter;
    uint32_t len;     /* 16 + segment + 16 */
    uint32_t packet;  /* index of the neb_tx_packet it came from */
    uint32_t segment; /* segment index within that packet */
    uint32_t reserved;
} neb_tx_wire;
/* sendInsideMessage (inside.go:154-240) for a whole batch of TUN reads: every packet is validated
 * and segmented exactly as decodeRead + SegmentSuperpacket do (TSO: per-segment seq, CWR/FIN/PSH,
 * IPv4 ID and lengths, IPv4 and TCP checksums; USO: lengths and UDP checksum; plain packets with
 * NEEDS_CSUM get FinishChecksum), each segment takes the next counter of its tunnel in batch order,
 * gets header.Encode(Message, remote_index, counter) and is sealed into its output slot (the seal
 * reads the payload straight from d_in, which must stay valid until the stream has run the batch;
 * only the patched L3/L4 headers are written into the slot first): wires[i] describes the
 * i-th segment of the batch (packet order, then segment order), wire_status[i] is its seal status
 * (NEB_STATUS_EXHAUSTED = dropped, inside.go:137-145, its counter still used). The segment count is
 * written to *d_nwires. Device pointers; asynchronous on `stream`. tunnels[].message_counter is
 * advanced on the device. */
NEB_API int neb_tx_seal_batch(neb_engine* e, int alg, neb_tx_tunnel* d_tunnels, uint32_t ntunnels,
                              const neb_tx_packet* d_packets, uint32_t npackets, const uint8_t* d_in,
                              uint8_t* d_out, size_t out_cap, neb_tx_wire* d_wires, int32_t* d_wire_status,
                              uint32_t max_wires, uint32_t* d_nwires, int32_t* d_packet_status, uint32_t key_hint,
                              void* stream);
/* The same over host memory (synchronous): the input span is uploaded, the outputs downloaded. */
NEB_API int neb_tx_seal_batch_host(neb_engine* e, int alg, neb_tx_tunnel* tunnels, uint32_t ntunnels,
                                   const neb_tx_packet* packets, uint32_t npackets, const uint8_t* in, size_t in_len,
                                   uint8_t* out, size_t out_cap, neb_tx_wire* wires, int32_t* wire_status,
                                   uint32_t max_wires, uint32_t* nwires, int32_t* packet_status, uint32_t key_hint);
/* ---- submission queue: many threads' small flushes -> device-sized batches -------------------- */
/* Nebula seals <= 128 packets per TX flush (overlay/batch/tx_batch.go:5, flushSendBatch
 * interface.go:465-487) and opens <= listen.batch = 64 per RX flush (main.go:181, listenOut
 * interface.go:381-413), from `routines` goroutines at once (interface.go:320-335). A queue
 * gathers those flushes into one device batch: each submission's packets are copied into pinned
 * staging, sealed or opened with the other submissions' by one zero-copy kernel launch, and copied
 * back. A batch goes to the device when it holds max_packets, when the next submission would not
 * fit its staging, on neb_queue_flush, or max_delay_us after its first submission. */
typedef struct neb_queue neb_queue;
typedef struct neb_queue_config {
    uint32_t max_packets;  /* packets per device batch (0: 16384) */
    uint32_t max_delay_us; /* a non-empty batch waits at most this long for more (0: 100 us) */
    uint64_t arena_bytes;  /* pinned staging per batch (0: max_packets x 1536) */
    uint32_t depth;        /* staging batches in rotation, 2..16 (0: 3) */
    uint32_t reserved;     /* 0 */
} neb_queue_config;
/* A queue for one algorithm and direction (open = 0: seal, 1: open). cfg may be NULL (defaults). */
NEB_API int neb_queue_create(neb_engine* e, int alg, int open, const neb_queue_config* cfg, neb_queue** out);
/* Sends out what is queued, waits for it, and frees the queue (no submission may be in progress). */
NEB_API int neb_queue_destroy(neb_queue* q);
/* Seal or open n packets of the caller's host arena (any memory) through the queue, blocking until
 * they are done: the arena bytes and statuses are those of neb_seal_batch_host / neb_open_batch_host
 * on the same descriptors. Thread-safe, meant to be called by many threads at once. Every
 * descriptor is checked against arena_len first (NEB_ERR_INVALID: nothing touched). A submission
 * larger than one batch goes through in pieces. An arena from neb_host_alloc (pinned, mapped) is
 * not copied: only its descriptors are staged and the kernels work on its bytes in place
 * (zero-copy), so it must stay allocated until the call returns; any other memory is copied
 * into the queue's staging and back. */
NEB_API int neb_queue_submit(neb_queue* q, const neb_desc* desc, uint32_t n, uint8_t* arena, size_t arena_len,
                             int32_t* status);
/* Send the batch being filled to the device now, without waiting for its deadline. */
NEB_API int neb_queue_flush(neb_queue* q);
/* stats[0..3]: device batches launched, packets, submissions, staged bytes (since creation). */
NEB_API int neb_queue_stats(neb_queue* q, uint64_t stats[4]);
/* Where a submission's time goes, in nanoseconds summed since creation: per device batch ns[0] fill
 * (first submission -> sealed), ns[1] drain (sealed -> launched: the last copy-ins), ns[2] device
 * (launched -> done: launch, kernel, completion); per submission ns[3] copy-in, ns[4] wait (copy-in
 * done -> its batch done), ns[5] copy-out. Divide by neb_queue_stats' batches / submissions. */
NEB_API int neb_queue_phases(neb_queue* q, uint64_t ns[6]);

/* ---- header (the AAD) --------------------------------------------------------------------- */

NEB_API void neb_header_encode(uint8_t b[16], uint8_t version, uint8_t type, uint8_t subtype, uint32_t remote_index,
                               uint64_t counter);
/* Returns NEB_ERR_INVALID when len < 16 (ErrHeaderTooShort). */
NEB_API int neb_header_parse(const uint8_t* b, size_t len, uint8_t* version, uint8_t* type, uint8_t* subtype,
                             uint16_t* reserved, uint32_t* remote_index, uint64_t* counter);

#ifdef __cplusplus
}
#endif
#endif /* NEBULA_AEAD_H */
