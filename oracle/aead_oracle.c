/*
 * aead_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, byte-at-a-time restatement of the arithmetic on Nebula's per-packet AEAD data plane.
 * It is the parity CHECKER for the HIP engine in nebula_amd/: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product path never calls it and has no CPU
 * fallback to it.
 *
 * What it restates (reference = /root/reference, slackhq/nebula):
 *   - noiseutil/aesgcm.go:24-49       CipherStateAESGCM.EncryptDanger/DecryptDanger:
 *                                     nonce = 00000000 || BE64(n), exhaustion check, Seal/Open.
 *   - noiseutil/chachapoly.go:23-48   CipherStateChaChaPoly: nonce = 00000000 || LE64(n).
 *   - noiseutil/cipher_state.go:11-18 RejectHeadroom / RejectAfterMessages.
 *   - header/header.go:102-110        header.Encode (the 16-byte AAD).
 *   - header/header.go:143-156        (*H).Parse.
 * The AEAD arithmetic itself is third-party and NOT under /root/reference:
 *   - AES-256-GCM: Go stdlib crypto/aes + crypto/cipher (go.mod:3, Go 1.26), reached through
 *     github.com/flynn/noise v1.1.0 CipherAESGCM (go.mod:10). Restated from the published
 *     algorithms FIPS-197 (AES) and NIST SP 800-38D (GCM, 96-bit IV, 128-bit tag).
 *   - ChaCha20-Poly1305: golang.org/x/crypto v0.54.0 chacha20poly1305 (go.mod:26), restated
 *     from RFC 8439 §2.3-2.8.
 * Pinned by: the reference's only AEAD known-answer vector (noiseutil/fips140_test.go:18-31),
 * the header KAT (header/header_test.go:17-53), RFC 8439 §2.8.2, and cross-checks against
 * OpenSSL libcrypto in tests/ (see tests/golden/make_golden.py).
 *
 * Deliberately simple: S-box AES, bit-serial GF(2^128) multiply, 64-bit-limb Poly1305.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define ORA_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ AES-256 (FIPS-197) */

static const uint8_t SBOX[256] = {
    0x63,0x7c,0x77,0x7b,0xf2,0x6b,0x6f,0xc5,0x30,0x01,0x67,0x2b,0xfe,0xd7,0xab,0x76,
    0xca,0x82,0xc9,0x7d,0xfa,0x59,0x47,0xf0,0xad,0xd4,0xa2,0xaf,0x9c,0xa4,0x72,0xc0,
    0xb7,0xfd,0x93,0x26,0x36,0x3f,0xf7,0xcc,0x34,0xa5,0xe5,0xf1,0x71,0xd8,0x31,0x15,
    0x04,0xc7,0x23,0xc3,0x18,0x96,0x05,0x9a,0x07,0x12,0x80,0xe2,0xeb,0x27,0xb2,0x75,
    0x09,0x83,0x2c,0x1a,0x1b,0x6e,0x5a,0xa0,0x52,0x3b,0xd6,0xb3,0x29,0xe3,0x2f,0x84,
    0x53,0xd1,0x00,0xed,0x20,0xfc,0xb1,0x5b,0x6a,0xcb,0xbe,0x39,0x4a,0x4c,0x58,0xcf,
    0xd0,0xef,0xaa,0xfb,0x43,0x4d,0x33,0x85,0x45,0xf9,0x02,0x7f,0x50,0x3c,0x9f,0xa8,
    0x51,0xa3,0x40,0x8f,0x92,0x9d,0x38,0xf5,0xbc,0xb6,0xda,0x21,0x10,0xff,0xf3,0xd2,
    0xcd,0x0c,0x13,0xec,0x5f,0x97,0x44,0x17,0xc4,0xa7,0x7e,0x3d,0x64,0x5d,0x19,0x73,
    0x60,0x81,0x4f,0xdc,0x22,0x2a,0x90,0x88,0x46,0xee,0xb8,0x14,0xde,0x5e,0x0b,0xdb,
    0xe0,0x32,0x3a,0x0a,0x49,0x06,0x24,0x5c,0xc2,0xd3,0xac,0x62,0x91,0x95,0xe4,0x79,
    0xe7,0xc8,0x37,0x6d,0x8d,0xd5,0x4e,0xa9,0x6c,0x56,0xf4,0xea,0x65,0x7a,0xae,0x08,
    0xba,0x78,0x25,0x2e,0x1c,0xa6,0xb4,0xc6,0xe8,0xdd,0x74,0x1f,0x4b,0xbd,0x8b,0x8a,
    0x70,0x3e,0xb5,0x66,0x48,0x03,0xf6,0x0e,0x61,0x35,0x57,0xb9,0x86,0xc1,0x1d,0x9e,
    0xe1,0xf8,0x98,0x11,0x69,0xd9,0x8e,0x94,0x9b,0x1e,0x87,0xe9,0xce,0x55,0x28,0xdf,
    0x8c,0xa1,0x89,0x0d,0xbf,0xe6,0x42,0x68,0x41,0x99,0x2d,0x0f,0xb0,0x54,0xbb,0x16};

static uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

/* FIPS-197 §5.2 KeyExpansion, Nk = 8, Nr = 14: 15 round keys of 16 bytes. */
static void aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            uint8_t t0 = t[0];
            t[0] = SBOX[t[1]] ^ rcon;
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[t0];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; j++) t[j] = SBOX[t[j]];
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 8) + j] ^ t[j];
    }
}

/* FIPS-197 §5.1 Cipher: SubBytes, ShiftRows, MixColumns, AddRoundKey on a column-major state. */
static void aes256_encrypt(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 14; r++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: row j of column c comes from column (c + j) mod 4 */
        for (int c = 0; c < 4; c++)
            for (int j = 0; j < 4; j++) t[4 * c + j] = SBOX[s[4 * ((c + j) & 3) + j]];
        if (r != 14) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                uint8_t x = a0 ^ a1 ^ a2 ^ a3;
                t[4 * c + 0] = a0 ^ x ^ xtime(a0 ^ a1);
                t[4 * c + 1] = a1 ^ x ^ xtime(a1 ^ a2);
                t[4 * c + 2] = a2 ^ x ^ xtime(a2 ^ a3);
                t[4 * c + 3] = a3 ^ x ^ xtime(a3 ^ a0);
            }
        }
        for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

ORA_API void ora_aes256_expand(const uint8_t key[32], uint8_t rk[240]) { aes256_expand(key, rk); }
ORA_API void ora_aes256_encrypt_block(const uint8_t key[32], const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240];
    aes256_expand(key, rk);
    aes256_encrypt(rk, in, out);
}

/* ------------------------------------------------------------------ GCM (NIST SP 800-38D) */

/* SP 800-38D §6.3 Algorithm 1: X·Y in GF(2^128), bit-reflected ("x^0 is the MSB of byte 0"). */
static void gf128_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t V[16], R[16] = {0};
    memcpy(V, Y, 16);
    for (int i = 0; i < 128; i++) {
        if ((X[i >> 3] >> (7 - (i & 7))) & 1)
            for (int j = 0; j < 16; j++) R[j] ^= V[j];
        int lsb = V[15] & 1;
        for (int j = 15; j > 0; j--) V[j] = (uint8_t)((V[j] >> 1) | (V[j - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xe1;
    }
    memcpy(Z, R, 16);
}

ORA_API void ora_gf128_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) { gf128_mul(X, Y, Z); }

/* GHASH_H over (A zero-padded) || (C zero-padded) || BE64(bitlen A) || BE64(bitlen C): §7.1 steps 5-6. */
static void ghash(const uint8_t H[16], const uint8_t* a, size_t alen, const uint8_t* c, size_t clen,
                  uint8_t Y[16]) {
    memset(Y, 0, 16);
    uint8_t blk[16];
    for (size_t off = 0; off < alen; off += 16) {
        size_t n = alen - off < 16 ? alen - off : 16;
        memset(blk, 0, 16);
        memcpy(blk, a + off, n);
        for (int j = 0; j < 16; j++) Y[j] ^= blk[j];
        gf128_mul(Y, H, Y);
    }
    for (size_t off = 0; off < clen; off += 16) {
        size_t n = clen - off < 16 ? clen - off : 16;
        memset(blk, 0, 16);
        memcpy(blk, c + off, n);
        for (int j = 0; j < 16; j++) Y[j] ^= blk[j];
        gf128_mul(Y, H, Y);
    }
    uint64_t abits = (uint64_t)alen * 8, cbits = (uint64_t)clen * 8;
    for (int j = 0; j < 8; j++) {
        blk[j] = (uint8_t)(abits >> (56 - 8 * j));
        blk[8 + j] = (uint8_t)(cbits >> (56 - 8 * j));
    }
    for (int j = 0; j < 16; j++) Y[j] ^= blk[j];
    gf128_mul(Y, H, Y);
}

static void inc32(uint8_t cb[16]) {
    for (int j = 15; j >= 12; j--)
        if (++cb[j]) break;
}

/* GCTR_K(ICB, X) (§6.5): XOR the keystream of successive inc32 counter blocks into X. */
static void gctr(const uint8_t rk[240], const uint8_t icb[16], const uint8_t* in, size_t len, uint8_t* out) {
    uint8_t cb[16], ks[16];
    memcpy(cb, icb, 16);
    for (size_t off = 0; off < len; off += 16) {
        aes256_encrypt(rk, cb, ks);
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t j = 0; j < n; j++) out[off + j] = in[off + j] ^ ks[j];
        inc32(cb);
    }
}

/* GCM-AE_K(IV, P, A) with a 96-bit IV (§7.1): out = C || T (len(P) + 16 bytes). out may alias pt. */
ORA_API void ora_aes256gcm_seal(const uint8_t key[32], const uint8_t iv[12], const uint8_t* aad, size_t aad_len,
                                const uint8_t* pt, size_t pt_len, uint8_t* out) {
    uint8_t rk[240], H[16] = {0}, J0[16], icb[16], S[16], EJ0[16];
    aes256_expand(key, rk);
    aes256_encrypt(rk, H, H);
    memcpy(J0, iv, 12);
    J0[12] = 0; J0[13] = 0; J0[14] = 0; J0[15] = 1;
    memcpy(icb, J0, 16);
    inc32(icb);
    gctr(rk, icb, pt, pt_len, out);
    ghash(H, aad, aad_len, out, pt_len, S);
    aes256_encrypt(rk, J0, EJ0);
    for (int j = 0; j < 16; j++) out[pt_len + j] = S[j] ^ EJ0[j];
}

/* GCM-AD_K(IV, C, A, T) (§7.2). Returns 0 and writes P, or -1 (auth failure) and zeroes the P
 * region like Go's crypto/cipher GCM Open does. out may alias ct. */
ORA_API int ora_aes256gcm_open(const uint8_t key[32], const uint8_t iv[12], const uint8_t* aad, size_t aad_len,
                               const uint8_t* ct_tag, size_t ct_tag_len, uint8_t* out) {
    if (ct_tag_len < 16) return -1;
    size_t ct_len = ct_tag_len - 16;
    uint8_t rk[240], H[16] = {0}, J0[16], icb[16], S[16], EJ0[16], T[16];
    aes256_expand(key, rk);
    aes256_encrypt(rk, H, H);
    memcpy(J0, iv, 12);
    J0[12] = 0; J0[13] = 0; J0[14] = 0; J0[15] = 1;
    ghash(H, aad, aad_len, ct_tag, ct_len, S);
    aes256_encrypt(rk, J0, EJ0);
    uint8_t diff = 0;
    for (int j = 0; j < 16; j++) {
        T[j] = S[j] ^ EJ0[j];
        diff |= T[j] ^ ct_tag[ct_len + j];
    }
    if (diff) {
        memset(out, 0, ct_len);
        return -1;
    }
    memcpy(icb, J0, 16);
    inc32(icb);
    gctr(rk, icb, ct_tag, ct_len, out);
    return 0;
}

/* H = E_K(0^128) and H^1..H^count (GCM bit order), as the engine's key install precomputes them. */
ORA_API void ora_gcm_hpowers(const uint8_t key[32], int count, uint8_t* out /* count*16 */) {
    uint8_t rk[240], H[16] = {0}, P[16];
    aes256_expand(key, rk);
    aes256_encrypt(rk, H, H);
    memcpy(P, H, 16);
    for (int i = 0; i < count; i++) {
        memcpy(out + 16 * i, P, 16);
        gf128_mul(P, H, P);
    }
}

/* ------------------------------------------------------------------ ChaCha20-Poly1305 (RFC 8439) */

static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static uint32_t ld32le(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static void st32le(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }

#define QR(a, b, c, d)                                   \
    a += b; d ^= a; d = rotl32(d, 16);                   \
    c += d; b ^= c; b = rotl32(b, 12);                   \
    a += b; d ^= a; d = rotl32(d, 8);                    \
    c += d; b ^= c; b = rotl32(b, 7);

/* RFC 8439 §2.3: the ChaCha20 block function. */
static void chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) s[4 + i] = ld32le(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; i++) s[13 + i] = ld32le(nonce + 4 * i);
    memcpy(x, s, sizeof s);
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; i++) st32le(out + 4 * i, x[i] + s[i]);
}

ORA_API void ora_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
    chacha20_block(key, counter, nonce, out);
}

/* RFC 8439 §2.4: ChaCha20 encryption starting at block counter `counter`. */
static void chacha20_xor(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], const uint8_t* in,
                         size_t len, uint8_t* out) {
    uint8_t ks[64];
    for (size_t off = 0; off < len; off += 64) {
        chacha20_block(key, counter++, nonce, ks);
        size_t n = len - off < 64 ? len - off : 64;
        for (size_t j = 0; j < n; j++) out[off + j] = in[off + j] ^ ks[j];
    }
}

/* RFC 8439 §2.5: Poly1305 with 44/44/42-bit limbs over 2^130 - 5. */
typedef struct { uint64_t r[3], h[3], pad[2]; } poly1305;

static void poly_init(poly1305* st, const uint8_t k[32]) {
    uint64_t t0 = (uint64_t)ld32le(k) | (uint64_t)ld32le(k + 4) << 32;
    uint64_t t1 = (uint64_t)ld32le(k + 8) | (uint64_t)ld32le(k + 12) << 32;
    /* clamp: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff */
    t0 &= 0x0ffffffc0fffffffULL;
    t1 &= 0x0ffffffc0ffffffcULL;
    st->r[0] = t0 & 0xfffffffffffULL;
    st->r[1] = ((t0 >> 44) | (t1 << 20)) & 0xfffffffffffULL;
    st->r[2] = (t1 >> 24) & 0x3ffffffffffULL;
    st->h[0] = st->h[1] = st->h[2] = 0;
    st->pad[0] = (uint64_t)ld32le(k + 16) | (uint64_t)ld32le(k + 20) << 32;
    st->pad[1] = (uint64_t)ld32le(k + 24) | (uint64_t)ld32le(k + 28) << 32;
}

/* acc = (acc + n) * r mod p, where n = the 16-byte block with a 2^(8*len) bit appended. */
static void poly_block(poly1305* st, const uint8_t* m, size_t len) {
    uint8_t b[17] = {0};
    memcpy(b, m, len);
    b[len] = 1;
    uint64_t t0 = (uint64_t)ld32le(b) | (uint64_t)ld32le(b + 4) << 32;
    uint64_t t1 = (uint64_t)ld32le(b + 8) | (uint64_t)ld32le(b + 12) << 32;
    uint64_t hibit = b[16];
    uint64_t h0 = st->h[0] + (t0 & 0xfffffffffffULL);
    uint64_t h1 = st->h[1] + (((t0 >> 44) | (t1 << 20)) & 0xfffffffffffULL);
    uint64_t h2 = st->h[2] + (((t1 >> 24) & 0x3ffffffffffULL) | (hibit << 40));
    uint64_t r0 = st->r[0], r1 = st->r[1], r2 = st->r[2];
    uint64_t s1 = r1 * (5 << 2), s2 = r2 * (5 << 2);
    unsigned __int128 d0 = (unsigned __int128)h0 * r0 + (unsigned __int128)h1 * s2 + (unsigned __int128)h2 * s1;
    unsigned __int128 d1 = (unsigned __int128)h0 * r1 + (unsigned __int128)h1 * r0 + (unsigned __int128)h2 * s2;
    unsigned __int128 d2 = (unsigned __int128)h0 * r2 + (unsigned __int128)h1 * r1 + (unsigned __int128)h2 * r0;
    uint64_t c;
    c = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & 0xfffffffffffULL;
    d1 += c; c = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & 0xfffffffffffULL;
    d2 += c; c = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & 0x3ffffffffffULL;
    h0 += c * 5; c = h0 >> 44; h0 &= 0xfffffffffffULL;
    h1 += c;
    st->h[0] = h0; st->h[1] = h1; st->h[2] = h2;
}

static void poly_finish(poly1305* st, uint8_t tag[16]) {
    uint64_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], c;
    c = h1 >> 44; h1 &= 0xfffffffffffULL; h2 += c;
    c = h2 >> 42; h2 &= 0x3ffffffffffULL; h0 += c * 5;
    c = h0 >> 44; h0 &= 0xfffffffffffULL; h1 += c;
    c = h1 >> 44; h1 &= 0xfffffffffffULL; h2 += c;
    c = h2 >> 42; h2 &= 0x3ffffffffffULL; h0 += c * 5;
    c = h0 >> 44; h0 &= 0xfffffffffffULL; h1 += c;
    /* g = h + 5 - 2^130; select h if g < 0 */
    uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= 0xfffffffffffULL;
    uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= 0xfffffffffffULL;
    uint64_t g2 = h2 + c - ((uint64_t)1 << 42);
    uint64_t mask = (g2 >> 63) - 1; /* all ones if g2 >= 0 */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    uint64_t lo = h0 | (h1 << 44), hi = (h1 >> 20) | (h2 << 24);
    unsigned __int128 t = (unsigned __int128)lo + st->pad[0];
    lo = (uint64_t)t;
    hi = hi + st->pad[1] + (uint64_t)(t >> 64);
    for (int i = 0; i < 8; i++) { tag[i] = (uint8_t)(lo >> (8 * i)); tag[8 + i] = (uint8_t)(hi >> (8 * i)); }
}

ORA_API void ora_poly1305(const uint8_t key[32], const uint8_t* m, size_t len, uint8_t tag[16]) {
    poly1305 st;
    poly_init(&st, key);
    for (size_t off = 0; off < len; off += 16) poly_block(&st, m + off, len - off < 16 ? len - off : 16);
    poly_finish(&st, tag);
}

/* RFC 8439 §2.8: mac_data = AAD || pad16 || CT || pad16 || LE64(len AAD) || LE64(len CT). */
static void aead_chacha_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad, size_t aad_len,
                            const uint8_t* ct, size_t ct_len, uint8_t tag[16]) {
    uint8_t otk[64];
    chacha20_block(key, 0, nonce, otk); /* §2.6: one-time key = first 32 bytes of block 0 */
    poly1305 st;
    poly_init(&st, otk);
    uint8_t zero[16] = {0}, lens[16];
    for (size_t off = 0; off < aad_len; off += 16) {
        size_t n = aad_len - off < 16 ? aad_len - off : 16;
        uint8_t b[16] = {0};
        memcpy(b, aad + off, n);
        poly_block(&st, b, 16);
    }
    for (size_t off = 0; off < ct_len; off += 16) {
        size_t n = ct_len - off < 16 ? ct_len - off : 16;
        uint8_t b[16] = {0};
        memcpy(b, ct + off, n);
        poly_block(&st, b, 16);
    }
    (void)zero;
    for (int i = 0; i < 8; i++) {
        lens[i] = (uint8_t)((uint64_t)aad_len >> (8 * i));
        lens[8 + i] = (uint8_t)((uint64_t)ct_len >> (8 * i));
    }
    poly_block(&st, lens, 16);
    poly_finish(&st, tag);
}

ORA_API void ora_chacha20poly1305_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                                       size_t aad_len, const uint8_t* pt, size_t pt_len, uint8_t* out) {
    chacha20_xor(key, 1, nonce, pt, pt_len, out);
    aead_chacha_tag(key, nonce, aad, aad_len, out, pt_len, out + pt_len);
}

ORA_API int ora_chacha20poly1305_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                                      size_t aad_len, const uint8_t* ct_tag, size_t ct_tag_len, uint8_t* out) {
    if (ct_tag_len < 16) return -1;
    size_t ct_len = ct_tag_len - 16;
    uint8_t tag[16], diff = 0;
    aead_chacha_tag(key, nonce, aad, aad_len, ct_tag, ct_len, tag);
    for (int j = 0; j < 16; j++) diff |= tag[j] ^ ct_tag[ct_len + j];
    if (diff) {
        memset(out, 0, ct_len);
        return -1;
    }
    chacha20_xor(key, 1, nonce, ct_tag, ct_len, out);
    return 0;
}

/* ------------------------------------------------------------------ Nebula conventions */

/* header/header.go:102-110 */
ORA_API void ora_header_encode(uint8_t b[16], uint8_t v, uint8_t t, uint8_t st, uint32_t ri, uint64_t c) {
    b[0] = (uint8_t)(v << 4 | (t & 0x0f));
    b[1] = st;
    b[2] = 0;
    b[3] = 0;
    for (int i = 0; i < 4; i++) b[4 + i] = (uint8_t)(ri >> (24 - 8 * i));
    for (int i = 0; i < 8; i++) b[8 + i] = (uint8_t)(c >> (56 - 8 * i));
}

/* header/header.go:143-156. Returns -1 (ErrHeaderTooShort) if len < 16. */
ORA_API int ora_header_parse(const uint8_t* b, size_t len, uint8_t* v, uint8_t* t, uint8_t* st, uint16_t* reserved,
                             uint32_t* ri, uint64_t* c) {
    if (len < 16) return -1;
    *v = (b[0] >> 4) & 0x0f;
    *t = b[0] & 0x0f;
    *st = b[1];
    *reserved = (uint16_t)(b[2] << 8 | b[3]);
    *ri = (uint32_t)b[4] << 24 | (uint32_t)b[5] << 16 | (uint32_t)b[6] << 8 | b[7];
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) x = x << 8 | b[8 + i];
    *c = x;
    return 0;
}

/* noiseutil/aesgcm.go:31-35 (alg 1: BE64) and noiseutil/chachapoly.go:30-34 (alg 2: LE64). */
ORA_API void ora_nonce(int alg, uint64_t n, uint8_t nb[12]) {
    nb[0] = nb[1] = nb[2] = nb[3] = 0;
    for (int i = 0; i < 8; i++) nb[4 + i] = alg == 1 ? (uint8_t)(n >> (56 - 8 * i)) : (uint8_t)(n >> (8 * i));
}

/* noiseutil/cipher_state.go:11-15 */
#define ORA_REJECT_AFTER_MESSAGES (UINT64_MAX - ((uint64_t)1 << 40))

ORA_API uint64_t ora_reject_after_messages(void) { return ORA_REJECT_AFTER_MESSAGES; }

/* EncryptDanger (aesgcm.go:24-37 / chachapoly.go:23-36): appends CT||tag after out[0:out_len].
 * Returns the new length, -2 for ErrMessageCounterExhausted. */
ORA_API long ora_encrypt_danger(int alg, const uint8_t key[32], uint8_t* out, size_t out_len, const uint8_t* ad,
                                size_t ad_len, const uint8_t* pt, size_t pt_len, uint64_t n) {
    if (n >= ORA_REJECT_AFTER_MESSAGES) return -2;
    uint8_t nb[12];
    ora_nonce(alg, n, nb);
    if (alg == 1) ora_aes256gcm_seal(key, nb, ad, ad_len, pt, pt_len, out + out_len);
    else ora_chacha20poly1305_seal(key, nb, ad, ad_len, pt, pt_len, out + out_len);
    return (long)(out_len + pt_len + 16);
}

/* DecryptDanger (aesgcm.go:39-49 / chachapoly.go:38-48). Returns new length or -1 (auth failure). */
ORA_API long ora_decrypt_danger(int alg, const uint8_t key[32], uint8_t* out, size_t out_len, const uint8_t* ad,
                                size_t ad_len, const uint8_t* ct, size_t ct_len, uint64_t n) {
    uint8_t nb[12];
    ora_nonce(alg, n, nb);
    int rc = alg == 1 ? ora_aes256gcm_open(key, nb, ad, ad_len, ct, ct_len, out + out_len)
                      : ora_chacha20poly1305_open(key, nb, ad, ad_len, ct, ct_len, out + out_len);
    if (rc) return -1;
    return (long)(out_len + ct_len - 16);
}

/* ------------------------------------------------------------------ batch form (same layout as the engine) */

/* Mirrors include/nebula_aead.h neb_desc; offsets index one byte arena. */
typedef struct {
    uint64_t src_off, dst_off, aad_off, counter;
    uint32_t len, aad_len, key_id, flags;
} ora_desc;

/* Seal (open=0) or open (open=1) every descriptor against a key table of 32-byte keys.
 * status[i]: 0 ok, 1 auth failure (payload zeroed), 2 counter exhausted. */
ORA_API void ora_batch(int alg, int open, const uint8_t* keys, const ora_desc* d, size_t n, uint8_t* arena,
                       int32_t* status) {
    for (size_t i = 0; i < n; i++) {
        const uint8_t* key = keys + 32 * (size_t)d[i].key_id;
        uint8_t nb[12];
        if (!open && d[i].counter >= ORA_REJECT_AFTER_MESSAGES) { status[i] = 2; continue; }
        ora_nonce(alg, d[i].counter, nb);
        if (!open) {
            if (alg == 1) ora_aes256gcm_seal(key, nb, arena + d[i].aad_off, d[i].aad_len, arena + d[i].src_off, d[i].len, arena + d[i].dst_off);
            else ora_chacha20poly1305_seal(key, nb, arena + d[i].aad_off, d[i].aad_len, arena + d[i].src_off, d[i].len, arena + d[i].dst_off);
            status[i] = 0;
        } else {
            int rc = alg == 1 ? ora_aes256gcm_open(key, nb, arena + d[i].aad_off, d[i].aad_len, arena + d[i].src_off, (size_t)d[i].len + 16, arena + d[i].dst_off)
                              : ora_chacha20poly1305_open(key, nb, arena + d[i].aad_off, d[i].aad_len, arena + d[i].src_off, (size_t)d[i].len + 16, arena + d[i].dst_off);
            status[i] = rc ? 1 : 0;
        }
    }
}
