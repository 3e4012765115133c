// chacha_layout.hip — microbenchmark: cost per 64-byte ChaCha20 block of the two lane layouts
// (DESIGN.md §3.3), 16 waves per CU as chacha_batch_kernel runs.
//   quad: one block per quad of lanes, one state column per lane, the diagonal rounds through
//         DPP quad permutes folded into the adds/XORs (the round-4 kernel's chacha_quad)
//   lane: one block per lane, the whole 16-word state in the lane's registers (no cross-lane ops)
// Reports ns per block per CU and cycles per block per SIMD (clock from s_memtime/s_memrealtime).
//
// build: hipcc --offload-arch=gfx950 -O3 -o chacha_layout chacha_layout.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                            \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

constexpr int kCalls = 256;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    constexpr int ctrl = S0 | (S1 << 2) | (S2 << 4) | (S3 << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}
template <int Q>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v, uint32_t o) {
    uint32_t r;
    asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[%c3,%c4,%c5,%c6] row_mask:0xf bank_mask:0xf"
        : "=v"(r) : "v"(v), "v"(o), "i"(Q & 3), "i"((Q >> 2) & 3), "i"((Q >> 4) & 3), "i"((Q >> 6) & 3));
    return r;
}
template <int Q>
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v, uint32_t o) {
    uint32_t r;
    asm("s_nop 1\n\tv_xor_b32_dpp %0, %1, %2 quad_perm:[%c3,%c4,%c5,%c6] row_mask:0xf bank_mask:0xf"
        : "=v"(r) : "v"(v), "v"(o), "i"(Q & 3), "i"((Q >> 2) & 3), "i"((Q >> 4) & 3), "i"((Q >> 6) & 3));
    return r;
}

#define QR(a, b, c, d)               \
    a += b; d ^= a; d = rotl(d, 16); \
    c += d; b ^= c; b = rotl(b, 12); \
    a += b; d ^= a; d = rotl(d, 8);  \
    c += d; b ^= c; b = rotl(b, 7);

__device__ __forceinline__ uint4 quad_block(uint32_t a0, uint32_t b0, uint32_t c0, uint32_t d0, uint32_t w) {
    uint32_t a = a0, b = b0, c = c0, d = d0;
#define QR_DPP(P1, P2, P3)                                         \
    a = dpp_add<P1>(b, a); d = rotl(dpp_xor<P3>(d, a), 16);         \
    c = dpp_add<P2>(c, d); b = rotl(dpp_xor<P1>(b, c), 12);         \
    a += b; d ^= a; d = rotl(d, 8);                                \
    c += d; b ^= c; b = rotl(b, 7);
    constexpr int kL1 = 0x39, kL2 = 0x4E, kL3 = 0x93;
    QR(a, b, c, d)
    QR_DPP(kL1, kL2, kL3)
#pragma unroll 3
    for (int i = 1; i < 10; i++) {
        QR_DPP(kL3, kL2, kL1)
        QR_DPP(kL1, kL2, kL3)
    }
#undef QR_DPP
    b = qperm<3, 0, 1, 2>(b);
    c = qperm<2, 3, 0, 1>(c);
    d = qperm<1, 2, 3, 0>(d);
    a += a0; b += b0; c += c0; d += d0;
    const bool hi2 = (w & 2u) != 0;
    uint32_t sa = hi2 ? a : c, sb = hi2 ? b : d;
    sa = qperm<2, 3, 0, 1>(sa);
    sb = qperm<2, 3, 0, 1>(sb);
    if (hi2) { a = sa; b = sb; } else { c = sa; d = sb; }
    const bool hi1 = (w & 1u) != 0;
    uint32_t sx = hi1 ? a : b, sy = hi1 ? c : d;
    sx = qperm<1, 0, 3, 2>(sx);
    sy = qperm<1, 0, 3, 2>(sy);
    if (hi1) { a = sx; c = sy; } else { b = sx; d = sy; }
    return make_uint4(a, b, c, d);
}

// one block per lane: x[0..15] = constants, key, counter, nonce
__device__ __forceinline__ uint32_t lane_block(const uint32_t k[8], uint32_t ctr, uint32_t n1, uint32_t n2) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = n1, x15 = n2;
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        QR(x0, x4, x8, x12)
        QR(x1, x5, x9, x13)
        QR(x2, x6, x10, x14)
        QR(x3, x7, x11, x15)
        QR(x0, x5, x10, x15)
        QR(x1, x6, x11, x12)
        QR(x2, x7, x8, x13)
        QR(x3, x4, x9, x14)
    }
    x0 += 0x61707865u; x1 += 0x3320646eu; x2 += 0x79622d32u; x3 += 0x6b206574u;
    x4 += k[0]; x5 += k[1]; x6 += k[2]; x7 += k[3]; x8 += k[4]; x9 += k[5]; x10 += k[6]; x11 += k[7];
    x12 += ctr; x14 += n1; x15 += n2;
    return x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15;
}

// two blocks per lane, their quarter-rounds interleaved (8 independent chains instead of 4)
__device__ __forceinline__ uint32_t lane_block2(const uint32_t k[8], uint32_t ctr, uint32_t n1, uint32_t n2) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = 0u, x14 = n1, x15 = n2;
    uint32_t y0 = x0, y1 = x1, y2 = x2, y3 = x3, y4 = x4, y5 = x5, y6 = x6, y7 = x7, y8 = x8, y9 = x9, y10 = x10,
             y11 = x11, y12 = ctr + 1u, y13 = 0u, y14 = n1, y15 = n2;
#pragma unroll 1
    for (int i = 0; i < 10; i++) {
        QR(x0, x4, x8, x12) QR(y0, y4, y8, y12)
        QR(x1, x5, x9, x13) QR(y1, y5, y9, y13)
        QR(x2, x6, x10, x14) QR(y2, y6, y10, y14)
        QR(x3, x7, x11, x15) QR(y3, y7, y11, y15)
        QR(x0, x5, x10, x15) QR(y0, y5, y10, y15)
        QR(x1, x6, x11, x12) QR(y1, y6, y11, y12)
        QR(x2, x7, x8, x13) QR(y2, y7, y8, y13)
        QR(x3, x4, x9, x14) QR(y3, y4, y9, y14)
    }
    return x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15 ^ y0 ^ y1 ^ y2 ^ y3 ^
           y4 ^ y5 ^ y6 ^ y7 ^ y8 ^ y9 ^ y10 ^ y11 ^ y12 ^ y13 ^ y14 ^ y15;
}

template <int MODE>
__global__ __launch_bounds__(1024, 4) void layout_kernel(const uint32_t* keys, uint32_t* out, uint64_t* clk) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (MODE == 0) {
        const uint32_t w = lane & 3u;
        const uint32_t ka = keys[(blockIdx.x + lane) & 255u], kc = keys[(blockIdx.x + lane + 7u) & 255u];
        for (int c = 0; c < kCalls; c++) {
            const uint4 ks = quad_block(0x61707865u + w, ka, kc, w == 0u ? (uint32_t)c : lane, w);
            acc ^= ks.x ^ ks.y ^ ks.z ^ ks.w;
        }
    } else if constexpr (MODE == 2) {
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; i++) k[i] = keys[(blockIdx.x + lane + 3u * i) & 255u];
        for (int c = 0; c < kCalls / 8; c++) acc ^= lane_block2(k, (uint32_t)(2 * c), lane, blockIdx.x);
    } else if constexpr (MODE == 3) {
        // the lane layout's instruction mix (add, xor, rotate) in 8 independent chains, no ChaCha
        // dependence pattern: 960 instructions per 64 blocks as the lane layout
        uint32_t a[8], b[8];
#pragma unroll
        for (int c = 0; c < 8; c++) { a[c] = keys[(lane + c) & 255u]; b[c] = keys[(lane + 9u * c) & 255u]; }
        for (int c = 0; c < kCalls / 4; c++) {
#pragma unroll 4
            for (int r = 0; r < 40; r++) {
#pragma unroll
                for (int q = 0; q < 8; q++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[q]) : "v"(b[q]));
#pragma unroll
                for (int q = 0; q < 8; q++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b[q]) : "v"(a[q]));
#pragma unroll
                for (int q = 0; q < 8; q++) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[q]));
            }
        }
#pragma unroll
        for (int c = 0; c < 8; c++) acc ^= a[c] ^ b[c];
    } else {
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; i++) k[i] = keys[(blockIdx.x + lane + 3u * i) & 255u];
        // a quarter of the calls: each produces 4x the blocks of a quad call
        for (int c = 0; c < kCalls / 4; c++) acc ^= lane_block(k, (uint32_t)c, lane, blockIdx.x);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int MODE>
static int run(const char* name, int blocks, const uint32_t* d_keys, uint32_t* d_out, uint64_t* d_clk, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(layout_kernel<MODE>, dim3(blocks), dim3(1024), 0, 0, d_keys, d_out, d_clk);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(layout_kernel<MODE>, dim3(blocks), dim3(1024), 0, 0, d_keys, d_out, d_clk);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t clk[2];
    CHECK(hipMemcpy(clk, d_clk, sizeof clk, hipMemcpyDeviceToHost));
    const double waves = (double)blocks * 16.0;
    const double nblocks = waves * 16.0 * kCalls;  // 16 blocks per wave per quad call, 64 per lane call (x1/4 calls)
    const double ns_per_block_cu = ms * 1e6 * cus / nblocks;
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 0.0;
    printf("{\"layout\": \"%s\", \"ms\": %.4f, \"blocks\": %.0f, \"ns_per_block_per_cu\": %.4f, \"clock_ghz\": %.3f, "
           "\"cycles_per_block_per_simd\": %.2f}\n",
           name, ms, nblocks, ns_per_block_cu, ghz, ns_per_block_cu * ghz * 4.0);
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 2;
    uint32_t h_keys[256];
    for (int i = 0; i < 256; i++) h_keys[i] = 0x9e3779b9u * (uint32_t)(i + 1);
    uint32_t *d_keys, *d_out;
    uint64_t* d_clk;
    CHECK(hipMalloc(&d_keys, sizeof h_keys));
    CHECK(hipMemcpy(d_keys, h_keys, sizeof h_keys, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_out, (size_t)blocks * 1024 * 4));
    CHECK(hipMalloc(&d_clk, 16));
    printf("# cus=%d blocks=%d calls=%d\n", cus, blocks, kCalls);
    for (int rep = 0; rep < 2; rep++) {
        if (run<0>("quad", blocks, d_keys, d_out, d_clk, cus)) return 1;
        if (run<1>("lane", blocks, d_keys, d_out, d_clk, cus)) return 1;
        if (run<2>("lane2", blocks, d_keys, d_out, d_clk, cus)) return 1;
        if (run<3>("mix_add_xor_rot", blocks, d_keys, d_out, d_clk, cus)) return 1;
    }
    return 0;
}
