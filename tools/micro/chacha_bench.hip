// chacha_bench.hip — microbenchmark: ChaCha20 keystream throughput per layout, 16 waves per CU
// (4 per SIMD, as chacha_batch_kernel runs). Not part of the engine.
//   quad1: a quad of lanes per block, one quarter-round column per lane, DPP for the diagonals
//          (the engine's chacha_quad): one 240-op dependent chain per lane per block
//   quad2: the same with two blocks interleaved per quad (two independent chains per lane)
//   lane:  one whole block per lane, the 4 quarter-rounds of a half-round independent (no DPP)
// Reports 64-byte blocks per ns over the GPU.
//
// build: hipcc --offload-arch=gfx950 -O3 -o chacha_bench chacha_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    constexpr int ctrl = S0 | (S1 << 2) | (S2 << 4) | (S3 << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}
#define QR(a, b, c, d)                \
    a += b; d ^= a; d = rotl(d, 16);  \
    c += d; b ^= c; b = rotl(b, 12);  \
    a += b; d ^= a; d = rotl(d, 8);   \
    c += d; b ^= c; b = rotl(b, 7);

__device__ __forceinline__ void quad_rounds(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        QR(a, b, c, d)
        b = qperm<1, 2, 3, 0>(b); c = qperm<2, 3, 0, 1>(c); d = qperm<3, 0, 1, 2>(d);
        QR(a, b, c, d)
        b = qperm<3, 0, 1, 2>(b); c = qperm<2, 3, 0, 1>(c); d = qperm<1, 2, 3, 0>(d);
    }
}
__device__ __forceinline__ void quad_rounds2(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                             uint32_t& f, uint32_t& g, uint32_t& h) {
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        QR(a, b, c, d)
        QR(e, f, g, h)
        b = qperm<1, 2, 3, 0>(b); c = qperm<2, 3, 0, 1>(c); d = qperm<3, 0, 1, 2>(d);
        f = qperm<1, 2, 3, 0>(f); g = qperm<2, 3, 0, 1>(g); h = qperm<3, 0, 1, 2>(h);
        QR(a, b, c, d)
        QR(e, f, g, h)
        b = qperm<3, 0, 1, 2>(b); c = qperm<2, 3, 0, 1>(c); d = qperm<1, 2, 3, 0>(d);
        f = qperm<3, 0, 1, 2>(f); g = qperm<2, 3, 0, 1>(g); h = qperm<1, 2, 3, 0>(h);
    }
}
__device__ __forceinline__ void lane_rounds(uint32_t (&x)[16]) {
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
}

constexpr int kThreads = 256;

template <int MODE>
__global__ __launch_bounds__(kThreads) void bench_kernel(uint32_t* out, int iters) {
    const uint32_t tid = blockIdx.x * kThreads + threadIdx.x;
    uint32_t acc = 0;
    if constexpr (MODE == 0) {
        for (int it = 0; it < iters; it++) {
            uint32_t a = 0x61707865u ^ tid, b = tid * 3u + it, c = tid ^ 0x9E3779B9u, d = it;
            quad_rounds(a, b, c, d);
            acc ^= a ^ b ^ c ^ d;
        }
    } else if constexpr (MODE == 1) {
        for (int it = 0; it < iters; it += 2) {
            uint32_t a = 0x61707865u ^ tid, b = tid * 3u + it, c = tid ^ 0x9E3779B9u, d = it;
            uint32_t e = 0x61707865u ^ tid, f = tid * 5u + it, g = tid ^ 0x7F4A7C15u, h = it + 1;
            quad_rounds2(a, b, c, d, e, f, g, h);
            acc ^= a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
        }
    } else {
        for (int it = 0; it < iters; it += 4) {  // one lane does a whole block = 4 quad-lane shares
            uint32_t x[16];
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] = tid * (2u * k + 1u) + it;
            lane_rounds(x);
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= x[k];
        }
    }
    out[tid] = acc;
}

template <int MODE>
static int run(uint32_t* d_out, int blocks, int iters, const char* name) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(bench_kernel<MODE>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(bench_kernel<MODE>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    // every lane does iters quarter-block shares: a block = 4 shares
    const double blocks64 = (double)blocks * kThreads * iters / 4.0;
    printf("{\"layout\": \"%s\", \"ms\": %.4f, \"blocks_per_ns\": %.3f}\n", name, best, blocks64 / (best * 1e6));
    fflush(stdout);
    return 0;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 4;  // 16 waves per CU
    const int iters = 256;
    uint32_t* d_out;
    CHECK(hipMalloc(&d_out, (size_t)blocks * kThreads * 4));
    if (run<0>(d_out, blocks, iters, "quad1") || run<1>(d_out, blocks, iters, "quad2") ||
        run<2>(d_out, blocks, iters, "lane"))
        return 1;
    return 0;
}
