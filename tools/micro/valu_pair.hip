// valu_pair.hip — microbenchmark: when does gfx950 issue two VALU instructions in one quad-cycle
// (the SQ_ACTIVE_INST_VALU2 counter)? Run under rocprofv3 --pmc SQ_INSTS_VALU
// SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES; each kernel also reports its own rate.
//   K0  v_add_u32, 8 independent chains per lane                     (valu_mix "add32")
//   K1  v_add_u32, 1 chain per lane (each add needs the previous one)
//   K2  v_add_u32, 2 chains
//   K3  add, rotate alternating, 8 chains
//   K4  4 adds then 4 rotates, 8 chains
//   K5  K0 at 1 wave per SIMD (4 per CU)
//   K6  add, xor, rotate of one quarter-round step on 4 chains (the lane layout's pattern)
//   K7  K6 with the 4 chains' adds and xors interleaved with 4 more chains' (8 chains)
//   K8  v_mov_b32_sdwa writing one byte of its destination (an LDS address byte), 8 chains
//   K9  K8's SDWA moves alternating with v_xor_b32 (VOP2), 8 chains
//   K10 v_perm_b32 (the T-table lookup address the kernels build today), 8 chains
// build: hipcc --offload-arch=gfx950 -O3 -o valu_pair valu_pair.hip
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

constexpr int kIters = 4000;

#define ADD(a, b) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b))
#define XOR(a, b) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b))
#define ROT(a) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a))
#define SDWA(a, b) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(b))
#define PERM(a, b, sel) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "v"(sel))

template <int K>
__global__ __launch_bounds__(1024) void pair_kernel(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    const uint32_t sel = 0x0c020500u ^ (seed & 0x01000000u);  // (a register operand: no literal in VOP3 here)
#pragma unroll
    for (int c = 0; c < 8; c++) {
        a[c] = seed ^ (threadIdx.x * 2654435761u) ^ c;
        b[c] = a[c] * 7u + 3u;
    }
    for (int it = 0; it < kIters; it++) {
        // 24 VALU per iteration in every kernel
        if constexpr (K == 0 || K == 5) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 8; c++) ADD(a[c], b[c]);
        } else if constexpr (K == 1) {
#pragma unroll
            for (int r = 0; r < 24; r++) ADD(a[0], b[0]);
        } else if constexpr (K == 2) {
#pragma unroll
            for (int r = 0; r < 12; r++) {
                ADD(a[0], b[0]);
                ADD(a[1], b[1]);
            }
        } else if constexpr (K == 3) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    ADD(a[c], b[c]);
                    ROT(a[c + 4]);
                }
        } else if constexpr (K == 4) {
#pragma unroll
            for (int r = 0; r < 3; r++) {
#pragma unroll
                for (int c = 0; c < 4; c++) ADD(a[c], b[c]);
#pragma unroll
                for (int c = 4; c < 8; c++) ROT(a[c]);
            }
        } else if constexpr (K == 6) {
#pragma unroll
            for (int r = 0; r < 2; r++) {
#pragma unroll
                for (int c = 0; c < 4; c++) ADD(a[c], b[c]);
#pragma unroll
                for (int c = 0; c < 4; c++) XOR(b[c], a[c]);
#pragma unroll
                for (int c = 0; c < 4; c++) ROT(b[c]);
            }
        } else if constexpr (K == 8) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 8; c++) SDWA(a[c], b[c]);
        } else if constexpr (K == 9) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    SDWA(a[c], b[c]);
                    XOR(b[c + 4], a[c + 4]);
                }
        } else if constexpr (K == 10) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 8; c++) PERM(a[c], b[c], sel);
        } else {
#pragma unroll
            for (int c = 0; c < 4; c++) { ADD(a[c], b[c]); ADD(a[c + 4], b[c + 4]); }
#pragma unroll
            for (int c = 0; c < 4; c++) { XOR(b[c], a[c]); XOR(b[c + 4], a[c + 4]); }
#pragma unroll
            for (int c = 0; c < 8; c++) ROT(b[c]);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) acc ^= a[c] ^ b[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int K>
static int run(int blocks, int threads, uint32_t* d_out, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(pair_kernel<K>, dim3(blocks), dim3(threads), 0, 0, d_out, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(pair_kernel<K>, dim3(blocks), dim3(threads), 0, 0, d_out, 2u);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double winstr = (double)blocks * threads / 64.0 * kIters * 24.0;
    printf("{\"kernel\": %d, \"ms\": %.4f, \"wave_instr_per_cu_per_ns\": %.4f}\n", K, ms, winstr / cus / (ms * 1e6));
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint32_t* d_out;
    CHECK(hipMalloc(&d_out, (size_t)cus * 2 * 1024 * 4));
    const int b = cus * 2;  // 16 waves per CU at a time
    if (run<0>(b, 1024, d_out, cus) || run<1>(b, 1024, d_out, cus) || run<2>(b, 1024, d_out, cus) ||
        run<3>(b, 1024, d_out, cus) || run<4>(b, 1024, d_out, cus) || run<5>(cus, 256, d_out, cus) ||
        run<6>(b, 1024, d_out, cus) || run<7>(b, 1024, d_out, cus) || run<8>(b, 1024, d_out, cus) ||
        run<9>(b, 1024, d_out, cus) || run<10>(b, 1024, d_out, cus))
        return 1;
    return 0;
}
