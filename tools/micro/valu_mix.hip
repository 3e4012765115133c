// valu_mix.hip — microbenchmark: issue rate of the VALU instruction kinds the ChaCha20-Poly1305
// kernel is made of, 16 waves per CU (4 per SIMD, as chacha_batch_kernel runs),
// 8 independent chains per lane so that latency is hidden and the rate is the issue rate.
//   add32:   v_add_u32
//   rot:     v_alignbit_b32 (the ChaCha rotates)
//   mad64:   v_mad_u64_u32 (the Poly1305 limb products, 32 x 32 + 64 -> 64)
//   shr64:   v_lshrrev_b64 (the Poly1305 carries)
// (each through inline asm, so the compiler neither folds a chain nor picks another instruction)
//   dpp:     v_mov_b32 with a DPP quad_perm (the quarter-round diagonals)
//   perm, bitop3, lshl_or, xor, add_dpp+nop: candidates for the rotates and the folded DPP adds
// Reports wave-instructions per CU per ns and, with the clock the kernel measured itself
// (s_memtime cycles over s_memrealtime at 100 MHz), cycles per wave-instruction per SIMD.
//
// build: hipcc --offload-arch=gfx950 -O3 -o valu_mix valu_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kIters = 2000;
constexpr int kChains = 8;
constexpr int kPerIter = 16;  // instructions per chain per iteration

template <int OP>
__global__ __launch_bounds__(1024, 4) void mix_kernel(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t a[kChains], b[kChains];
    uint64_t q[kChains];
#pragma unroll
    for (int c = 0; c < kChains; c++) {
        a[c] = seed ^ (threadIdx.x * 2654435761u) ^ c;
        b[c] = a[c] * 7u + 3u;
        q[c] = ((uint64_t)a[c] << 32) | b[c];
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int k = 0; k < kPerIter; k++) {
#pragma unroll
            for (int c = 0; c < kChains; c++) {
                // inline asm: one instruction each, so the compiler can neither fold a chain of
                // rotates or multiply-adds nor pick another instruction
                if constexpr (OP == 0) {
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
                } else if constexpr (OP == 1) {
                    asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[c]));
                } else if constexpr (OP == 2) {
                    uint64_t carry;
                    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(carry) : "v"(a[c]), "v"(b[c]));
                } else if constexpr (OP == 3) {
                    asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(q[c]));
                } else if constexpr (OP == 4) {
                    a[c] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a[c], 0x39, 0xF, 0xF, false);
                } else if constexpr (OP == 5) {
                    asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
                } else if constexpr (OP == 6) {
                    asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[c]) : "v"(b[c]));
                } else if constexpr (OP == 7) {
                    asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[c]) : "v"(b[c]));
                } else if constexpr (OP == 8) {
                    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(b[c]));
                } else {
                    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
                                 : "+v"(a[c]) : "v"(b[c]));
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < kChains; c++) acc ^= a[c] ^ (uint32_t)q[c] ^ (uint32_t)(q[c] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
static int run(const char* name, int blocks, uint32_t* d_out, uint64_t* d_clk, int ops_per_chain_iter) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(mix_kernel<OP>, dim3(blocks), dim3(1024), 0, 0, d_out, d_clk, 1u);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(mix_kernel<OP>, dim3(blocks), dim3(1024), 0, 0, d_out, d_clk, 2u);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t clk[2];
    CHECK(hipMemcpy(clk, d_clk, sizeof clk, hipMemcpyDeviceToHost));
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const double waves = (double)blocks * 16.0;
    const double winstr = waves * kIters * kPerIter * kChains * ops_per_chain_iter;
    const double per_cu_ns = winstr / cus / (ms * 1e6);
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 0.0;  // memtime cycles per 10 ns
    // cycles per wave-instruction on one SIMD: 4 SIMDs per CU
    const double cyc = ghz > 0 ? ghz * 4.0 / per_cu_ns : 0.0;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"wave_instr_per_cu_per_ns\": %.4f, \"clock_ghz\": %.3f, "
           "\"cycles_per_wave_instr_per_simd\": %.3f}\n",
           name, ms, per_cu_ns, ghz, cyc);
    return 0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 2;  // 2 waves of workgroups, 16 waves per CU at a time
    uint32_t* d_out;
    uint64_t* d_clk;
    CHECK(hipMalloc(&d_out, (size_t)blocks * 1024 * 4));
    CHECK(hipMalloc(&d_clk, 16));
    printf("# cus=%d blocks=%d iters=%d chains=%d\n", cus, blocks, kIters, kChains);
    if (run<0>("add32", blocks, d_out, d_clk, 1)) return 1;
    if (run<1>("rot", blocks, d_out, d_clk, 1)) return 1;
    if (run<2>("mad64", blocks, d_out, d_clk, 1)) return 1;
    if (run<3>("shr64", blocks, d_out, d_clk, 1)) return 1;
    if (run<4>("dpp", blocks, d_out, d_clk, 1)) return 1;
    if (run<5>("perm", blocks, d_out, d_clk, 1)) return 1;
    if (run<6>("bitop3", blocks, d_out, d_clk, 1)) return 1;
    if (run<7>("lshl_or", blocks, d_out, d_clk, 1)) return 1;
    if (run<8>("xor", blocks, d_out, d_clk, 1)) return 1;
    if (run<9>("add_dpp+nop", blocks, d_out, d_clk, 1)) return 1;
    return 0;
}
