// b128_bench.hip — ds_read_b128 lookups in two conflict-free patterns (16 waves per CU):
//  ROW:  the 16 lanes of a lane group read 16 entries of ONE 256-byte row (the nibble GHASH table)
//  SCAT: the 16 lanes read 16 different rows, lane f in bank group f (the byte-window table)
// Each lane runs CH independent chains of dependent lookups (the next address comes from the data),
// so CH = 1 measures latency and CH = 8 throughput. Not part of the engine.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kThreads = 1024;

template <int SCAT, int CH>
__global__ __launch_bounds__(kThreads, 4) void k(uint32_t* out, int iters) {
    __shared__ uint4 tab[256 * 16];  // 64 KiB: entry e of row r at r*16 + e (16-B units)
    const uint32_t tid = threadIdx.x, f = tid & 15u;
    for (uint32_t i = tid; i < 256u * 16u; i += kThreads) {
        const uint32_t h = i * 2654435761u;
        tab[i] = make_uint4(h, h ^ 0x9E3779B9u, h * 7u, h >> 3);
    }
    __syncthreads();
    uint32_t x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = tid * (2u * c + 1u);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t addr;
            if (SCAT) addr = ((x[c] & 255u) << 8) | (((f + (uint32_t)it) & 15u) << 4);  // row = data, bank group = lane
            else addr = ((((uint32_t)it + (uint32_t)c) & 255u) << 8) | ((x[c] & 15u) << 4);   // row = step, entry = data
            const uint4 e = *reinterpret_cast<const uint4*>(__builtin_assume_aligned(reinterpret_cast<const char*>(tab) + addr, 16));
            x[c] = e.x ^ e.y ^ e.z ^ e.w ^ x[c];
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) r ^= x[c];
    out[blockIdx.x * kThreads + tid] = r;
}

template <int SCAT, int CH>
static void run(uint32_t* d_out, int blocks, int iters, int cus) {
    hipLaunchKernelGGL((k<SCAT, CH>), dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((k<SCAT, CH>), dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double wave_reads = (double)blocks * (kThreads / 64) * iters * CH;
    printf("{\"pattern\": \"%s\", \"chains\": %d, \"ms\": %.4f, \"wave_b128_per_cu_per_ns\": %.4f}\n", SCAT ? "scattered rows" : "one row",
           CH, best, wave_reads / cus / (best * 1e6));
    fflush(stdout);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* d_out;
    hipMalloc(&d_out, (size_t)cus * 4 * kThreads * 4);
    const int iters = 2000;
    run<0, 1>(d_out, cus * 4, iters, cus);
    run<1, 1>(d_out, cus * 4, iters, cus);
    run<0, 8>(d_out, cus * 4, iters, cus);
    run<1, 8>(d_out, cus * 4, iters, cus);
    return 0;
}
