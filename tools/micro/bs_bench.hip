// bs_bench.hip — throughput of the bitsliced AES-256-CTR pass (tools/experimental/bs_aes.hpp) alone:
// 16 waves per CU, every wave running NPASS passes back to back. Reports ns per pass per wave and
// VALU instructions per pass from the code object (counted separately). Not part of the engine.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../experimental/bs_aes.hpp"

__global__ __launch_bounds__(1024, 4) void bs_kernel(const uint32_t* rec, uint4* out, int npass) {
    const uint32_t lane = threadIdx.x & 63u;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int it = 0; it < npass; it++) {
        uint4 ks[8];
        neb::bs_ctr_pass(lane * 0x9E3779B9u ^ blockIdx.x, (uint32_t)it, 2u + (uint32_t)it, 0u, rec, lane, ks);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            acc.x ^= ks[j].x; acc.y ^= ks[j].y; acc.z ^= ks[j].z; acc.w ^= ks[j].w;
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int npass = argc > 1 ? atoi(argv[1]) : 20;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t h_rec[neb::kKeyRecDwords];
    for (uint32_t i = 0; i < neb::kKeyRecDwords; i++) h_rec[i] = i * 2654435761u;
    uint32_t* d_rec;
    uint4* d_out;
    hipMalloc(&d_rec, sizeof h_rec);
    hipMemcpy(d_rec, h_rec, sizeof h_rec, hipMemcpyHostToDevice);
    hipMalloc(&d_out, (size_t)cus * 1024 * 16);
    hipLaunchKernelGGL(bs_kernel, dim3(cus), dim3(1024), 0, 0, d_rec, d_out, npass);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(bs_kernel, dim3(cus), dim3(1024), 0, 0, d_rec, d_out, npass);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("{\"npass\": %d, \"ms\": %.4f, \"us_per_pass_per_wave\": %.3f, \"blocks_per_s\": %.4e}\n", npass, best,
           best * 1e3 / npass, (double)cus * 16 * 16 * 32 * npass / (best * 1e-3));
    return 0;
}
