// gather_bench.hip — microbenchmark: AES-round-shaped table lookups split between the LDS
// (ds_read_b32, conflict-free 32-copy layout as in aes_gcm.hip's TLook4) and the vector memory
// path (buffer_load_dword from an L1-resident 4 KiB table). NV of every round's 16 lookups go to
// vector memory. Reports ns per launch and lookups per CU-cycle-equivalent, so the split that
// balances the two pipes can be read off. Not part of the engine.
//
// build: hipcc --offload-arch=gfx950 -O3 -o gather_bench gather_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t s) {
    return __builtin_amdgcn_perm(a, b, s);
}

constexpr int kThreads = 1024;

template <int NV>
__global__ __launch_bounds__(kThreads, 4) void gather_kernel(const uint32_t* __restrict__ gtab, uint32_t* out,
                                                             int iters) {
    __shared__ uint2 ttab[2 * 256 * 32];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t i = tid; i < 2u * 256u * 32u; i += kThreads) ttab[i] = make_uint2(i * 0x9E3779B9u, i * 0x85EBCA6Bu);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)gtab, 0, 4096, 0x00020000);
    const uint32_t c = lane & 31u, hi = c >> 4;
    const uint32_t lb = ((c << 3) | (hi << 2)) | (1u << 16) | (((c << 3) | ((hi ^ 1u) << 2)) << 24);
    uint32_t s[4] = {tid * 0x01000193u, tid ^ 0xA5A5A5A5u, blockIdx.x * 0x27D4EB2Fu + tid, ~tid};
    const char* tb = reinterpret_cast<const char*>(ttab);
    for (int it = 0; it < iters; it++) {
        uint32_t a[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            // lookup j: column j & 3, table (row) j >> 2, state word (col + row) & 3, byte row
            const int col = j & 3, row = j >> 2;
            const uint32_t w = s[(col + row) & 3];
            // VMEM lookups: the first NV of the order 0, 4, 8, 12, 1, 5, ... (spread over rows)
            const int rank = (j & 3) * 4 + (j >> 2);
            if (rank < NV) {
                const uint32_t off = (__builtin_amdgcn_ubfe(w, 8 * row, 8) << 2) | ((uint32_t)row << 10);
                a[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
            } else {
                const uint32_t sel = (row & 1 ? 0x0C000003u : 0x0C000000u) | (row & 2 ? 0x00020000u : 0x000C0000u) |
                                     ((4u + (uint32_t)row) << 8);
                a[j] = *reinterpret_cast<const uint32_t*>(
                    __builtin_assume_aligned(tb + perm(w, lb, sel), 4));
            }
        }
#pragma unroll
        for (int col = 0; col < 4; col++)
            s[col] = x3(x3(a[col], a[col + 4], a[col + 8]), a[col + 12], 0x1B1B1B1Bu + (uint32_t)it);
    }
    out[blockIdx.x * kThreads + tid] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

// VALU issue rate: NCH independent v_bitop3 chains per lane, 16 waves per CU (one 1024-lane
// workgroup with the same 128 KiB LDS footprint as the engine, 4 waves per SIMD).
template <int NCH>
__global__ __launch_bounds__(kThreads, 4) void valu_kernel(uint32_t* out, int iters) {
    __shared__ uint32_t pad[32 * 1024];
    const uint32_t tid = threadIdx.x;
    if (tid == 0) pad[0] = 0;
    uint32_t v[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) v[i] = tid * (2u * i + 1u);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int rep = 0; rep < 16; rep++)
#pragma unroll
            for (int i = 0; i < NCH; i++) v[i] = x3(v[i], v[(i + 1) % NCH], v[(i + 2) % NCH]);
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < NCH; i++) r ^= v[i];
    out[blockIdx.x * kThreads + tid] = r ^ pad[tid & 1];
}

template <int NCH>
static int run_valu(uint32_t* d_out, int blocks, int iters, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(valu_kernel<NCH>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(valu_kernel<NCH>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double wave_ops = (double)blocks * (kThreads / 64) * iters * 16.0 * NCH;
    printf("{\"valu_chains\": %d, \"ms\": %.4f, \"wave_valu_per_cu_per_ns\": %.4f}\n", NCH, best,
           wave_ops / cus / (best * 1e6));
    fflush(stdout);
    return 0;
}

template <int NV>
static int run(const uint32_t* d_tab, uint32_t* d_out, int blocks, int iters, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(gather_kernel<NV>, dim3(blocks), dim3(kThreads), 0, 0, d_tab, d_out, iters);  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(gather_kernel<NV>, dim3(blocks), dim3(kThreads), 0, 0, d_tab, d_out, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double lookups = (double)blocks * kThreads * iters * 16.0;
    const double wave_lookups = lookups / 64.0;  // wave-instructions
    // per CU: wave-instructions per ns
    printf("{\"nv\": %d, \"ms\": %.4f, \"wave_lookups_per_cu_per_ns\": %.4f, \"lookups_per_s\": %.4e}\n", NV, best,
           wave_lookups / cus / (best * 1e6), lookups / (best * 1e-3));
    fflush(stdout);
    return 0;
}

// Pure LDS lookup stream with NS independent AES-round states per lane (NS x 16 lookups in flight
// per round): if the rate rises with NS, one state per lane is latency-bound, not LDS-bound.
template <int NS>
__global__ __launch_bounds__(kThreads, 4) void ilp_kernel(uint32_t* out, int iters) {
    __shared__ uint2 ttab[2 * 256 * 32];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t i = tid; i < 2u * 256u * 32u; i += kThreads) ttab[i] = make_uint2(i * 0x9E3779B9u, i * 0x85EBCA6Bu);
    __syncthreads();
    const uint32_t c = lane & 31u, hi = c >> 4;
    const uint32_t lb = ((c << 3) | (hi << 2)) | (1u << 16) | (((c << 3) | ((hi ^ 1u) << 2)) << 24);
    uint32_t s[NS][4];
#pragma unroll
    for (int q = 0; q < NS; q++) {
        s[q][0] = tid * 0x01000193u + q;
        s[q][1] = tid ^ (0xA5A5A5A5u + q);
        s[q][2] = blockIdx.x * 0x27D4EB2Fu + tid + 7 * q;
        s[q][3] = ~tid + q;
    }
    const char* tb = reinterpret_cast<const char*>(ttab);
    for (int it = 0; it < iters; it += NS) {
#pragma unroll
        for (int q = 0; q < NS; q++) {
            uint32_t a[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int col = j & 3, row = j >> 2;
                const uint32_t w = s[q][(col + row) & 3];
                const uint32_t sel = (row & 1 ? 0x0C000003u : 0x0C000000u) | (row & 2 ? 0x00020000u : 0x000C0000u) |
                                     ((4u + (uint32_t)row) << 8);
                a[j] = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(tb + perm(w, lb, sel), 4));
            }
#pragma unroll
            for (int col = 0; col < 4; col++)
                s[q][col] = x3(x3(a[col], a[col + 4], a[col + 8]), a[col + 12], 0x1B1B1B1Bu + (uint32_t)it);
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < NS; q++) r ^= s[q][0] ^ s[q][1] ^ s[q][2] ^ s[q][3];
    out[blockIdx.x * kThreads + tid] = r;
}

template <int NS>
static int run_ilp(uint32_t* d_out, int blocks, int iters, int cus) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(ilp_kernel<NS>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(ilp_kernel<NS>, dim3(blocks), dim3(kThreads), 0, 0, d_out, iters);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double wave_lookups = (double)blocks * (kThreads / 64) * iters * 16.0;  // rounds total = iters
    printf("{\"states_per_lane\": %d, \"ms\": %.4f, \"wave_lookups_per_cu_per_ns\": %.4f}\n", NS, best,
           wave_lookups / cus / (best * 1e6));
    fflush(stdout);
    return 0;
}

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 400;
    int dev = 0, cus = 0;
    CHECK(hipSetDevice(dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 4;
    uint32_t h_tab[1024];
    for (int i = 0; i < 1024; i++) h_tab[i] = (uint32_t)i * 2654435761u;
    uint32_t *d_tab, *d_out;
    CHECK(hipMalloc(&d_tab, sizeof h_tab));
    CHECK(hipMemcpy(d_tab, h_tab, sizeof h_tab, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_out, (size_t)blocks * kThreads * 4));
    printf("# cus=%d blocks=%d iters=%d\n", cus, blocks, iters);
    if (run<0>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (argc > 2 && argv[2][0] == 'i') {  // LDS lookup stream, 1 / 2 / 4 independent states per lane
        if (run_ilp<1>(d_out, blocks, iters, cus) || run_ilp<2>(d_out, blocks, iters, cus) ||
            run_ilp<4>(d_out, blocks, iters, cus))
            return 1;
        return 0;
    }
    if (argc > 2) {  // valu only
        if (run_valu<4>(d_out, blocks, iters, cus)) return 1;
        return run_valu<8>(d_out, blocks, iters, cus);
    }
    if (run<2>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run<4>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run<5>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run<6>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run<8>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run<16>(d_tab, d_out, blocks, iters, cus)) return 1;
    if (run_valu<4>(d_out, blocks, iters, cus)) return 1;
    if (run_valu<8>(d_out, blocks, iters, cus)) return 1;
    return 0;
}
