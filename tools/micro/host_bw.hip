// host_bw.hip — microbenchmark: how fast a kernel reads and writes pinned host memory
// (hipHostMalloc, as neb_host_alloc returns) over PCIe, by access shape. It models the zero-copy
// seal: G lanes per packet, each lane moving V 16-byte vectors per round, so one packet's group
// touches G*16*V contiguous bytes per round (the engine today: G = 4, V = 1, 64 B). Packets sit
// 1344 B apart, 1280 B each. Modes: read (host -> registers), write (registers -> host), copy
// (host -> host through registers, both PCIe directions at once, as the zero-copy seal does).
// Not part of the engine.
//
// build: hipcc --offload-arch=gfx950 -O3 -o host_bw host_bw.hip
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

constexpr int kPkts = 65536, kStride = 1344, kLen = 1280, kThreads = 256;

template <int MODE, int G, int V>
__global__ __launch_bounds__(kThreads) void bw_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                      uint32_t* sink) {
    const uint32_t gt = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t pkt = gt / G, sub = gt % G;
    if (pkt >= (uint32_t)kPkts) return;
    constexpr int seg = G * 16 * V, rounds = kLen / seg;
    const size_t base = (size_t)pkt * (kStride / 16) + sub * V;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int r = 0; r < rounds; r++) {
        const size_t off = base + (size_t)r * (seg / 16);
        uint4 v[V];
#pragma unroll
        for (int i = 0; i < V; i++) {
            if (MODE == 1) v[i] = make_uint4(gt + r, r, i, gt);
            else v[i] = src[off + i];
        }
#pragma unroll
        for (int i = 0; i < V; i++) {
            if (MODE == 0) {
                acc.x ^= v[i].x; acc.y ^= v[i].y; acc.z ^= v[i].z; acc.w ^= v[i].w;
            } else {
                v[i].x ^= 0x5A5A5A5Au;
                dst[off + i] = v[i];
            }
        }
    }
    if (MODE == 0 && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = gt;
}

template <int MODE, int G, int V>
static int run(const char* where, const uint4* src, uint4* dst, uint32_t* sink) {
    const int blocks = (kPkts * G + kThreads - 1) / kThreads;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((bw_kernel<MODE, G, V>), dim3(blocks), dim3(kThreads), 0, 0, src, dst, sink);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((bw_kernel<MODE, G, V>), dim3(blocks), dim3(kThreads), 0, 0, src, dst, sink);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double bytes = (double)kPkts * (kLen / (G * 16 * V)) * G * 16 * V * (MODE == 2 ? 2 : 1);
    static const char* names[] = {"read", "write", "copy"};
    printf("{\"mem\": \"%s\", \"mode\": \"%s\", \"lanes_per_pkt\": %d, \"vec_per_lane\": %d, \"seg_bytes\": %d, "
           "\"ms\": %.4f, \"GBps_total\": %.2f}\n",
           where, names[MODE], G, V, G * 16 * V, best, bytes / (best * 1e6));
    fflush(stdout);
    return 0;
}

template <int MODE>
static int sweep(const char* where, const uint4* src, uint4* dst, uint32_t* sink) {
    if (run<MODE, 4, 1>(where, src, dst, sink)) return 1;   // the engine: 64 B per packet-round
    if (run<MODE, 4, 2>(where, src, dst, sink)) return 1;   // 128 B
    if (run<MODE, 4, 4>(where, src, dst, sink)) return 1;   // 256 B
    if (run<MODE, 8, 1>(where, src, dst, sink)) return 1;   // 128 B by 8 lanes
    if (run<MODE, 16, 1>(where, src, dst, sink)) return 1;  // 256 B by 16 lanes
    if (run<MODE, 16, 4>(where, src, dst, sink)) return 1;  // 1 KiB
    return 0;
}

int main() {
    const size_t bytes = (size_t)kPkts * kStride;
    uint4 *h_src, *h_dst, *d_src, *d_dst;
    uint32_t* sink;
    CHECK(hipHostMalloc((void**)&h_src, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc((void**)&h_dst, bytes, hipHostMallocDefault));
    CHECK(hipMalloc((void**)&d_src, bytes));
    CHECK(hipMalloc((void**)&d_dst, bytes));
    CHECK(hipMalloc((void**)&sink, 64));
    for (size_t i = 0; i < bytes / 16; i++) h_src[i] = make_uint4((uint32_t)i, (uint32_t)(i * 3), 7u, (uint32_t)~i);
    CHECK(hipMemcpy(d_src, h_src, bytes, hipMemcpyHostToDevice));
    if (sweep<0>("host", h_src, h_dst, sink) || sweep<1>("host", h_src, h_dst, sink) ||
        sweep<2>("host", h_src, h_dst, sink))
        return 1;
    if (run<2, 4, 1>("device", d_src, d_dst, sink)) return 1;
    // host -> device and device -> host legs of the split form
    if (run<2, 4, 1>("host_to_dev", h_src, d_dst, sink) || run<2, 4, 4>("host_to_dev", h_src, d_dst, sink)) return 1;
    if (run<2, 4, 1>("dev_to_host", d_src, h_dst, sink) || run<2, 4, 4>("dev_to_host", d_src, h_dst, sink)) return 1;
    return 0;
}
