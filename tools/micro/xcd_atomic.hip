// xcd_atomic.hip — microbenchmark: returning integer atomic adds on counters private to the adding
// workgroup's XCD (index = XCC_ID * nbins + bin), at agent scope (the default atomicAdd: executed
// at the memory side) against workgroup scope (executed in the XCD's own L2, coherent for adders
// of that XCD only). The mixed-key binning's histogram pass (sched_body.hpp) is 1 Mi such adds
// (DESIGN.md §3.2). Checks that every count arrives (sum over bins and XCDs = adds made).
// build: hipcc --offload-arch=gfx950 -O3 -o xcd_atomic xcd_atomic.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHECK(x)                                                            \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

template <int SCOPE>  // 0 agent (atomicAdd), 1 workgroup scope, XCD-private counters
__global__ __launch_bounds__(256) void add_kernel(uint32_t* cnt, uint32_t* out, uint32_t n, uint32_t nbins, uint32_t pad) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t bin = (i * 2654435761u) % nbins;  // a random-looking bin per packet
    const uint32_t x = xcc_id();
    uint32_t* c = cnt + (size_t)x * pad + bin;
    uint32_t r;
    if constexpr (SCOPE == 0)
        r = atomicAdd(c, 1u);
    else
        r = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    out[i] = r;
}

template <int SCOPE>
static int run(const char* name, uint32_t n, uint32_t nbins) {
    const uint32_t pad = (nbins + 31u) & ~31u;  // each XCD's counters on lines of their own
    uint32_t *cnt, *out;
    CHECK(hipMalloc(&cnt, (size_t)8 * pad * 4));
    CHECK(hipMalloc(&out, (size_t)n * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e9f;
    bool ok = true;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipMemset(cnt, 0, (size_t)8 * pad * 4));
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(add_kernel<SCOPE>, dim3((n + 255) / 256), dim3(256), 0, 0, cnt, out, n, nbins, pad);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
        std::vector<uint32_t> h((size_t)8 * pad);
        CHECK(hipMemcpy(h.data(), cnt, h.size() * 4, hipMemcpyDeviceToHost));
        uint64_t sum = 0;
        for (uint32_t v : h) sum += v;
        // every rank an add returned is below its counter's final value and unique per counter
        std::vector<uint32_t> r(n);
        CHECK(hipMemcpy(r.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
        uint64_t rsum = 0;
        for (uint32_t v : r) rsum += v;
        // sum over counters of c*(c-1)/2 must equal the sum of returned ranks
        uint64_t expect = 0;
        for (uint32_t v : h) expect += (uint64_t)v * (v - (v ? 1 : 0)) / 2;
        if (sum != n || rsum != expect) ok = false;
    }
    printf("{\"mode\": \"%s\", \"adds\": %u, \"bins\": %u, \"best_us\": %.2f, \"counts_ok\": %s}\n", name, n, nbins,
           best * 1000.0f, ok ? "true" : "false");
    CHECK(hipFree(cnt));
    CHECK(hipFree(out));
    return ok ? 0 : 2;
}

int main() {
    int rc = 0;
    for (uint32_t nb : {12288u, 4096u * 8u}) {
        rc |= run<0>("agent", 1u << 20, nb);
        rc |= run<1>("workgroup_xcd_private", 1u << 20, nb);
    }
    rc |= run<0>("agent", 1u << 16, 4096);
    rc |= run<1>("workgroup_xcd_private", 1u << 16, 4096);
    return rc;
}
