// Which hardware queue each stream lands on (run under rocprofv3 --kernel-trace): streams created in
// the default way, with priorities, and with a full CU mask. One empty kernel per stream, in order;
// the trace's queue_id column per stream_id answers it.
//   queue_map <plain> <prio_hi> <prio_lo> <cumask>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void touch(int* p, int v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[v] = v;
}

int main(int argc, char** argv) {
    const int plain = argc > 1 ? std::atoi(argv[1]) : 6;
    const int hi = argc > 2 ? std::atoi(argv[2]) : 0;
    const int lo = argc > 3 ? std::atoi(argv[3]) : 0;
    const int cum = argc > 4 ? std::atoi(argv[4]) : 0;
    int* d = nullptr;
    if (hipMalloc((void**)&d, 4096) != hipSuccess) return 1;
    int pmin = 0, pmax = 0;
    (void)hipDeviceGetStreamPriorityRange(&pmin, &pmax);
    std::vector<hipStream_t> s;
    std::vector<const char*> kind;
    for (int i = 0; i < plain; i++) {
        hipStream_t x;
        if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) return 2;
        s.push_back(x);
        kind.push_back("plain");
    }
    for (int i = 0; i < hi; i++) {
        hipStream_t x;
        if (hipStreamCreateWithPriority(&x, hipStreamNonBlocking, pmax) != hipSuccess) return 3;
        s.push_back(x);
        kind.push_back("prio_hi");
    }
    for (int i = 0; i < lo; i++) {
        hipStream_t x;
        if (hipStreamCreateWithPriority(&x, hipStreamNonBlocking, pmin) != hipSuccess) return 4;
        s.push_back(x);
        kind.push_back("prio_lo");
    }
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0xffffffffu);
    for (int i = 0; i < cum; i++) {
        hipStream_t x;
        if (hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data()) != hipSuccess) return 5;
        s.push_back(x);
        kind.push_back("cumask");
    }
    for (size_t i = 0; i < s.size(); i++) {
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s[i], d, (int)i);
        if (hipStreamSynchronize(s[i]) != hipSuccess) return 6;
        std::printf("stream %zu %s\n", i, kind[i]);
    }
    std::printf("priority range %d..%d\n", pmin, pmax);
    for (auto x : s) (void)hipStreamDestroy(x);
    (void)hipFree(d);
    return 0;
}
