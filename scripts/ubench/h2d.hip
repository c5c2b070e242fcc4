// H2D copy-rate microbenchmark: one pinned 1 GB host buffer to HBM by (A) one hipMemcpyAsync,
// (B) segments on one stream, (C) segments spread over 2 / 4 streams, (D) a kernel reading the
// pinned buffer through its device pointer (zero-copy) with 16-B loads.  GB/s = 1e9 bytes / s,
// best and median of 5.  Run once as is and once with HSA_ENABLE_SDMA=0 (blit-kernel copies).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = i + j < n16 ? src[i + j] : uint4{};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i + j < n16) dst[i + j] = v[j];
    }
}

int main(int argc, char **argv) {
    const size_t N = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 30);
    void *h = nullptr, *d = nullptr, *hd = nullptr;
    CK(hipHostMalloc(&h, N, hipHostMallocDefault));
    memset(h, 0x41, N);
    CK(hipMalloc(&d, N));
    CK(hipHostGetDevicePointer(&hd, h, 0));
    hipStream_t st[4];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1, ej[4];
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &e : ej) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto run = [&](const char *name, auto &&body) {
        std::vector<float> ms;
        for (int r = 0; r < 6; ++r) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            body();
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);  // the first run warms up
        }
        std::sort(ms.begin(), ms.end());
        printf("%-34s best %6.2f GB/s  median %6.2f GB/s  (%.3f ms)\n", name, N / (ms[0] * 1e6),
               N / (ms[ms.size() / 2] * 1e6), ms[ms.size() / 2]);
        fflush(stdout);
    };
    // the other streams join st[0] at the start and st[0] waits for them at the end
    auto fan = [&](int ns, size_t seg) {
        CK(hipEventRecord(ej[0], st[0]));
        for (int s = 1; s < ns; ++s) CK(hipStreamWaitEvent(st[s], ej[0], 0));
        size_t i = 0;
        for (size_t off = 0; off < N; off += seg, ++i) {
            const size_t len = std::min(seg, N - off);
            CK(hipMemcpyAsync((char *)d + off, (char *)h + off, len, hipMemcpyHostToDevice, st[i % ns]));
        }
        for (int s = 1; s < ns; ++s) {
            CK(hipEventRecord(ej[s], st[s]));
            CK(hipStreamWaitEvent(st[0], ej[s], 0));
        }
    };
    run("A one copy", [&] { CK(hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, st[0])); });
    for (size_t seg : {4ull << 20, 32ull << 20, 128ull << 20}) {
        char nm[64];
        snprintf(nm, sizeof nm, "B %3zu MB segments, 1 stream", seg >> 20);
        run(nm, [&] { fan(1, seg); });
    }
    for (int ns : {2, 4}) {
        char nm[64];
        snprintf(nm, sizeof nm, "C 32 MB segments, %d streams", ns);
        run(nm, [&] { fan(ns, 32ull << 20); });
    }
    for (int g : {256, 1024, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "D zero-copy kernel, %d WGs", g);
        run(nm, [&] { k_pull<<<g, 256, 0, st[0]>>>((const uint4 *)hd, (uint4 *)d, N / 16); });
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    return 0;
}
