// Dispatch / latency floor of a launch on gfx950 (diagnostic): how the time of
// a small latency-bound kernel grows with its workgroup count.  Each kernel
// runs `depth` dependent global loads per thread (index from the last value)
// over a buffer that sits in L2 / the Infinity Cache, then one store.  Reports
// the average per launch of 200 back-to-back launches (hipEvents around them:
// duration + the gap between dependent dispatches) for G workgroups of 256
// threads.  Build: hipcc --offload-arch=gfx950 -O3 -o dispatch_probe dispatch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void __launch_bounds__(256) k_chain(const int* __restrict__ nxt, int* __restrict__ out, int depth,
                                              int mask) {
    int i = (blockIdx.x * 256 + threadIdx.x) & mask;
    for (int t = 0; t < depth; ++t) i = nxt[i];
    out[blockIdx.x * 256 + threadIdx.x] = i;
}

int main() {
    const int N = 1 << 22;  // 16 MB of indices
    std::vector<int> h(N);
    for (int i = 0; i < N; ++i) h[i] = (int)((i * 2654435761u + 12345u) & (N - 1));
    int *nxt = nullptr, *out = nullptr;
    CK(hipMalloc(&nxt, N * sizeof(int)));
    CK(hipMalloc(&out, 4096 * 256 * sizeof(int)));
    CK(hipMemcpy(nxt, h.data(), N * sizeof(int), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grids[] = {1, 16, 64, 128, 256, 384, 512, 768, 1024, 2048};
    const int depths[] = {0, 1, 3};
    std::printf("# average us per launch (200 back-to-back launches of 256-thread workgroups)\n");
    std::printf("%8s", "wgs");
    for (int dd : depths) std::printf("  depth%d", dd);
    std::printf("\n");
    for (int g : grids) {
        std::printf("%8d", g);
        for (int dd : depths) {
            for (int w = 0; w < 20; ++w) k_chain<<<g, 256>>>(nxt, out, dd, N - 1);
            CK(hipEventRecord(e0));
            for (int r = 0; r < 200; ++r) k_chain<<<g, 256>>>(nxt, out, dd, N - 1);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("  %6.2f", 1e3 * ms / 200);
        }
        std::printf("\n");
    }
    return 0;
}
