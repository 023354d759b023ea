// Single-wave latency probe (r05): what one wave pays, in s_memrealtime ticks
// (10 ns), for the operations k_dual_bfrt's one-wave tail is made of -- two
// back-to-back stamps, a chain of dependent ds_bpermute (a __shfl_up scan
// step), a chain of dependent LDS loads, a chain of readlane-indexed steps.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void lat(unsigned long long* out, int* sink, int n) {
    __shared__ int s[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) s[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int v = lane;  // n dependent bpermutes
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int k = 0; k < n; ++k) v = __shfl_up(v, 1) + 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int p = lane;  // n dependent LDS loads
    for (int k = 0; k < n; ++k) p = s[p];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int acc = 0;  // n readlane steps with a loop-variable lane index
    for (int k = 0; k < n; ++k) {
        const int r = __builtin_amdgcn_readlane(p, k & 63);
        if (r == p) acc += k;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t5 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        out[0] = t1 - t0;
        out[1] = t3 - t2;
        out[2] = t4 - t3;
        out[3] = t5 - t4;
    }
    sink[lane] = v + p + acc;
}

int main() {
    unsigned long long* out;
    int* sink;
    hipMalloc(&out, 64);
    hipMalloc(&sink, 64 * sizeof(int));
    unsigned long long h[4], a[4] = {0, 0, 0, 0};
    const int n = 64, R = 20;
    for (int it = 0; it < R + 1; ++it) {
        lat<<<1, 64>>>(out, sink, n);
        hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
        if (it)
            for (int i = 0; i < 4; ++i) a[i] += h[i];
    }
    printf("two stamps back to back %.3f us; per dependent bpermute %.1f ns; per dependent LDS load %.1f ns; "
           "per readlane step %.1f ns\n",
           a[0] / 100.0 / R, a[1] * 10.0 / R / n, a[2] * 10.0 / R / n, a[3] * 10.0 / R / n);
    return 0;
}
