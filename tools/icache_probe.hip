// Instruction-fetch probe (r05): does straight-line code that a launch runs
// once pay for its instruction fetch?  One wave runs a block of NB independent
// fp64 adds twice (the block is the body of a two-trip loop the compiler may
// not unroll), stamping s_memrealtime (100 MHz) before, between and after: the
// first trip runs cold code, the second the same code from the instruction
// cache.  Before each probe launch a read of 64 MiB (the code out of L2, still
// in the MALL) or 1 GiB (out of the MALL too) evicts it further (r05zi: the
// cold trip costs ~0.1-0.3 us per 8 KB in every case).  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o /tmp/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP4(x) x x x x
#define REP16(x) REP4(x) REP4(x) REP4(x) REP4(x)
#define REP64(x) REP16(x) REP16(x) REP16(x) REP16(x)
#define REP256(x) REP64(x) REP64(x) REP64(x) REP64(x)

template <int SALT>
__global__ void probe(unsigned long long* out, double* sink, int trips) {
    double a0 = threadIdx.x * 1.0 + SALT, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long t[3];
    t[0] = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < trips; ++r) {
        // 4 x 256 = 1024 independent v_add_f64 (8 bytes each: ~8 KB of code)
        REP256(asm volatile("v_add_f64 %0, %0, 1.0\n v_add_f64 %1, %1, 1.0\n v_add_f64 %2, %2, 1.0\n v_add_f64 %3, %3, 1.0"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));)
        t[r + 1 < 3 ? r + 1 : 2] = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (threadIdx.x == 0) {
        out[0] = t[1] - t[0];
        out[1] = t[2] - t[1];
    }
    sink[threadIdx.x] = a0 + a1 + a2 + a3;
}

// reads n doubles (grid-stride): with 64 MB the probe's code is out of every
// XCD's L2 (4 MB each) but still in the 256 MB MALL; with 1 GB out of both
__global__ void evict(const double* buf, size_t n, double* sink) {
    double a = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += buf[i];
    if (a == 12345.678) sink[0] = a;
}

int main() {
    unsigned long long* out;
    double* sink;
    double* buf;
    hipMalloc(&out, 64);
    hipMalloc(&sink, 64 * sizeof(double));
    const size_t big = (size_t)1 << 27;  // 1 GiB of doubles
    hipMalloc(&buf, big * sizeof(double));
    hipMemset(buf, 0, big * sizeof(double));
    unsigned long long h[2];
    const size_t modes[3] = {0, (size_t)8 << 20, big};  // none, 64 MiB, 1 GiB
    const char* names[3] = {"hot (no eviction)", "after 64 MiB read (L2 evicted)", "after 1 GiB read (MALL evicted)"};
    for (int md = 0; md < 3; ++md) {
        double f = 0.0, s2 = 0.0;
        const int R = 8;
        for (int it = 0; it < R + 1; ++it) {
            if (modes[md]) evict<<<2048, 256>>>(buf, modes[md], sink);
            probe<1><<<1, 64>>>(out, sink, 2);
            hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
            if (it > 0) {  // (the first: the code object's first load)
                f += h[0] / 100.0;
                s2 += h[1] / 100.0;
            }
        }
        printf("%-34s first trip %.2f us, second trip %.2f us (~8 KB of straight-line code)\n", names[md], f / R,
               s2 / R);
    }
    return 0;
}
