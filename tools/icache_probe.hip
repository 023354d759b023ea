// Instruction-fetch probe (r05): does straight-line code that a launch runs
// once pay for its instruction fetch?  One wave runs a block of NB independent
// fp64 adds twice (the block is the body of a two-trip loop the compiler may
// not unroll), stamping s_memrealtime (100 MHz) before, between and after: the
// first trip runs cold code, the second the same code from the instruction
// cache.  A second kernel of the same shape but a different body is launched
// in between to evict the first one's lines.  Build:
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

int main() {
    unsigned long long* out;
    double* sink;
    hipMalloc(&out, 64);
    hipMalloc(&sink, 64 * sizeof(double));
    unsigned long long h[2];
    for (int it = 0; it < 5; ++it) {
        probe<1><<<1, 64>>>(out, sink, 2);
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        printf("salt 1: first trip %.2f us, second trip %.2f us (4096 fp64 adds, ~8 KB of code)\n", h[0] / 100.0,
               h[1] / 100.0);
        probe<2><<<1, 64>>>(out, sink, 2);
        hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        printf("salt 2: first trip %.2f us, second trip %.2f us\n", h[0] / 100.0, h[1] / 100.0);
    }
    return 0;
}
