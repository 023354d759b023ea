// kernarg_probe.hip -- what the by-value Dev argument costs a latency kernel.
// The hot kernels take Dev (~800 B) by value; their prologues load its fields
// from the kernarg segment in several dependent scalar rounds before the
// control-block load can issue.  Three variants of one kernel shape (read ~30
// Dev fields, then the control block, then one dependent load, write one
// value), 256 workgroups x 256 threads, 4000 back-to-back launches:
//   val  -- Dev by value (as the library);
//   ptr  -- const Dev* to a device copy (fields through the scalar cache / L2);
//   min  -- only the three pointers it needs by value (lower bound).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../easylp_amd/csrc kernarg_probe.hip -o /tmp/kernarg_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "elp_internal.h"

using elp::Dev;
using elp::DevCtl;

__device__ __forceinline__ double body(const Dev& d, int lane) {
    // fields the ratio kernel's prologue touches (pointers and sizes)
    const DevCtl* c = d.ctl;
    const int st = c->status;
    double acc = 0.0;
    const int64_t i = lane % (d.m > 0 ? d.m : 1);
    acc += d.y[i] + d.xr[i] + d.rlo[i] + d.rhi[i];
    acc += (double)d.cover[i] + (double)d.Rl[i] + (double)d.ypos[i] + (double)d.rpos[i];
    acc += d.alS[i % (d.ldm > 0 ? d.ldm : 1)] + d.alU[i] + d.vvec[i % 64] + d.vrow[i % 64];
    acc += d.Minv[i] + d.MinvT[i] + d.AS[i] + d.blockmin[i % 64];
    acc += (double)d.tile_w + (double)d.ntiles + (double)d.n + (double)d.N + (double)d.col0;
    if (st == 12345) acc += d.cost[i] + d.lb[i] + d.ub[i] + d.xval[i];
    return acc;
}

__global__ void __launch_bounds__(256) k_val(Dev d, double* out) {
    const double a = body(d, threadIdx.x);
    if (threadIdx.x == 0) out[blockIdx.x] = a;
}
__global__ void __launch_bounds__(256) k_ptr(const Dev* __restrict__ dp, double* out) {
    const Dev& d = *dp;
    const double a = body(d, threadIdx.x);
    if (threadIdx.x == 0) out[blockIdx.x] = a;
}
__global__ void __launch_bounds__(256) k_min(const DevCtl* __restrict__ c, const double* __restrict__ y,
                                             double* out) {
    const int st = c->status;
    double a = y[threadIdx.x] + (double)st;
    if (threadIdx.x == 0) out[blockIdx.x] = a;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const int m = 4096, G = 256, L = 4000;
    Dev d{};
    d.m = m;
    d.n = 50000;
    d.N = 50000;
    d.ldm = 512;
    d.tile_w = 128;
    d.ntiles = 391;
    double* pool = nullptr;
    CK(hipMalloc(&pool, sizeof(double) * (size_t)m * 32));
    CK(hipMemset(pool, 0, sizeof(double) * (size_t)m * 32));
    double** dbl[] = {&d.y, &d.xr, &d.rlo, &d.rhi, &d.alS, &d.alU, &d.vvec, &d.vrow, &d.Minv, &d.MinvT,
                      &d.AS, &d.blockmin, &d.cost, &d.lb, &d.ub, &d.xval};
    for (int t = 0; t < 16; ++t) *dbl[t] = pool + (size_t)t * m;
    int32_t** ints[] = {&d.cover, &d.Rl, &d.ypos, &d.rpos};
    for (int t = 0; t < 4; ++t) *ints[t] = reinterpret_cast<int32_t*>(pool + (size_t)(16 + t) * m);
    DevCtl* ctl = nullptr;
    CK(hipMalloc(&ctl, sizeof(DevCtl)));
    CK(hipMemset(ctl, 0, sizeof(DevCtl)));
    d.ctl = ctl;
    Dev* dd = nullptr;
    CK(hipMalloc(&dd, sizeof(Dev)));
    CK(hipMemcpy(dd, &d, sizeof(Dev), hipMemcpyHostToDevice));
    double* out = nullptr;
    CK(hipMalloc(&out, sizeof(double) * G));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("sizeof(Dev) = %zu B\n", sizeof(Dev));
    for (int rep = 0; rep < 3; ++rep) {
        for (int v = 0; v < 3; ++v) {
            for (int w = 0; w < 200; ++w) {  // warm
                if (v == 0) k_val<<<G, 256, 0, st>>>(d, out);
                else if (v == 1) k_ptr<<<G, 256, 0, st>>>(dd, out);
                else k_min<<<G, 256, 0, st>>>(ctl, d.y, out);
            }
            CK(hipEventRecord(e0, st));
            for (int l = 0; l < L; ++l) {
                if (v == 0) k_val<<<G, 256, 0, st>>>(d, out);
                else if (v == 1) k_ptr<<<G, 256, 0, st>>>(dd, out);
                else k_min<<<G, 256, 0, st>>>(ctl, d.y, out);
            }
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("rep %d %s: %.3f us per launch (back-to-back)\n", rep, v == 0 ? "val" : v == 1 ? "ptr" : "min",
                   1e3 * ms / L);
        }
    }
    return 0;
}
