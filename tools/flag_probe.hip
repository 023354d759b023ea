// flag_probe.hip -- VERDICT r03 #3: what overlapping the select kernel's
// alpha_S = Minv a_R with FTRAN-z's A[:,S] alpha_S inside ONE launch could save
// against the two dependent launches the solver uses (k_select_ftran ->
// k_ftran_zr).  Shapes of C3 at the end of the solve: k = 268 bump positions,
// m = 5000 rows, 67 producer workgroups (4 bump rows each, one wave per row),
// 157 consumer row tiles of 32 rows (8 waves: a half-wave per 32-position
// chunk, chunk sums in LDS, as k_ftran_zr).  Every variant computes the same
// z = A[:,S] (Minv a_R) bits.
//   pair     -- producer kernel, then consumer kernel (the library's seam);
//   fused    -- one launch: producers store alpha_S, then count themselves in
//               an agent-scope counter (release); consumer tiles prefetch their
//               first AS chunk, spin on the counter (acquire), then finish;
//   fused_uc -- as fused with alpha_S and the counter in uncached memory (no
//               L2 writeback / invalidate: stores and polling loads meet in HBM);
//   chunk_uc -- uncached, one counter per 32-position chunk (8 producer
//               workgroups each): a half-wave waits only for its own chunk.
// Each variant: 2000 back-to-back iterations on one stream, events around them.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/flag_probe.hip -o /tmp/flag_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr int K = 268, LDM = 272, M = 5000, CH = 32, ROWS = 32, ZW = 8;
constexpr int NRW = (K + 3) / 4;           // producer workgroups
constexpr int NRT = (M + ROWS - 1) / ROWS;  // consumer row tiles
constexpr int NCH = (K + CH - 1) / CH;      // chunks
constexpr unsigned long long SPIN_TICKS = 1000000ull;  // 10 ms of the 100 MHz clock

struct Buf {
    const double* Minv;  // K x LDM row-major
    const double* aR;    // K
    const double* AS;    // M x K column-major (ld M)
    double* alS;         // K (cached or uncached)
    double* z;           // M
    unsigned long long* cnt;  // [1 + NCH] counters
    int* fail;
};

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// one wave per bump row p: alpha_S[p] = Minv[p, :] . aR (lane-strided chain + tree)
template <bool UC>
__device__ void produce(const Buf& b, int wg) {
    const int lane = threadIdx.x & 63, p = wg * 4 + (threadIdx.x >> 6);
    if (p >= K) return;
    double acc = 0.0;
    for (int i = lane; i < K; i += 64) acc = fma(b.Minv[(size_t)p * LDM + i], b.aR[i], acc);
    acc = wave_sum(acc);
    if (lane == 0) {
        if (UC) __hip_atomic_store(&b.alS[p], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else b.alS[p] = acc;
    }
}

__device__ __forceinline__ double ld_al(const Buf& b, int p, bool uc) {
    return uc ? __hip_atomic_load(&b.alS[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : b.alS[p];
}

// row tile t: z_i = sum over chunks (chunk chain over its 32 positions), chunk
// sums added in order; half-wave h of wave w owns chunks 2w + h, + 16, ...
// wait: 0 none, 1 one counter (>= want), 2 the chunk's counter (>= want2)
template <bool UC>
__device__ void consume(const Buf& b, int t, int wait, unsigned long long want, unsigned long long want2) {
    __shared__ double zl[NCH][ROWS];
    __shared__ int s_ok;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
    const int i = t * ROWS + r, ch0 = 2 * w + hh;
    const int ii = i < M ? i : M - 1;
    double a0[CH];
    if (ch0 < NCH) {  // the first chunk's AS values: before any wait
#pragma unroll
        for (int u = 0; u < CH; ++u) a0[u] = b.AS[(size_t)min(ch0 * CH + u, K - 1) * M + ii];
    }
    if (threadIdx.x == 0) s_ok = 1;
    if (wait == 1) {
        if (threadIdx.x == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(b.cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
                    s_ok = 0;
                    atomicOr(b.fail, 1);
                    break;
                }
            }
        }
        __syncthreads();
    } else if (wait == 2 && ch0 < NCH) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(b.cnt + 1 + ch0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want2) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) {
                atomicOr(b.fail, 1);
                break;
            }
        }
    }
    if (ch0 < NCH) {
        double acc = 0.0;
        const int len = min(CH, K - ch0 * CH);
#pragma unroll
        for (int u = 0; u < CH; ++u)
            if (u < len) acc = fma(a0[u], ld_al(b, ch0 * CH + u, UC), acc);
        zl[ch0][r] = acc;
    }
    __syncthreads();
    if (w == 0 && hh == 0 && i < M) {
        double z = 0.0;
        for (int c = 0; c < NCH; ++c) z = z + zl[c][r];
        b.z[i] = z;
    }
}

__global__ void __launch_bounds__(256) k_prod(Buf b) { produce<false>(b, blockIdx.x); }
__global__ void __launch_bounds__(ZW * 64) k_cons(Buf b) { consume<false>(b, blockIdx.x, 0, 0, 0); }

// fused: [NRW producer workgroups (first 256 threads)][NRT consumer tiles]
template <bool UC, int MODE>  // MODE 1 one counter, 2 per-chunk counters
__global__ void __launch_bounds__(ZW * 64) k_fused(Buf b, unsigned long long it) {
    if ((int)blockIdx.x < NRW) {
        if (threadIdx.x < 256) produce<UC>(b, blockIdx.x);
        __builtin_amdgcn_s_waitcnt(0);  // this wave's stores acknowledged (gfx9: stores count in vmcnt)
        if (MODE == 1) {
            __syncthreads();
            if (threadIdx.x == 0) {
                if (!UC) __threadfence();  // release alpha_S (L2 writeback across XCDs)
                __hip_atomic_fetch_add(b.cnt, 1ull, UC ? __ATOMIC_RELAXED : __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            // the workgroup's 4 rows lie in chunk blockIdx / 8: count once the stores are done
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_fetch_add(b.cnt + 1 + (blockIdx.x * 4) / CH, 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    const int t = blockIdx.x - NRW;
    // producers per chunk: 8 workgroups (4 rows each) except the last chunk
    const int ch0 = 2 * ((threadIdx.x & 511) >> 6) + ((threadIdx.x & 63) >> 5);
    const int pc = ch0 < NCH ? (min(K, (ch0 + 1) * CH) - ch0 * CH + 3) / 4 : 0;
    consume<UC>(b, t, MODE, (it + 1) * NRW, (it + 1) * (unsigned long long)pc);
}

int main() {
    std::vector<double> hM((size_t)K * LDM), haR(K), hAS((size_t)M * K);
    srand(7);
    for (auto& v : hM) v = rand() / (double)RAND_MAX - 0.5;
    for (auto& v : haR) v = rand() / (double)RAND_MAX;
    for (auto& v : hAS) v = rand() / (double)RAND_MAX;
    double *dM, *daR, *dAS, *dal, *dal_uc, *dz;
    unsigned long long *dcnt, *dcnt_uc;
    int* dfail;
    CK(hipMalloc(&dM, hM.size() * 8));
    CK(hipMalloc(&daR, K * 8));
    CK(hipMalloc(&dAS, hAS.size() * 8));
    CK(hipMalloc(&dal, K * 8));
    CK(hipMalloc(&dz, M * 8));
    CK(hipMalloc(&dcnt, (1 + NCH) * 8));
    CK(hipMalloc(&dfail, 4));
    CK(hipExtMallocWithFlags((void**)&dal_uc, K * 8, hipDeviceMallocUncached));
    CK(hipExtMallocWithFlags((void**)&dcnt_uc, (1 + NCH) * 8, hipDeviceMallocUncached));
    CK(hipMemcpy(dM, hM.data(), hM.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(daR, haR.data(), K * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dAS, hAS.data(), hAS.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dfail, 0, 4));
    Buf b{dM, daR, dAS, dal, dz, dcnt, dfail};
    Buf bu{dM, daR, dAS, dal_uc, dz, dcnt_uc, dfail};
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> ref(M), got(M);
    const int L = 2000;
    auto run = [&](const char* name, int v) {
        CK(hipMemsetAsync(dcnt, 0, (1 + NCH) * 8, st));
        CK(hipMemsetAsync(dcnt_uc, 0, (1 + NCH) * 8, st));
        CK(hipMemsetAsync(dz, 0, M * 8, st));
        CK(hipStreamSynchronize(st));
        for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up; counters keep counting
            const unsigned long long base = (unsigned long long)rep * L;
            CK(hipEventRecord(e0, st));
            for (int it = 0; it < L; ++it) {
                if (v == 0) {
                    hipLaunchKernelGGL(k_prod, dim3(NRW), dim3(256), 0, st, b);
                    hipLaunchKernelGGL(k_cons, dim3(NRT), dim3(ZW * 64), 0, st, b);
                } else if (v == 1) {
                    hipLaunchKernelGGL((k_fused<false, 1>), dim3(NRW + NRT), dim3(ZW * 64), 0, st, b, base + it);
                } else if (v == 2) {
                    hipLaunchKernelGGL((k_fused<true, 1>), dim3(NRW + NRT), dim3(ZW * 64), 0, st, bu, base + it);
                } else {
                    hipLaunchKernelGGL((k_fused<true, 2>), dim3(NRW + NRT), dim3(ZW * 64), 0, st, bu, base + it);
                }
            }
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
        }
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        int fail = 0;
        CK(hipMemcpy(&fail, dfail, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(got.data(), dz, M * 8, hipMemcpyDeviceToHost));
        if (v == 0) ref = got;
        int bad = 0;
        for (int i = 0; i < M; ++i) bad += got[i] != ref[i];
        printf("%-9s %7.2f us per iteration  (z mismatches vs pair: %d, spin timeouts: %d)\n", name, 1e3 * ms / L,
               bad, fail);
        fflush(stdout);
        return fail == 0;
    };
    if (!run("pair", 0)) return 2;
    // the single kernels alone (same stream, back to back)
    for (int which = 0; which < 2; ++which) {
        CK(hipEventRecord(e0, st));
        for (int it = 0; it < L; ++it) {
            if (which == 0) hipLaunchKernelGGL(k_prod, dim3(NRW), dim3(256), 0, st, b);
            else hipLaunchKernelGGL(k_cons, dim3(NRT), dim3(ZW * 64), 0, st, b);
        }
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-9s %7.2f us per launch\n", which ? "consumer" : "producer", 1e3 * ms / L);
    }
    if (!run("fused", 1)) return 3;
    if (!run("fused_uc", 2)) return 4;
    if (!run("chunk_uc", 3)) return 5;
    return 0;
}
