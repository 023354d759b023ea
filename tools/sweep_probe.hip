// sweep_probe.hip -- standalone probe of the pricing sweep's geometry (not part
// of the solver).  Streams a tile-major AR of NY rows x N columns (the k_price
// layout: [N/128 tiles][cap rows][128 columns]) with an fma per element, under
// several launch geometries, and reports us per launch (HIP events around 200
// back-to-back launches).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sweep_probe tools/sweep_probe.hip && /tmp/sweep_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int TC = 128;

// S waves per 128-column tile, wave w takes rows p = w (mod S), UNR rows in flight
template <int S, int UNR>
__global__ void __launch_bounds__(64 * S) k_tile(const double* __restrict__ AR, const double* __restrict__ yy,
                                                int ny, int cap, double* __restrict__ out) {
    __shared__ double part[S][TC];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double* col = AR + (size_t)blockIdx.x * cap * TC + 2 * lane;
    double a0 = 0.0, a1 = 0.0;
    int p = w;
    for (; p + S * (UNR - 1) < ny; p += S * UNR) {
        dbl2 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = *reinterpret_cast<const dbl2*>(col + (size_t)(p + S * u) * TC);
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const double y = yy[p + S * u];
            a0 = fma(v[u].x, y, a0);
            a1 = fma(v[u].y, y, a1);
        }
    }
    for (; p < ny; p += S) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(col + (size_t)p * TC);
        a0 = fma(v.x, yy[p], a0);
        a1 = fma(v.y, yy[p], a1);
    }
    part[w][2 * lane] = a0;
    part[w][2 * lane + 1] = a1;
    __syncthreads();
    if (threadIdx.x < TC) {
        double t = 0.0;
        for (int i = 0; i < S; ++i) t += part[i][threadIdx.x];
        out[(size_t)blockIdx.x * TC + threadIdx.x] = t;
    }
}

// R row blocks per tile as separate workgroups (S waves each): grid = tiles * R,
// each workgroup a contiguous slice of the tile's rows; partials to global
template <int S, int UNR>
__global__ void __launch_bounds__(64 * S) k_split(const double* __restrict__ AR, const double* __restrict__ yy,
                                                 int ny, int cap, int R, double* __restrict__ out) {
    __shared__ double part[S][TC];
    const int tile = blockIdx.x / R, rb = blockIdx.x % R;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int L = (ny + R - 1) / R, r0 = rb * L, r1 = min(ny, r0 + L);
    const double* col = AR + (size_t)tile * cap * TC + 2 * lane;
    double a0 = 0.0, a1 = 0.0;
    int p = r0 + w;
    for (; p + S * (UNR - 1) < r1; p += S * UNR) {
        dbl2 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = *reinterpret_cast<const dbl2*>(col + (size_t)(p + S * u) * TC);
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const double y = yy[p + S * u];
            a0 = fma(v[u].x, y, a0);
            a1 = fma(v[u].y, y, a1);
        }
    }
    for (; p < r1; p += S) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(col + (size_t)p * TC);
        a0 = fma(v.x, yy[p], a0);
        a1 = fma(v.y, yy[p], a1);
    }
    part[w][2 * lane] = a0;
    part[w][2 * lane + 1] = a1;
    __syncthreads();
    if (threadIdx.x < TC) {
        double t = 0.0;
        for (int i = 0; i < S; ++i) t += part[i][threadIdx.x];
        out[((size_t)tile * R + rb) * TC + threadIdx.x] = t;
    }
}

// one wave per column strip of 128/G*... columns: the G lane groups take the
// row classes p = g (mod G) (the tile kernel's S waves folded into one wave),
// W such waves per workgroup (independent strips).  Strip width = 128 / (G/... )
// = 2 * 64 / G columns; dispatch granularity = W waves.
template <int G, int UNR, int W>
__global__ void __launch_bounds__(64 * W) k_strip(const double* __restrict__ AR, const double* __restrict__ yy,
                                                 int ny, int cap, int nstrips, double* __restrict__ out) {
    constexpr int LPR = 64 / G, SW = 2 * LPR, SPT = TC / SW;
    __shared__ double part[W][G][SW];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * W + wv;
    if (s >= nstrips) return;
    const int tile = s / SPT, sub = s % SPT, g = lane / LPR, cl = lane % LPR;
    const double* col = AR + (size_t)tile * cap * TC + sub * SW + 2 * cl;
    double a0 = 0.0, a1 = 0.0;
    int pb = 0;
    for (; pb + G * UNR <= ny; pb += G * UNR) {
        dbl2 v[UNR];
        double y[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            v[u] = *reinterpret_cast<const dbl2*>(col + (size_t)(pb + g + G * u) * TC);
            y[u] = yy[pb + g + G * u];
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            a0 = fma(v[u].x, y[u], a0);
            a1 = fma(v[u].y, y[u], a1);
        }
    }
    for (int p = pb + g; p < ny; p += G) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(col + (size_t)p * TC);
        a0 = fma(v.x, yy[p], a0);
        a1 = fma(v.y, yy[p], a1);
    }
    part[wv][g][2 * cl] = a0;
    part[wv][g][2 * cl + 1] = a1;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (lane < SW) {
        double t = 0.0;
        for (int i = 0; i < G; ++i) t += part[wv][i][lane];
        out[(size_t)tile * TC + sub * SW + lane] = t;
    }
}

// plain streaming read of the same bytes (copy-rate reference): grid-stride dbl2
__global__ void k_stream(const dbl2* __restrict__ a, size_t n2, double* out) {
    double acc = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        const dbl2 v = a[i];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <class F>
static double time_us(F launch, int reps = 200) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 10; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return 1e3 * ms / reps;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 50000;
    const int nys[] = {100, 268, 500};  // (ny multiple of 4: the strip kernels' remainder is per group)
    const int cap = 1024;
    const int ntiles = (n + TC - 1) / TC;
    const size_t elems = (size_t)ntiles * cap * TC;
    double *AR, *yy, *out;
    CK(hipMalloc(&AR, elems * sizeof(double)));
    CK(hipMalloc(&yy, cap * sizeof(double)));
    CK(hipMalloc(&out, (size_t)ntiles * 64 * TC * sizeof(double)));
    std::vector<double> h(elems, 0.5);
    CK(hipMemcpy(AR, h.data(), elems * sizeof(double), hipMemcpyHostToDevice));
    CK(hipMemcpy(yy, h.data(), cap * sizeof(double), hipMemcpyHostToDevice));
    for (int ny : nys) {
        const double mb = 8.0 * ny * (double)ntiles * TC / 1e6;
        printf("n %d tiles %d |Y| %d: %.1f MB per sweep\n", n, ntiles, ny, mb);
        auto rep = [&](const char* name, double us) {
            printf("  %-26s %8.2f us  %6.2f TB/s\n", name, us, mb / us);
        };
        rep("tile S1 U16", time_us([&] { k_tile<1, 16><<<ntiles, 64>>>(AR, yy, ny, cap, out); }));
        rep("tile S2 U16 (k_price)", time_us([&] { k_tile<2, 16><<<ntiles, 128>>>(AR, yy, ny, cap, out); }));
        rep("tile S4 U16", time_us([&] { k_tile<4, 16><<<ntiles, 256>>>(AR, yy, ny, cap, out); }));
        rep("tile S8 U16", time_us([&] { k_tile<8, 16><<<ntiles, 512>>>(AR, yy, ny, cap, out); }));
        rep("tile S4 U8", time_us([&] { k_tile<4, 8><<<ntiles, 256>>>(AR, yy, ny, cap, out); }));
        rep("tile S2 U32", time_us([&] { k_tile<2, 32><<<ntiles, 128>>>(AR, yy, ny, cap, out); }));
        {
            const int ns4 = ntiles * 4, ns8 = ntiles * 8;
            rep("strip G4 U16 W1", time_us([&] { k_strip<4, 16, 1><<<ns4, 64>>>(AR, yy, ny, cap, ns4, out); }));
            rep("strip G4 U8 W1", time_us([&] { k_strip<4, 8, 1><<<ns4, 64>>>(AR, yy, ny, cap, ns4, out); }));
            rep("strip G4 U16 W2", time_us([&] { k_strip<4, 16, 2><<<(ns4 + 1) / 2, 128>>>(AR, yy, ny, cap, ns4, out); }));
            rep("strip G8 U16 W1", time_us([&] { k_strip<8, 16, 1><<<ns8, 64>>>(AR, yy, ny, cap, ns8, out); }));
            rep("strip G8 U8 W1", time_us([&] { k_strip<8, 8, 1><<<ns8, 64>>>(AR, yy, ny, cap, ns8, out); }));
            rep("strip G2 U16 W1", time_us([&] { k_strip<2, 16, 1><<<ntiles * 2, 64>>>(AR, yy, ny, cap, ntiles * 2, out); }));
        }
        for (int R : {2, 3, 4, 6, 8})
            for (int s = 0; s < 2; ++s) {
                char nm[64];
                snprintf(nm, sizeof nm, "split R%d %s", R, s ? "S2 U16" : "S1 U16");
                if (s) rep(nm, time_us([&] { k_split<2, 16><<<ntiles * R, 128>>>(AR, yy, ny, cap, R, out); }));
                else rep(nm, time_us([&] { k_split<1, 16><<<ntiles * R, 64>>>(AR, yy, ny, cap, R, out); }));
            }
        // plain stream over a contiguous buffer of the same size (reference rate)
        const size_t n2 = (size_t)(mb * 1e6 / 16);
        rep("stream 1024x256", time_us([&] { k_stream<<<1024, 256>>>((const dbl2*)AR, n2, out); }));
        rep("stream 4096x256", time_us([&] { k_stream<<<4096, 256>>>((const dbl2*)AR, n2, out); }));
    }
    return 0;
}
