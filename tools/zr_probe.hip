// FTRAN-z shape probe: z_i = sum_p A[i, S_p] alpha_p over row tiles, one fma
// chain per 32-position chunk (the reduction k_ftran_zr and the oracle share),
// column-major AS ([k][m], the library's layout).  Variants: rows per lane
// RPL (8- or 16-byte loads), lanes per chunk LPC (a wave runs 64 / LPC chunks
// at once), W waves per row tile (tile = LPC * RPL rows).  "cold" runs flush
// the 256 MiB Infinity Cache first (a 1 GiB read), as the C4 pricing sweep does
// between two FTRAN-z launches; "warm" runs back to back (C3: AR + AS fit).
//   hipcc --offload-arch=gfx950 -O3 -o tools/zr_probe tools/zr_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int ZC = 32;

template <int W, int RPL, int LPC>
__global__ void __launch_bounds__(64 * W) k_z(const double* __restrict__ AS, const double* __restrict__ alS, int m,
                                              int k, double* __restrict__ z) {
    constexpr int TR = LPC * RPL, CPW = 64 / LPC;
    extern __shared__ double lds[];  // [nch][TR] partials, then [k] alpha
    const int nch = (k + ZC - 1) / ZC;
    double* part = lds;
    double* als = lds + nch * TR;
    for (int p = threadIdx.x; p < k; p += blockDim.x) als[p] = alS[p];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int sub = lane % LPC, cg = lane / LPC;
    const int i0 = blockIdx.x * TR + sub * RPL;
    const int ic = i0 < m ? i0 : m - RPL;
    for (int ch = w * CPW + cg; ch < nch; ch += W * CPW) {
        const int c0 = ch * ZC, len = min(ZC, k - c0);
        if constexpr (RPL == 1) {
            double a[ZC];
#pragma unroll
            for (int t = 0; t < ZC; ++t) {
                const int tt = t < len ? t : len - 1;
                a[t] = AS[(size_t)(c0 + tt) * m + ic];
            }
            double acc = 0.0;
#pragma unroll
            for (int t = 0; t < ZC; ++t)
                if (t < len) acc = fma(a[t], als[c0 + t], acc);
            part[ch * TR + sub] = acc;
        } else {
            double2 a[ZC];
#pragma unroll
            for (int t = 0; t < ZC; ++t) {
                const int tt = t < len ? t : len - 1;
                a[t] = *(const double2*)(AS + (size_t)(c0 + tt) * m + ic);
            }
            double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
            for (int t = 0; t < ZC; ++t)
                if (t < len) {
                    acc0 = fma(a[t].x, als[c0 + t], acc0);
                    acc1 = fma(a[t].y, als[c0 + t], acc1);
                }
            part[ch * TR + 2 * sub] = acc0;
            part[ch * TR + 2 * sub + 1] = acc1;
        }
    }
    __syncthreads();
    const int i = blockIdx.x * TR + (int)threadIdx.x;
    if ((int)threadIdx.x < TR && i < m) {
        double s = 0.0;
        for (int ch = 0; ch < nch; ++ch) s += part[ch * TR + threadIdx.x];
        z[i] = s;
    }
}

__global__ void k_flush(const double2* __restrict__ b, size_t n, double* out) {
    double acc = 0.0;
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < n; j += (size_t)gridDim.x * blockDim.x) {
        const double2 v = b[j];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main() {
    const size_t fl_n = (size_t)1 << 26;  // 1 GiB of double2
    double2* fl;
    double* out;
    CK(hipMalloc(&fl, fl_n * sizeof(double2)));
    CK(hipMemset(fl, 0, fl_n * sizeof(double2)));
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Case { int m, k; } cases[] = {{5000, 270}, {10000, 300}, {10000, 529}, {10000, 800}};
    std::vector<double> zref;
    for (auto cs : cases) {
        const int m = cs.m, k = cs.k;
        const size_t ncm = (size_t)k * m;
        double *cm, *al, *z;
        CK(hipMalloc(&cm, ncm * 8));
        CK(hipMalloc(&al, (size_t)k * 8));
        CK(hipMalloc(&z, (size_t)m * 8));
        std::vector<double> h(ncm);
        for (size_t j = 0; j < h.size(); ++j) h[j] = (double)((j * 2654435761u) % 1000) / 1000.0;
        CK(hipMemcpy(cm, h.data(), ncm * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(al, h.data(), (size_t)k * 8, hipMemcpyHostToDevice));
        const double mb = 8.0 * m * k / 1e6;
        printf("m %d k %d: %.1f MB\n", m, k, mb);
        bool first = true;
        auto run = [&](const char* name, int tr, auto launch) {
            for (int cold = 0; cold < 2; ++cold) {
                double tot = 0.0;
                const int reps = 40;
                for (int rep = 0; rep < reps + 3; ++rep) {
                    if (cold) k_flush<<<2048, 256>>>(fl, fl_n, out);
                    CK(hipEventRecord(e0));
                    launch();
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms = 0.f;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep >= 3) tot += ms;
                }
                const double us = 1e3 * tot / reps;
                printf("  %-22s %4d tiles %-5s %8.2f us  %6.2f TB/s\n", name, (m + tr - 1) / tr, cold ? "cold" : "warm",
                       us, mb / us);
            }
            std::vector<double> hz(m);  // every variant must give the same bits
            CK(hipMemcpy(hz.data(), z, (size_t)m * 8, hipMemcpyDeviceToHost));
            if (first) zref = hz, first = false;
            else if (hz != zref) printf("    MISMATCH vs the first variant\n");
        };
        auto lds = [&](int tr) { return ((size_t)(k + ZC - 1) / ZC * tr + k) * 8; };
#define V(W_, R_, L_)                                                                                       \
    run("W" #W_ " RPL" #R_ " LPC" #L_, L_ * R_, [&] {                                                       \
        k_z<W_, R_, L_><<<(m + L_ * R_ - 1) / (L_ * R_), 64 * W_, lds(L_ * R_)>>>(cm, al, m, k, z);           \
    })
        V(8, 1, 32);  // the library's shape (32-row tiles, 8 B loads, 2 chunks per wave)
        V(4, 1, 32);
        V(4, 2, 16);  // 32-row tiles, 16 B loads, 4 chunks per wave
        V(8, 2, 16);
        V(8, 2, 32);  // 64-row tiles, 16 B loads
        V(4, 1, 16);  // 16-row tiles, 8 B loads, 4 chunks per wave
        V(8, 1, 16);
        V(2, 2, 16);
        V(2, 1, 16);
        CK(hipGetLastError());
        CK(hipFree(cm));
        CK(hipFree(al));
        CK(hipFree(z));
    }
    return 0;
}
