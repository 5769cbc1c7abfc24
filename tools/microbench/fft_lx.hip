// The 4096-point row transform of the spectral passes: Stockham plan (qg_fft.hpp, four LDS
// round trips + the split step's reads) against the lane-exchange plan (qg_fft_lx.hpp, two
// LDS round trips, register<->lane transposes by v_permlane*_swap / DPP, the split pairs
// exchanged in registers).  Checks the outputs agree and times both, rows L2-resident
// (transform cost) and streamed from HBM.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../julia-ocean-modelling_amd/csrc fft_lx.hip -o fft_lx
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "qg_fft.hpp"
#include "qg_fft_lx.hpp"

using namespace qg;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int N = 4096, T = 512;
using Plan = FftPlan<N, T>;
constexpr size_t LDS_OLD = sizeof(double2) * (2 * LdsSize<N>::value + Plan::TW);
constexpr size_t LDS_NEW = sizeof(double2) * lx::LDS_ELEMS;

__device__ __forceinline__ int row_of(int i, int rows_per_wg, int nres) {
    return (blockIdx.x * rows_per_wg + i) % nres;
}

// forward + split-pair read: out[k] = Z_k + conj Z_{N-k}, k < N/2
__global__ __launch_bounds__(T, 2) void fwd_old(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    using Fwd = FftFromReg<N, T, false>;
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + LdsSize<N>::value, *twl = lds + 2 * LdsSize<N>::value;
    fft_init_twiddles<N, T>(twl, tw);
    __syncthreads();
    const double2 *Zb = Fwd::result_in_b1 ? b1 : b0;
    const int t = threadIdx.x;
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
        double2 v[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) v[p] = in[(size_t)j * N + t + p * T];
        Fwd::run(v, b0, b1, twl);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = t + q * T;
            const double2 Zk = Zb[lay<Plan::LAST_NS>(k)], Zm = Zb[lay<Plan::LAST_NS>((N - k) & (N - 1))];
            out[(size_t)j * N + k] = make_double2(Zk.x + Zm.x, Zk.y - Zm.y);
        }
        if constexpr (Fwd::b0_read_late) __syncthreads();
    }
}

__global__ __launch_bounds__(T, 2) void fwd_new(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + N, *tw512 = lds + 2 * N, *stash = tw512 + 512;
    lx::fill_tw512(tw512, tw);
    __syncthreads();
    const int t = threadIdx.x;
    const int m = lx::mirror_group(t);
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
        double2 v[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) v[p] = in[(size_t)j * N + t + p * T];
        lx::fft<false, false, true>(v, b0, b1, tw512, t);
        lx::mirror_exchange(v, stash, t);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = m + q * T;
            const double2 Zk = v[q], Zm = t == 0 ? v[(8 - q) & 7] : v[7 - q];
            out[(size_t)j * N + k] = make_double2(Zk.x + Zm.x, Zk.y - Zm.y);
        }
    }
}

// inverse: out = IDFT(in) in natural order
__global__ __launch_bounds__(T, 2) void inv_old(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    using Inv = FftFromLds<N, T, true, true>;
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + LdsSize<N>::value, *twl = lds + 2 * LdsSize<N>::value;
    fft_init_twiddles<N, T>(twl, tw);
    __syncthreads();
    const int t = threadIdx.x;
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
#pragma unroll
        for (int p = 0; p < 8; ++p) b0[t + p * T] = in[(size_t)j * N + t + p * T];
        __syncthreads();
        double2 xo[Plan::R_LAST];
        Inv::run(b0, b1, twl, xo);
#pragma unroll
        for (int p = 0; p < 8; ++p) out[(size_t)j * N + t + p * T] = xo[p];
        if constexpr (Inv::b0_read_late) __syncthreads();
    }
}

__global__ __launch_bounds__(T, 2) void inv_new(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + N, *tw512 = lds + 2 * N, *stash = tw512 + 512;
    lx::fill_tw512(tw512, tw);
    __syncthreads();
    const int t = threadIdx.x;
    const int g = lx::mirror_group(t);
    const int gp = ((t & ~32) == 0) ? g : 512 - g;  // the partner lane's group
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
        double2 v[8];
        // registers 0-3 of the own group, 4-7 of the partner's (as the split step leaves
        // them), then the exchange
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = in[(size_t)j * N + (r < 4 ? g : gp) + r * T];
        lx::mirror_exchange(v, stash, t);
        lx::fft<true, true, false>(v, b0, b1, tw512, t);
#pragma unroll
        for (int p = 0; p < 8; ++p) out[(size_t)j * N + t + p * T] = v[p];
    }
}

// as the spectral passes run it: the next row prefetched during the transform (hook); ONE:
// the one-buffer transform, half the LDS, two workgroups per CU
template <bool ONE>
__global__ __launch_bounds__(T, 2) void fwd_pf(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = ONE ? lds : lds + N, *tw512 = lds + (ONE ? N : 2 * N), *stash = tw512 + 512;
    lx::fill_tw512(tw512, tw);
    __syncthreads();
    const int t = threadIdx.x;
    const int m = lx::mirror_group(t);
    double2 pf[8];
    {
        const int j = row_of(0, rows, nres);
#pragma unroll
        for (int p = 0; p < 8; ++p) pf[p] = in[(size_t)j * N + t + p * T];
    }
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
        double2 v[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) v[p] = pf[p];
        lx::fft<false, false, true, ONE>(v, b0, b1, tw512, t, [&]() {
            if (i + 1 < rows) {
                const int jn = row_of(i + 1, rows, nres);
#pragma unroll
                for (int p = 0; p < 8; ++p) pf[p] = in[(size_t)jn * N + t + p * T];
            }
        });
        lx::mirror_exchange(v, stash, t);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = m + q * T;
            const double2 Zk = v[q], Zm = t == 0 ? v[(8 - q) & 7] : v[7 - q];
            out[(size_t)j * N + k] = make_double2(Zk.x + Zm.x, Zk.y - Zm.y);
        }
    }
}

template <bool ONE>
__global__ __launch_bounds__(T, 2) void inv_pf(const double2 *in, double2 *out, const double2 *tw, int rows, int nres) {
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = ONE ? lds : lds + N, *tw512 = lds + (ONE ? N : 2 * N), *stash = tw512 + 512;
    lx::fill_tw512(tw512, tw);
    __syncthreads();
    const int t = threadIdx.x;
    const int g = lx::mirror_group(t);
    const int gp = ((t & ~32) == 0) ? g : 512 - g;
    double2 pf[8];
    auto load = [&](int j) {
#pragma unroll
        for (int r = 0; r < 8; ++r) pf[r] = in[(size_t)j * N + (r < 4 ? g : gp) + r * T];
    };
    load(row_of(0, rows, nres));
    for (int i = 0; i < rows; ++i) {
        const int j = row_of(i, rows, nres);
        double2 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = pf[r];
        lx::mirror_exchange(v, stash, t);
        lx::fft<true, true, false, ONE>(v, b0, b1, tw512, t, [&]() {
            if (i + 1 < rows) load(row_of(i + 1, rows, nres));
        });
#pragma unroll
        for (int p = 0; p < 8; ++p) out[(size_t)j * N + t + p * T] = v[p];
    }
}

typedef void (*Kern)(const double2 *, double2 *, const double2 *, int, int);
constexpr size_t LDS_ONE = sizeof(double2) * (lx::N + 512 + 8);

int main() {
    const int WG = 256, ROWS = 64;
    const int NROWS = WG * ROWS;  // streamed case: every row distinct (1 GB per array)
    std::vector<double2> tw(N), h(N * 16);
    for (int m = 0; m < N; ++m) {
        const long double a = -2.0L * 3.14159265358979323846264338327950288L * m / N;
        tw[m] = make_double2((double)cosl(a), (double)sinl(a));
    }
    unsigned long long s = 12345;
    auto rnd = [&]() {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        return (double)(s >> 11) * 0x1.0p-53 - 0.5;
    };
    double2 *din, *dout1, *dout2, *dtw;
    CK(hipMalloc(&din, sizeof(double2) * (size_t)N * NROWS));
    CK(hipMalloc(&dout1, sizeof(double2) * (size_t)N * NROWS));
    CK(hipMalloc(&dout2, sizeof(double2) * (size_t)N * NROWS));
    CK(hipMalloc(&dtw, sizeof(double2) * N));
    CK(hipMemcpy(dtw, tw.data(), sizeof(double2) * N, hipMemcpyHostToDevice));
    std::vector<double2> hin((size_t)N * NROWS);
    for (auto &x : hin) x = make_double2(rnd(), rnd());
    CK(hipMemcpy(din, hin.data(), sizeof(double2) * hin.size(), hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void *)fwd_old, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_OLD));
    CK(hipFuncSetAttribute((const void *)inv_old, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_OLD));
    CK(hipFuncSetAttribute((const void *)fwd_new, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_NEW));
    CK(hipFuncSetAttribute((const void *)inv_new, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_NEW));
    std::printf("LDS bytes: old %zu new %zu\n", LDS_OLD, LDS_NEW);

    // correctness on 16 rows
    auto compare = [&](Kern ka, size_t la, Kern kb, size_t lb, const char *name, bool half) -> int {
        const int rows = 16;
        CK(hipMemset(dout1, 0, sizeof(double2) * N * rows));
        CK(hipMemset(dout2, 0, sizeof(double2) * N * rows));
        ka<<<1, T, la>>>(din, dout1, dtw, rows, rows);
        kb<<<1, T, lb>>>(din, dout2, dtw, rows, rows);
        CK(hipDeviceSynchronize());
        std::vector<double2> a((size_t)N * rows), b((size_t)N * rows);
        CK(hipMemcpy(a.data(), dout1, sizeof(double2) * a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dout2, sizeof(double2) * b.size(), hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (int j = 0; j < rows; ++j)
            for (int k = 0; k < (half ? N / 2 : N); ++k) {
                const size_t i = (size_t)j * N + k;
                md = fmax(md, fmax(fabs(a[i].x - b[i].x), fabs(a[i].y - b[i].y)));
                mx = fmax(mx, fmax(fabs(a[i].x), fabs(a[i].y)));
            }
        std::printf("%s: max |old - new| = %.3e (max |old| %.3e, rel %.3e)\n", name, md, mx, md / mx);
        return 0;
    };
    if (compare(fwd_old, LDS_OLD, fwd_new, LDS_NEW, "forward+split", true)) return 1;
    if (compare(inv_old, LDS_OLD, inv_new, LDS_NEW, "inverse", false)) return 1;
    for (auto k : {(const void *)fwd_pf<false>, (const void *)inv_pf<false>})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_NEW));
    for (auto k : {(const void *)fwd_pf<true>, (const void *)inv_pf<true>})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_ONE));
    if (compare(fwd_new, LDS_NEW, fwd_pf<true>, LDS_ONE, "forward+split one-buffer", true)) return 1;
    if (compare(inv_new, LDS_NEW, inv_pf<true>, LDS_ONE, "inverse one-buffer", false)) return 1;
    {
        // prefetching passes: two buffers (one workgroup per CU, 256 x 64 rows) against one
        // buffer (two per CU, 512 x 32 rows), same rows in all
        struct P {
            const char *name;
            Kern k;
            size_t lds;
            int wg, rows;
        } ps[] = {{"fwd_pf2", fwd_pf<false>, LDS_NEW, 256, 64}, {"fwd_pf1", fwd_pf<true>, LDS_ONE, 512, 32},
                  {"inv_pf2", inv_pf<false>, LDS_NEW, 256, 64}, {"inv_pf1", inv_pf<true>, LDS_ONE, 512, 32}};
        hipEvent_t f0, f1;
        CK(hipEventCreate(&f0));
        CK(hipEventCreate(&f1));
        for (int rep = 0; rep < 3; ++rep)
            for (int nres : {16, NROWS})
                for (auto &k : ps) {
                    k.k<<<k.wg, T, k.lds>>>(din, dout1, dtw, k.rows, nres);
                    CK(hipEventRecord(f0));
                    const int it = 10;
                    for (int r = 0; r < it; ++r) k.k<<<k.wg, T, k.lds>>>(din, dout1, dtw, k.rows, nres);
                    CK(hipEventRecord(f1));
                    CK(hipEventSynchronize(f1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, f0, f1));
                    const double us = ms * 1e3 / it;
                    std::printf("rep %d %-8s rows %s: %8.1f us per launch, %6.3f us per row per CU\n", rep, k.name,
                                nres == 16 ? "L2 " : "HBM", us, us / 64);
                }
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct K {
        const char *name;
        Kern k;
        size_t lds;
    } ks[] = {{"fwd_old", fwd_old, LDS_OLD}, {"fwd_new", fwd_new, LDS_NEW}, {"inv_old", inv_old, LDS_OLD}, {"inv_new", inv_new, LDS_NEW}};
    for (int rep = 0; rep < 3; ++rep) {
        for (int nres : {16, NROWS}) {
            for (auto &k : ks) {
                k.k<<<WG, T, k.lds>>>(din, dout1, dtw, ROWS, nres);
                CK(hipEventRecord(e0));
                const int it = 10;
                for (int r = 0; r < it; ++r) k.k<<<WG, T, k.lds>>>(din, dout1, dtw, ROWS, nres);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / it;
                std::printf("rep %d %-8s rows %s: %8.1f us per launch, %6.3f us per row per CU\n", rep, k.name,
                            nres == 16 ? "L2 " : "HBM", us, us / ROWS);
            }
        }
    }
    return 0;
}
