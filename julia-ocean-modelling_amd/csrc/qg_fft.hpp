// In-LDS complex FFT for one row of length N (power of two), executed by a whole
// workgroup of T threads.  Stockham autosort formulation: every pass reads R values per
// butterfly into registers, applies the twiddles, does an R-point DFT in registers and
// writes back in natural order, so no bit-reversal pass is needed.  Twiddles come from a
// table tw[m] = exp(-2*pi*i*m/N) (L2/L1-resident, N complex doubles).
#pragma once

#include "qg_common.hpp"

namespace qg {

template <bool INV>
__device__ __forceinline__ double2 mul_mi(double2 a) {  // a * (-i) forward, a * (+i) inverse
    return INV ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
}

template <bool INV>
__device__ __forceinline__ void dft2(double2 &a0, double2 &a1) {
    const double2 t = a0;
    a0 = cadd(t, a1);
    a1 = csub(t, a1);
}

template <bool INV>
__device__ __forceinline__ void dft4(double2 &a0, double2 &a1, double2 &a2, double2 &a3) {
    const double2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_mi<INV>(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

template <bool INV>
__device__ __forceinline__ void dft8(double2 (&v)[8]) {
    constexpr double h = 0.70710678118654752440;
    double2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    double2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4<INV>(e0, e1, e2, e3);
    dft4<INV>(o0, o1, o2, o3);
    // twiddles W8^k, W8 = exp(-+ i pi/4)
    const double2 w1 = INV ? make_double2(h, h) : make_double2(h, -h);
    const double2 w3 = INV ? make_double2(-h, h) : make_double2(-h, -h);
    o1 = cmul(o1, w1);
    o2 = mul_mi<INV>(o2);
    o3 = cmul(o3, w3);
    v[0] = cadd(e0, o0);
    v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1);
    v[5] = csub(e1, o1);
    v[2] = cadd(e2, o2);
    v[6] = csub(e2, o2);
    v[3] = cadd(e3, o3);
    v[7] = csub(e3, o3);
}

template <int R, bool INV>
__device__ __forceinline__ void dftR(double2 (&v)[R]) {
    if constexpr (R == 2) dft2<INV>(v[0], v[1]);
    else if constexpr (R == 4) dft4<INV>(v[0], v[1], v[2], v[3]);
    else dft8<INV>(v);
}

// radix of the next pass: 8 while the remaining length allows it and every thread still gets
// a butterfly (or radix 4 would not fill the threads either), else 4, else 2
template <int N, int T, int NS>
struct PassRadix {
    static constexpr int REM = N / NS;
    static constexpr int value =
        (REM % 8 == 0 && (N / 8 >= T || N / 4 < T)) ? 8 : ((REM % 4 == 0) ? 4 : 2);
};

// LDS index with one pad slot per 8 complex values: keeps the radix-8 scatter of the first
// pass (lane stride 8 x 16 B) free of ds_write_b128 bank conflicts.
__host__ __device__ constexpr int lpad(int x) { return x + (x >> 3); }
template <int N>
struct LdsSize {
    static constexpr int value = lpad(N - 1) + 1;  // complex elements
};

template <int N, int T, int R, int NS, bool INV>
__device__ __forceinline__ void stockham_pass(double2 *buf, const double2 *__restrict__ tw, int t) {
    constexpr int NB = N / R;                 // butterflies in this pass
    constexpr int PER = (NB + T - 1) / T;     // per thread
    double2 v[PER][R];
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int j = t + p * T;
        if (NB % T == 0 || j < NB) {
            const int k = j % NS;
#pragma unroll
            for (int r = 0; r < R; ++r) v[p][r] = buf[lpad(j + r * NB)];
            if constexpr (NS > 1) {
                // W^(r k) by repeated multiplication of one table twiddle W^k (error <= R eps)
                double2 w = tw[k * (N / (NS * R))];
                if (INV) w.y = -w.y;
                double2 wr = w;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    v[p][r] = cmul(v[p][r], wr);
                    if (r + 1 < R) wr = cmul(wr, w);
                }
            }
            dftR<R, INV>(v[p]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int j = t + p * T;
        if (NB % T == 0 || j < NB) {
            const int k = j % NS;
            const int base = (j / NS) * NS * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[lpad(base + r * NS)] = v[p][r];
        }
    }
    __syncthreads();
}

template <int N, int T, int NS, bool INV>
__device__ __forceinline__ void fft_passes(double2 *buf, const double2 *__restrict__ tw, int t) {
    if constexpr (NS < N) {
        constexpr int R = PassRadix<N, T, NS>::value;
        stockham_pass<N, T, R, NS, INV>(buf, tw, t);
        fft_passes<N, T, NS * R, INV>(buf, tw, t);
    }
}

// threadIdx.x laundered through an opaque move: the FFT's LDS addresses and twiddle indices
// are row-invariant, and without this the compiler hoists all of them (several passes' worth)
// out of the caller's row loop and keeps them live in VGPRs
__device__ __forceinline__ int opaque_tid() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
    return t;
}

// Unnormalised DFT of buf[lpad(0..N)) in place (natural order in and out).  Caller must have
// synchronised after writing buf; returns after a barrier.
template <int N, int T, bool INV>
__device__ __forceinline__ void fft_lds(double2 *buf, const double2 *__restrict__ tw) {
    fft_passes<N, T, 1, INV>(buf, tw, opaque_tid());
}

}  // namespace qg
