// In-LDS complex FFT for one row of length N (power of two), executed by a whole workgroup
// of T threads.  Stockham autosort formulation, out of place between two LDS buffers
// (ping-pong): every pass reads R values per butterfly, applies the twiddles, does an R-point
// DFT in registers and writes the next buffer in natural order -- one barrier per pass and no
// bit-reversal pass.  When one butterfly per thread covers the row (N / R == T) the first
// pass can take its inputs from registers and the last pass can leave its outputs in
// registers, in exactly the element order of a coalesced row access (element t + r*T), so the
// caller's global load / store feeds the transform without an LDS round trip.
//
// When two row buffers do not fit in LDS (N = 8192) the passes run in place on one buffer
// with a barrier between each pass's reads and writes (callers pass b1 == b0).
//
// Twiddles live in LDS (row-invariant, filled once per workgroup from the global table
// tw[m] = exp(-2 pi i m / N)): one small table per pass, entries exp(-2 pi i k / (NS R)),
// k < NS; passes with NS > 256 use a two-level table (64 low + NS/64 high entries, one
// complex multiply to combine).
//
// C: the complex type the transform computes and stores in -- double2 (default), or float2
// for the F32-state wide-row solver (half the LDS bytes and registers, F32 arithmetic; the
// twiddles are the F64 table rounded once).
//
// LDS layouts: a pass with stride NS < 8 scatters with a lane stride of NS*16 B, which
// conflicts in the 8-lane groups of ds_write_b128; its output buffer is XOR-swizzled within
// aligned 8-element blocks, x ^ ((x >> 3) & 7).  That is conflict-free both for those writes
// and for the next pass's contiguous ds_read_b128 (16-lane groups, 64 banks); a pad slot per 8
// values (the layout before) fixed the writes but left those reads 2-way conflicted: 256
// extra LDS cycles per 4096-point row, measured as SQ_LDS_BANK_CONFLICT in the wide-row passes
// (tools/lds_bank_model.py models both).  8-byte elements (float2) are banked in 16-lane
// groups of 16 slots: x ^ ((x >> 4) & 7) keeps both the scattered writes and the contiguous
// reads distinct there, and the stride-8 pass (whose 16-lane groups span two 8-lane runs 64
// elements apart) flips bit 3 by bit 6.  All other buffers (caller-written rows, wide-stride
// pass outputs) are read and written contiguously and use the identity layout.
#pragma once

#include "qg_common.hpp"

namespace qg {

template <bool INV, class C>
__device__ __forceinline__ C mul_mi(C a) {  // a * (-i) forward, a * (+i) inverse
    return INV ? cmake<C>(-a.y, a.x) : cmake<C>(a.y, -a.x);
}

template <bool INV, class C>
__device__ __forceinline__ void dft2(C &a0, C &a1) {
    const C t = a0;
    a0 = cadd(t, a1);
    a1 = csub(t, a1);
}

template <bool INV, class C>
__device__ __forceinline__ void dft4(C &a0, C &a1, C &a2, C &a3) {
    const C t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_mi<INV>(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

template <bool INV, class C>
__device__ __forceinline__ void dft8(C (&v)[8]) {
    using R = typename CxReal<C>::R;
    constexpr R h = (R)0.70710678118654752440;
    C e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    C o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4<INV>(e0, e1, e2, e3);
    dft4<INV>(o0, o1, o2, o3);
    // twiddles W8^k, W8 = exp(-+ i pi/4)
    const C w1 = INV ? cmake<C>(h, h) : cmake<C>(h, -h);
    const C w3 = INV ? cmake<C>(-h, h) : cmake<C>(-h, -h);
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

template <int R, bool INV, class C>
__device__ __forceinline__ void dftR(C (&v)[R]) {
    if constexpr (R == 2) dft2<INV>(v[0], v[1]);
    else if constexpr (R == 4) dft4<INV>(v[0], v[1], v[2], v[3]);
    else dft8<INV>(v);
}

// radix of the pass with stride NS: 8 while the remaining length allows it and every thread
// still gets a butterfly (or radix 4 would not fill the threads either), else 4, else 2
template <int N, int T, int NS>
struct PassRadix {
    static constexpr int REM = N / NS;
    static constexpr int value =
        (REM % 8 == 0 && (N / 8 >= T || N / 4 < T)) ? 8 : ((REM % 4 == 0) ? 4 : 2);
};

__host__ __device__ constexpr int lpad(int x) { return x + (x >> 3); }
// layout of the buffer written by the pass with stride NS (caller: NS = 0); EB = element bytes
template <int NS, int EB = 16>
__device__ __forceinline__ int lay(int x) {
    if constexpr (NS > 0 && NS < 8) return EB == 16 ? x ^ ((x >> 3) & 7) : x ^ ((x >> 4) & 7);
    else if constexpr (NS == 8 && EB == 8) return x ^ (((x >> 6) & 1) << 3);
    else return x;
}
template <int N>
struct LdsSize {  // complex elements of one row buffer (any layout; sized for the padded one)
    static constexpr int value = lpad(N - 1) + 1;
};

// pass sequence facts, by recursion over the stride NS
template <int N, int T, int NS, bool END = (NS >= N)>
struct Passes {
    static constexpr int R = PassRadix<N, T, NS>::value;
    using Next = Passes<N, T, NS * R>;
    static constexpr int count = 1 + Next::count;
    static constexpr int last_ns = (NS * R >= N) ? NS : Next::last_ns;
    static constexpr int tw_here = NS == 1 ? 0 : (NS <= 256 ? NS : 64 + NS / 64);
    static constexpr int tw_total = tw_here + Next::tw_total;  // this pass and the later ones
};
template <int N, int T, int NS>
struct Passes<N, T, NS, true> {
    static constexpr int count = 0, last_ns = 0, tw_here = 0, tw_total = 0;
};

constexpr int LDS_COMPLEX_MAX = 160 * 1024 / 16;  // double2 elements in a CU's 160 KB LDS

template <int N, int T>
struct FftPlan {
    using P = Passes<N, T, 1>;
    static constexpr int R0 = P::R;
    static constexpr int NPASS = P::count;
    static constexpr int LAST_NS = P::last_ns;
    static constexpr int R_LAST = N / LAST_NS;
    static constexpr int TW = P::tw_total;
    // one butterfly per thread in the first / last pass, in row order t + r*T
    static constexpr bool REG_IN = (N / R0 == T);
    static constexpr bool REG_OUT = (N / R_LAST == T);
    // two row buffers (ping-pong, one barrier per pass) when they fit, else one buffer
    // transformed in place (two barriers per pass): N = 8192
    static constexpr bool PINGPONG = 2 * LdsSize<N>::value + TW <= LDS_COMPLEX_MAX;
    static constexpr int LDS = (PINGPONG ? 2 : 1) * LdsSize<N>::value + TW;  // complex elements
    template <int NS>
    static constexpr int tw_off() { return P::tw_total - Passes<N, T, NS>::tw_total; }
};

template <int N, int T, int NS, class C>
__device__ __forceinline__ void fill_twiddles(C *twl, const double2 *__restrict__ tw, int t) {
    if constexpr (NS < N) {
        using P = Passes<N, T, NS>;
        constexpr int R = P::R, S = N / (NS * R), off = FftPlan<N, T>::template tw_off<NS>();
        if constexpr (NS > 1) {
            for (int e = t; e < P::tw_here; e += T) {
                int m;
                if constexpr (NS <= 256) m = e * S;
                else m = e < 64 ? e * S : 64 * (e - 64) * S;
                cconv(twl[off + e], tw[m]);
            }
        }
        fill_twiddles<N, T, NS * R>(twl, tw, t);
    }
}

// Fill the LDS twiddle tables (caller synchronises before the first transform).
template <int N, int T, class C>
__device__ __forceinline__ void fft_init_twiddles(C *twl, const double2 *__restrict__ tw) {
    fill_twiddles<N, T, 1>(twl, tw, threadIdx.x);
}

// The same fill in two halves.  fft_init_twiddles issues one load per pass and writes it to
// LDS before the next pass's load goes out: one memory latency per pass, in front of a
// kernel's first row.  fft_twiddle_load issues all of this thread's loads (flat entry e of the
// LDS tables -> global index tw_src(e)); the caller then issues its own first loads and calls
// fft_twiddle_store before its first barrier, so the latencies overlap.
template <int N, int T>
struct TwFill {
    static constexpr int TW = FftPlan<N, T>::TW;
    static constexpr int PER = (TW + T - 1) / T > 0 ? (TW + T - 1) / T : 1;
    double2 v[PER];
};
template <int N, int T, int NS>
__device__ __forceinline__ int tw_src(int e) {  // e >= tw_off<NS>()
    if constexpr (NS >= N) {
        return 0;
    } else {
        using P = Passes<N, T, NS>;
        constexpr int R = P::R, S = N / (NS * R), off = FftPlan<N, T>::template tw_off<NS>();
        if (P::tw_here > 0 && e < off + P::tw_here) {
            const int l = e - off;
            if constexpr (NS <= 256) return l * S;
            else return l < 64 ? l * S : 64 * (l - 64) * S;
        }
        return tw_src<N, T, NS * R>(e);
    }
}
template <int N, int T>
__device__ __forceinline__ void fft_twiddle_load(TwFill<N, T> &f, const double2 *__restrict__ tw) {
#pragma unroll
    for (int p = 0; p < TwFill<N, T>::PER; ++p) {
        const int e = threadIdx.x + p * T;
        if (e < TwFill<N, T>::TW) f.v[p] = tw[tw_src<N, T, 1>(e)];
    }
}
template <int N, int T, class C>
__device__ __forceinline__ void fft_twiddle_store(C *twl, const TwFill<N, T> &f) {
#pragma unroll
    for (int p = 0; p < TwFill<N, T>::PER; ++p) {
        const int e = threadIdx.x + p * T;
        if (e < TwFill<N, T>::TW) cconv(twl[e], f.v[p]);
    }
}

// One pass: butterflies j = t, t + T, ...; reads `src` (layout of the writer with stride
// IN_NS) or registers `io` (FROM_REG), writes `dst` with layout lay<NS> then a barrier, or
// leaves the result in `io` (TO_REG, no barrier).
template <int N, int T, int NS, int IN_NS, bool INV, bool FROM_REG, bool TO_REG, class C>
__device__ __forceinline__ void fft_pass(const C *src, C *dst, const C *twl, int t,
                                         C (&io)[PassRadix<N, T, NS>::value]) {
    constexpr int R = PassRadix<N, T, NS>::value;
    constexpr int NB = N / R;
    constexpr int PER = (NB + T - 1) / T;
    static_assert(!(FROM_REG || TO_REG) || (NB == T), "register I/O needs one butterfly per thread");
    C v[PER][R];
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int j = t + p * T;
        if (NB % T == 0 || j < NB) {
            const int k = j % NS;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if constexpr (FROM_REG) v[p][r] = io[r];
                else v[p][r] = src[lay<IN_NS, sizeof(C)>(j + r * NB)];
            }
            if constexpr (NS > 1) {
                constexpr int off = FftPlan<N, T>::template tw_off<NS>();
                C w;
                if constexpr (NS <= 256) w = twl[off + k];
                else w = cmul(twl[off + (k & 63)], twl[off + 64 + (k >> 6)]);
                if (INV) w.y = -w.y;
                // W^(r k) by repeated multiplication (error <= R eps)
                C wr = w;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    v[p][r] = cmul(v[p][r], wr);
                    if (r + 1 < R) wr = cmul(wr, w);
                }
            }
            dftR<R, INV>(v[p]);
        }
    }
    if constexpr (TO_REG) {
#pragma unroll
        for (int r = 0; r < R; ++r) io[r] = v[0][r];
    } else {
        if constexpr (!FftPlan<N, T>::PINGPONG && !FROM_REG) __syncthreads();  // in place: reads first
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int j = t + p * T;
            if (NB % T == 0 || j < NB) {
                const int k = j % NS;
                const int base = (j / NS) * NS * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) dst[lay<NS, sizeof(C)>(base + r * NS)] = v[p][r];
            }
        }
        __syncthreads();
    }
}

// Passes NS .. end, ping-ponging src -> dst.  LAST_REG: the final pass leaves its output in
// `io` (element t + r*T).  Returns nothing; which buffer holds the result is FftRun::final.
template <int N, int T, int NS, int IN_NS, bool INV, bool LAST_REG, class C>
__device__ __forceinline__ void fft_run(C *src, C *dst, const C *twl, int t, C (&io)[FftPlan<N, T>::R_LAST]) {
    if constexpr (NS < N) {
        constexpr int R = PassRadix<N, T, NS>::value;
        if constexpr (LAST_REG && NS * R >= N) {
            fft_pass<N, T, NS, IN_NS, INV, false, true>(src, dst, twl, t, io);
        } else {
            C dummy[R];
            fft_pass<N, T, NS, IN_NS, INV, false, false>(src, dst, twl, t, dummy);
            fft_run<N, T, NS * R, NS, INV, LAST_REG>(dst, src, twl, t, io);
        }
    }
}

// thread index laundered through an opaque move: the FFT's LDS addresses and twiddle indices
// are row-invariant, and without this the compiler hoists all of them (several passes' worth)
// out of the caller's row loop and keeps them live in VGPRs
__device__ __forceinline__ int opaque_tid() {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
    return t;
}

// Forward/inverse transform whose input row is in b0 (identity layout, written by the caller
// and synchronised).  Result: registers `io` (element t + r*T) when OUT_REG, else the buffer
// b0 or b1 named by result_in_b1 with layout lay<LAST_NS>.
template <int N, int T, bool INV, bool OUT_REG, class C = double2>
struct FftFromLds {
    using Plan = FftPlan<N, T>;
    // passes that write a buffer: all, or all but the last
    static constexpr int WRITES = Plan::NPASS - (OUT_REG ? 1 : 0);
    static constexpr bool result_in_b1 = Plan::PINGPONG && (WRITES % 2) == 1;
    // buffer read after the last barrier (by the last pass when OUT_REG, else by the caller)
    static constexpr bool b0_read_late = !Plan::PINGPONG || (OUT_REG ? (WRITES % 2 == 0) : !result_in_b1);
    __device__ static __forceinline__ void run(C *b0, C *b1, const C *twl, C (&io)[Plan::R_LAST]) {
        fft_run<N, T, 1, 0, INV, OUT_REG>(b0, b1, twl, opaque_tid(), io);
    }
};

// Transform whose input is in registers `in` (element t + r*T, needs Plan::REG_IN).  Result
// in b0 or b1 (result_in_b1) with layout lay<LAST_NS>, synchronised.
template <int N, int T, bool INV, class C = double2>
struct FftFromReg {
    using Plan = FftPlan<N, T>;
    static constexpr bool result_in_b1 = Plan::PINGPONG && (Plan::NPASS % 2) == 0;
    static constexpr bool b0_read_late = !result_in_b1;
    __device__ static __forceinline__ void run(C (&in)[Plan::R0], C *b0, C *b1, const C *twl) {
        const int t = opaque_tid();
        fft_pass<N, T, 1, 0, INV, true, false>((const C *)nullptr, b0, twl, t, in);
        C dummy[Plan::R_LAST];
        fft_run<N, T, Plan::R0, 1, INV, false>(b0, b1, twl, t, dummy);
    }
};

}  // namespace qg
