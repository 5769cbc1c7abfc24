// Spectral (FACR) direct solver kernels for gfx950 -- see qg_spectral.hpp for the method.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "qg_fft.hpp"
#include "qg_fft_lx.hpp"
#include "qg_spectral.hpp"

namespace qg {

constexpr int CARRY_WAVES = 8;
constexpr int PIN_THREADS = 256;
__host__ __device__ inline int pin_kblocks(int KH) { return (2 * KH + PIN_THREADS - 1) / PIN_THREADS; }

template <int N>
struct Geo {
    // threads per row: N/8 (one radix-8 butterfly per thread and pass: 4 passes at N = 4096).
    // One workgroup per CU (two row buffers + twiddles = 154 KB of LDS at N = 4096);
    // registers capped at 512 / (T / 256) per lane so the whole workgroup stays resident.
    // (below N = 2048 the N/8 workgroup would be too small to keep a CU busy: N/4, <= 256)
    // (N = 8192: 1024 threads, registers capped at 128 -- some spill; capability, not speed)
    static constexpr int T0 = N / 8 >= 256 ? N / 8 : (N / 4 < 256 ? N / 4 : 256);
    static constexpr int T = T0 < 64 ? 64 : (T0 > 1024 ? 1024 : T0);
    static constexpr int MINW = T / 256 < 1 ? 1 : T / 256;
    static constexpr int KH = N / 2 + 1;
    // wavenumber slots per thread over k in [0, N/2); the real Nyquist line k = N/2 rides in
    // the imaginary part of the (also real) k = 0 slot of thread 0
    static constexpr int KQ = N / 2 >= T ? N / 2 / T : 1;
    static constexpr int EP = (N + T - 1) / T;  // row elements per thread
};

// Storage of the fields (S) and of the spectral intermediate u: double2 for F64 states,
// float2 for F32 states; the transform and the recurrences always run in F64.
template <class S>
struct Store;
template <>
struct Store<double> {
    using C = double2;
    __device__ static C c(double2 v) { return v; }
};
template <>
struct Store<float> {
    using C = float2;
    __device__ static C c(double2 v) { return make_float2((float)v.x, (float)v.y); }
};
// store of the spectral intermediate u
__device__ __forceinline__ void st_u(double2 *p, double2 v) {
    *p = v;
}
__device__ __forceinline__ void st_u(float2 *p, float2 v) {
    *p = v;
}
__device__ __forceinline__ double2 d2(double2 v) { return v; }
__device__ __forceinline__ double2 d2(float2 v) { return make_double2(v.x, v.y); }

__device__ __forceinline__ double2 cfma(double s, double2 x, double2 y) {  // s*x + y
    return make_double2(s * x.x + y.x, s * x.y + y.y);
}

// coefficient loads of the power-of-two passes
#define QG_CRR(o) a.crr[o]
#define QG_CCS(o) a.ccs[o]
#define QG_CR(o) a.cr[o]

// ------------------------------------------------------------------------------------
// pass A: project + row DFT + chunk-local backward filter (one workgroup per chunk)
// ------------------------------------------------------------------------------------
template <int N, class S>
__global__ __launch_bounds__(Geo<N>::T, Geo<N>::MINW) void spec_passA(SpecArgs a) {
    using US = typename Store<S>::C;
    using G = Geo<N>;
    constexpr int T = G::T, KQ = G::KQ, EP = G::EP, NH = N / 2;
    using Plan = FftPlan<N, T>;
    using FwdReg = FftFromReg<N, T, false>;
    using FwdLds = FftFromLds<N, T, false, false>;
    // N = 4096: the lane-exchange transform (qg_fft_lx.hpp), whose output leaves each thread
    // the elements g + 512 r of its mirror group g, so the split pairs (k, N - k) meet in
    // registers; this thread's lines are then k = g + q T
    constexpr bool LX = N == lx::N && T == lx::T;
    constexpr bool RES_B1 = Plan::REG_IN ? FwdReg::result_in_b1 : FwdLds::result_in_b1;
    constexpr bool B0_LATE = !LX && (Plan::REG_IN ? FwdReg::b0_read_late : FwdLds::b0_read_late);
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = LX ? lds + N : (Plan::PINGPONG ? lds + LdsSize<N>::value : lds),
            *twl = LX ? lds + 2 * N : lds + (Plan::PINGPONG ? 2 : 1) * LdsSize<N>::value;
    double2 *stash = lds + 2 * N + 512;  // (LX: tw512 = twl, then the mirror stash)
    const double2 *Zb = RES_B1 ? b1 : b0;
    // set-up loads first (twiddles, r of the real line k = N/2 (see spec_passB), the first
    // row), their LDS writes after: one memory latency in front of the first row, not one per
    // load
    TwFill<N, T> twf;
    if constexpr (!LX) fft_twiddle_load<N, T>(twf, a.tw);
    double2 tw5 = make_double2(0, 0);
    if constexpr (LX) tw5 = a.tw[threadIdx.x];  // W^m, m < 512 (T = 512)
    __shared__ double crN[2];
    double crv = 0;
    if (threadIdx.x < 2) crv = QG_CR(threadIdx.x * a.KS + NH);
    const int t = threadIdx.x, c = blockIdx.x;
    const int g = LX ? lx::mirror_group(t) : t;  // lines k = g + q T
    const int s0 = c * a.L, e = s0 + a.L - 1;
    const int KS = a.KS;
    const int64_t ld = a.ld;
    // u: backward filter state.  bw: the chunk summary WLS = sum_j r^(e-j) u_j, accumulated
    // with a running weight om = r^(e-j) (om *= r per row); cs = r csc.  So a row needs only r:
    // one 8-byte load per line (the coefficient tables do not fit in L1 and are re-read from
    // L2 every row: r01 measured ~18 us of pass A in those reloads with (r, 1/r) + cs).
    // Slot (0, t = 0): .x = k 0, .y = k N/2.
    double2 u[KQ][2], bw[KQ][2], om[KQ][2];
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            u[q][s] = make_double2(0, 0);
            bw[q][s] = make_double2(0, 0);
            om[q][s] = make_double2(1, 1);
        }
    const double p0 = a.pin_in[0], p1 = a.pin_in[1], p2 = a.pin_in[2], p3 = a.pin_in[3];
    const double csch = 0.5 * a.csc;
    double dc = 0;
    double *hline = a.hline;
    // register prefetch: row j-1 is loaded while row j is transformed (the barriers only wait
    // for LDS traffic, so the global loads stay in flight across the FFT)
    // (the storage type until used: F32 values converted at the load would make it wait at once)
    S pf1[EP], pf2[EP];
    auto load_into = [&](int j, auto &d1, auto &d2) {
        const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
        const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
#pragma unroll
        for (int p = 0; p < EP; ++p) {
            const int i = t + p * T;
            if (N % T == 0 || i < N) {
                d1[p] = r1[i];
                d2[p] = r2[i];
            }
        }
    };
    constexpr bool PF = N < 8192;  // (N = 8192: no register prefetch, registers are short)
    // the drop-in lean mode: row j of the inputs also goes to zcopy (ghost ring included),
    // from the registers the projection reads -- stores only, no extra reads
    auto copy_row = [&](int j, auto &d1, auto &d2) {
        S *o1 = static_cast<S *>(a.zcopy1) + (size_t)(j + 1) * ld, *o2 = static_cast<S *>(a.zcopy2) + (size_t)(j + 1) * ld;
        S *g1 = ghost_row_target(static_cast<S *>(a.zcopy1), ld, a.P, j, true);
        S *g2 = ghost_row_target(static_cast<S *>(a.zcopy2), ld, a.P, j, true);
#pragma unroll
        for (int p = 0; p < EP; ++p) {
            const int i = t + p * T;
            if (N % T == 0 || i < N) {
                store_row_with_ghosts(o1, g1, N, i, d1[p]);
                store_row_with_ghosts(o2, g2, N, i, d2[p]);
            }
        }
    };
    const bool zcopy = a.zcopy1 != nullptr;
    // r of this thread's lines, loaded once: row-invariant, and at this kernel's register
    // budget (224 VGPRs before at 4096) the values fit without spilling, so no row reloads
    // them from L2 (below 1024 no gain measured)
    constexpr bool COEF_HOIST = N >= 1024 && N <= 4096;
    double rqh[KQ][2];
    if constexpr (COEF_HOIST) {
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int k = g + q * T;
                rqh[q][s] = (NH % T == 0 || k < NH) ? QG_CR(s * KS + k) : 0.0;
            }
    }
    // LX: stage 2's twiddle powers in scalar registers (see lx::Stage2Tw; measured 106.1 ->
    // 104.5 us at 4096^2, r05i)
    lx::Stage2Tw s2f{};
    if constexpr (LX) s2f = lx::stage2_powers<false>(a.tw, t);
    // one row: consume the prefetched row (c1, c2), refill them with row j - 1, transform,
    // split, filter
    auto row_step = [&](int j, auto &c1, auto &c2) {
        if constexpr (!PF) load_into(j, c1, c2);
        if constexpr (!COEF_HOIST) asm volatile("" ::: "memory");  // keep coefficient loads in the loop (see pass B)
        // this row's r, issued ahead of the next row's prefetch: loads complete in order
        // (vmcnt), so r loaded after the prefetch would make the recurrence wait for the
        // whole next row
        double rq[KQ][2];
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int k = g + q * T;
                if constexpr (COEF_HOIST) rq[q][s] = rqh[q][s];
                else if (NH % T == 0 || k < NH) rq[q][s] = QG_CR(s * KS + k);
            }
#define QG_PA_R(q, s, o) rq[q][s]
        if (zcopy) copy_row(j, c1, c2);
        double2 zr[8];  // LX: Z_(g + 512 r) after the transform and the mirror exchange
        if constexpr (LX) {
#pragma unroll
            for (int p = 0; p < EP; ++p) zr[p] = make_double2(p0 * c1[p] + p1 * c2[p], p2 * c1[p] + p3 * c2[p]);
            const int tt = opaque_tid();
            lx::fft<false, false, true>(zr, b0, b1, twl, tt, [&]() {
                if (PF && j - 1 >= s0) load_into(j - 1, c1, c2);
            }, s2f);
            lx::mirror_exchange(zr, stash, tt);
        } else if constexpr (Plan::REG_IN) {  // first FFT pass straight from the prefetch registers
            double2 in[Plan::R0];
#pragma unroll
            for (int p = 0; p < EP; ++p) in[p] = make_double2(p0 * c1[p] + p1 * c2[p], p2 * c1[p] + p3 * c2[p]);
            if (PF && j - 1 >= s0) load_into(j - 1, c1, c2);
            FwdReg::run(in, b0, b1, twl);
        } else {
#pragma unroll
            for (int p = 0; p < EP; ++p) {
                const int i = t + p * T;
                if (N % T == 0 || i < N) b0[i] = make_double2(p0 * c1[p] + p1 * c2[p], p2 * c1[p] + p3 * c2[p]);
            }
            if (PF && j > s0) load_into(j - 1, c1, c2);
            __syncthreads();
            double2 unused[Plan::R_LAST];
            FwdLds::run(b0, b1, twl, unused);
        }
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = g + q * T;
            if (NH % T == 0 || k < NH) {
                // Z_k and its split partner Z_(N-k) (k = 0: Z_(N/2)).  LX: register q and the
                // partner lane's register 7 - q, now in register 7 - q (thread 0, group 0, is
                // its own partner: Z_(512 (8 - q)), Z_2048 in register 4)
                double2 Zk, Zm;
                if constexpr (LX) {
                    Zk = zr[q];
                    Zm = t == 0 ? zr[q == 0 ? 4 : (8 - q) & 7] : zr[7 - q];
                } else {
                    Zk = Zb[lay<Plan::LAST_NS>(k)];
                    Zm = Zb[lay<Plan::LAST_NS>(k == 0 ? NH : N - k)];
                }
                if (k == 0) {  // the two real lines k = 0 and k = N/2
                    const double2 Zn = Zm;
                    dc += Zk.x;
                    hline[j] = Zk.x;
                    const double2 B[2] = {make_double2(Zk.x, Zn.x), make_double2(Zk.y, Zn.y)};
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o0 = s * KS;
                        const double r0 = QG_PA_R(q, s, o0), rN = crN[s];
                        (void)o0;
                        u[q][s] = make_double2((r0 * a.csc) * B[s].x + r0 * u[q][s].x,
                                               (rN * a.csc) * B[s].y + rN * u[q][s].y);
                        if constexpr (LX) {  // slot order: the pair packed in slot 0
                            st_u(Urow + s * KS, Store<S>::c(u[q][s]));
                        } else {
                            st_u(Urow + s * KS, Store<S>::c(make_double2(u[q][s].x, 0)));
                            st_u(Urow + s * KS + NH, Store<S>::c(make_double2(u[q][s].y, 0)));
                        }
                        bw[q][s] = make_double2(om[q][s].x * u[q][s].x + bw[q][s].x, om[q][s].y * u[q][s].y + bw[q][s].y);
                        om[q][s] = make_double2(om[q][s].x * r0, om[q][s].y * rN);
                    }
                } else {
                    // 2 B_s: the split's halves ride in the scale, r (csc / 2) = (r csc) / 2
                    // exactly (a power of two), so u is bit for bit the halved form's
                    const double2 B[2] = {make_double2(Zk.x + Zm.x, Zk.y - Zm.y), make_double2(Zk.y + Zm.y, Zm.x - Zk.x)};
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o = s * KS + k;
                        const double r = QG_PA_R(q, s, o);  // cs = r csc
                        (void)o;
                        u[q][s] = cfma(r, u[q][s], cscale(B[s], r * csch));
                        st_u(Urow + s * KS + (LX ? t + q * T : k), Store<S>::c(u[q][s]));
                        bw[q][s] = cfma(om[q][s].x, u[q][s], bw[q][s]);
                        om[q][s].x *= r;
                    }
                }
            }
        }
        if constexpr (B0_LATE) __syncthreads();  // the next row's first pass overwrites b0
    };
#undef QG_PA_R
    if constexpr (PF) load_into(e, pf1, pf2);
    if constexpr (LX) twl[t] = tw5;
    else fft_twiddle_store<N, T>(twl, twf);
    if (threadIdx.x < 2) crN[threadIdx.x] = crv;
    __syncthreads();
    for (int j = e; j >= s0; --j) row_step(j, pf1, pf2);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const int k = g + q * T;
        if (NH % T == 0 || k < NH) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const size_t o = ((size_t)c * 2 + s) * KS;
                if (k == 0) {
                    a.ULS[o] = make_double2(u[q][s].x, 0);
                    a.ULS[o + NH] = make_double2(u[q][s].y, 0);
                    a.WLS[o] = make_double2(bw[q][s].x, 0);
                    a.WLS[o + NH] = make_double2(bw[q][s].y, 0);
                } else {
                    a.ULS[o + k] = u[q][s];
                    a.WLS[o + k] = bw[q][s];
                }
            }
        }
    }
    if (t == 0) a.dcpart[c] = dc;
}

// Block-wide reductions: wave64 shuffles, then the wave totals combined by every thread in a
// fixed order (same bits on every rank), two barriers per call.  red: >= NT/64 doubles.
template <int NT>
__device__ double block_sum(double v, double *red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[w] = v;
    __syncthreads();
    double r = 0;
    for (int g = 0; g < NT / 64; ++g) r += red[g];
    __syncthreads();
    return r;
}

template <int NT>
__device__ double block_exscan(double v, double *red) {  // exclusive prefix sum in thread order
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) red[w] = incl;
    __syncthreads();
    double base = 0;
    for (int g = 0; g < w; ++g) base += red[g];
    __syncthreads();
    double ex = __shfl_up(incl, 1, 64);
    if (lane == 0) ex = 0;
    return base + ex;
}

// The local part of the singular k = 0 Poisson line (one workgroup of NT threads).  With h_j
// the rank's line, S_j = sum_{i<=j} h_i and m_loc = mean S, it writes
//   line_j = dx^2/M * sum_{i<j} (S_i - m_loc)
// and records H = S_{P-1}, Q = sum S.  The global line (spec_pin) is this plus an affine
// correction in j; for one rank the correction is exactly zero.  Tiled block scans: tiles of
// NT * LINE_PER values staged in LDS with coalesced accesses, LINE_PER consecutive values per
// thread, running carries between tiles; the second sweep recomputes S instead of storing it.
constexpr int LINE_PER = 8;
template <int NT>
__device__ void local_line(const SpecArgs &a, double *red, double *tile) {
    constexpr int TILE = NT * LINE_PER;
    const int t = threadIdx.x, n = (int)a.P;
    auto tp = [](int x) { return x + (x >> 4); };  // pad: conflict-free strided b64 reads
    auto stage_h = [&](int j0) {
        for (int u = t; u < TILE; u += NT) tile[tp(u)] = j0 + u < n ? a.hline[j0 + u] : 0.0;
        __syncthreads();
    };
    // scan of this thread's LINE_PER staged values (after f(value, j)) joined across the
    // workgroup and offset by `carry`; inclusive or exclusive; returns the tile total
    auto scan_tile = [&](double carry, bool excl, auto f, int j0) {
        double v[LINE_PER], acc = 0;
#pragma unroll
        for (int u = 0; u < LINE_PER; ++u) {
            const int x = t * LINE_PER + u;
            const double d = f(tile[tp(x)], j0 + x);
            v[u] = excl ? acc : acc + d;
            acc += d;
        }
        const double off = carry + block_exscan<NT>(acc, red);
#pragma unroll
        for (int u = 0; u < LINE_PER; ++u) tile[tp(t * LINE_PER + u)] = off + v[u];
        return block_sum<NT>(acc, red);  // ends with a barrier: the scanned tile is visible
    };
    auto ident = [](double x, int) { return x; };
    double carryS = 0, q = 0;
    for (int j0 = 0; j0 < n; j0 += TILE) {  // sweep 1: S, its total H and its sum Q
        stage_h(j0);
        carryS += scan_tile(carryS, false, ident, j0);
        for (int u = t; u < TILE; u += NT)
            if (j0 + u < n) q += tile[tp(u)];
        __syncthreads();
    }
    const double Q = block_sum<NT>(q, red), H = carryS;
    const double mloc = Q / (double)n;
    const double scale = (a.dx * a.dx) / (double)a.M;
    carryS = 0;
    double carryX = 0;
    auto dev = [&](double S, int j) { return j < n ? S - mloc : 0.0; };
    for (int j0 = 0; j0 < n; j0 += TILE) {  // sweep 2: S again, then X = exclusive scan of S - m
        stage_h(j0);
        carryS += scan_tile(carryS, false, ident, j0);
        carryX += scan_tile(carryX, true, dev, j0);
        for (int u = t; u < TILE; u += NT)
            if (j0 + u < n) a.line[j0 + u] = scale * tile[tp(u)];
        __syncthreads();
    }
    if (t == 0) {
        a.rec[rec_DSUM(a.KS) + 1] = H;
        a.rec[rec_DSUM(a.KS) + 2] = Q;
    }
}

// The closure of one (system s, wavenumber k) line from the rank records: EXT = (Uext, Wext),
// and, for the pinned system, this line's part of the pin value (returned).  Used by spec_pin
// (after the record all-gather) and, for one rank, by spec_carry itself.
__device__ double pin_line(const SpecArgs &a, int s, int k, double delta) {
    const int G = a.nranks, KS = a.KS;
    const int64_t Pl = a.P;
    const int64_t RS = a.rec_stride;
    auto rec = [&](int g) { return a.grec + (int64_t)g * RS; };
    double pin_part = 0;
    double2 *Ue = a.EXT + (size_t)s * KS + k;
    double2 *We = a.EXT + (size_t)(2 + s) * KS + k;
    if (s == 0 && a.pinned0 && k == 0) {
        *Ue = make_double2(0, 0);
        *We = make_double2(0, 0);
        return 0;
    }
    const Coef cf = a.coef[s * KS + k];
    const bool dl = (s == 0 && a.pinned0);
    const double rPl1 = exp((double)(Pl - 1) * cf.lr);
    auto AU = [&](int g) {
        double2 v = reinterpret_cast<const double2 *>(rec(g) + rec_AU(KS))[s * KS + k];
        if (dl && g == 0) v.x += cf.cs * delta;
        return v;
    };
    auto AW = [&](int g) {
        double2 v = reinterpret_cast<const double2 *>(rec(g) + rec_AW(KS))[s * KS + k];
        if (dl && g == 0) v.x += rPl1 * (cf.cs * delta);
        return v;
    };
    auto Uext = [&](int g) {  // u_true at the start of rank g+1 (ring)
        double2 acc = make_double2(0, 0);
        for (int m = G - 1; m >= 0; --m) acc = cfma(cf.rP, acc, AU((g + 1 + m) % G));
        return cscale(acc, cf.inv1mrPt);
    };
    auto Wext = [&](int g) {  // w_true at the end of rank g-1 (ring)
        double2 acc = make_double2(0, 0);
        for (int m = G - 1; m >= 0; --m) {
            const int gg = ((g - 1 - m) % G + G) % G;
            acc = cfma(cf.rP, acc, cfma(cf.gamP, Uext(gg), AW(gg)));
        }
        return cscale(acc, cf.inv1mrPt);
    };
    const double2 ue = Uext(a.rank), we = Wext(a.rank);
    *Ue = ue;
    *We = we;
    if (dl && k >= 1) {  // pinning value: rank 0, chunk 0, row 0
        const double2 ue0 = a.rank == 0 ? ue : Uext(0);
        const double2 we0 = a.rank == 0 ? we : Wext(0);
        double2 u0 = reinterpret_cast<const double2 *>(rec(0) + rec_ULS0(KS))[k];
        u0.x += cf.cs * delta;
        const double2 uin0 = cfma(exp((double)(a.Nc - 1) * a.L * cf.lr), ue0,
                                  reinterpret_cast<const double2 *>(rec(0) + rec_UIN0(KS))[k]);
        const double2 w0 = cfma(cf.r, we0, cfma(cf.q, uin0, u0));
        const double X = w0.x;
        pin_part = (2 * k == a.M) ? X : 2 * X;
    }
    return pin_part;
}

// carry-in state of line (s, k) entering chunk c: cu = r^L u_in, w = w_in (see header), from
// the chunk's zero-closure carries (UIN_c, WIN_c) and the line's closure (Ue, We)
__device__ __forceinline__ void carry_in(const SpecArgs &a, const Coef &cf, int s, int c, double delta, bool inject,
                                         double2 Ue, double2 We, double2 uinc, double2 winc, double2 &cu,
                                         double2 &w) {
    const int64_t n = (int64_t)c * a.L;
    const double2 uin = cfma(exp((double)(a.Nc - 1 - c) * a.L * cf.lr), Ue, uinc);
    cu = cscale(uin, cf.q);
    double gc = 0;
    if (n > 0) gc = exp((double)(a.P - n + 1) * cf.lr) * (expm1(2.0 * n * cf.lr) / expm1(2.0 * cf.lr));
    double2 wi = cfma(gc, Ue, winc);
    wi = cfma(exp((double)n * cf.lr), We, wi);
    if (s == 0 && inject && c >= 1) wi.x += exp((double)(n - 1) * cf.lr) * (cf.cs * delta);
    w = wi;
}

// ------------------------------------------------------------------------------------
// carry: segment-parallel chunk scans.  A workgroup owns CARRY_KB consecutive k of one
// system; each wave's 64 lanes are CARRY_KB k x (64 / CARRY_KB) chunk segments, so the
// workgroup runs CARRY_SEG segments per k (short serial chains, ~260 workgroups at M = 4096).
// Zero carries at the rank boundaries (cross-rank and periodic closure are applied by
// spec_pin / spec_passB).
//   v_c = ULS_c + q v_{c+1}, v_Nc = 0      UIN_c = v_{c+1},  AU = v_0
//   w_c = (WLS_c + gam UIN_c) + q w_{c-1}   WIN_c = w_{c-1},  AW = w_{Nc-1}
// ------------------------------------------------------------------------------------
constexpr int CARRY_KB = 16;
constexpr int CARRY_SEG = CARRY_WAVES * (64 / CARRY_KB);
constexpr int CARRY_REG = 8;  // chunks per segment held in registers

// MINW: waves per SIMD the registers must allow.  4 lets two workgroups share a CU, for grids
// with more carry workgroups than CUs (M = 4096: 2 x 129 + 2 = 260 on 256 CUs left 4 of them
// for a second round; with two per CU 26.0 -> 21.8 us despite a small spill).  Smaller M keeps
// 1 (no spill: 1024^2 11.8 vs 13.5 us).
template <int MINW>
__global__ __launch_bounds__(64 * CARRY_WAVES, MINW) void spec_carry(SpecArgs a) {
    __shared__ double2 agg[CARRY_SEG][CARRY_KB];
    __shared__ double qlen_s[CARRY_SEG][CARRY_KB];
    constexpr int NT = 64 * CARRY_WAVES;
    if ((int)blockIdx.x == (a.KH + CARRY_KB - 1) / CARRY_KB) {  // the extra column
        __shared__ double red[CARRY_WAVES];
        if (blockIdx.y == 0) {
            if (a.pinned0) {
                __shared__ double tile[NT * LINE_PER * 17 / 16];
                local_line<NT>(a, red, tile);
            }
        } else {  // sum of the k = 0 Poisson line over this rank (-> delta), fixed order
            double d = 0;
            for (int c = threadIdx.x; c < a.Nc; c += NT) d += a.dcpart[c];
            d = block_sum<NT>(d, red);
            if (threadIdx.x == 0) a.rec[rec_DSUM(a.KS)] = d;
        }
        return;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int kk = lane % CARRY_KB, seg = wv * (64 / CARRY_KB) + lane / CARRY_KB;
    const int k = blockIdx.x * CARRY_KB + kk, s = blockIdx.y;
    const bool ok = k < a.KH;
    const int KS = a.KS, Nc = a.Nc;
    const int SL = (Nc + CARRY_SEG - 1) / CARRY_SEG;
    const int c0 = min(seg * SL, Nc), c1 = min(c0 + SL, Nc);
    double q = 0, gam = 0;
    if (ok) {
        q = a.coef[s * KS + k].q;
        gam = a.coef[s * KS + k].gam;
    }
    auto at = [&](const double2 *base, int c) { return base[((size_t)c * 2 + s) * KS + k]; };
    auto put = [&](double2 *base, int c, double2 v) { base[((size_t)c * 2 + s) * KS + k] = v; };
    // the segment's summaries, loaded once (all loads in flight together) when they fit in
    // registers; longer segments stream them from memory
    const bool inreg = SL <= CARRY_REG;
    double2 uls[CARRY_REG], wls[CARRY_REG], uin[CARRY_REG];
    if (ok && inreg) {
#pragma unroll
        for (int m = 0; m < CARRY_REG; ++m) {
            const int c = c0 + m;
            uls[m] = c < c1 ? at(a.ULS, c) : make_double2(0, 0);
            wls[m] = c < c1 ? at(a.WLS, c) : make_double2(0, 0);
        }
    }

    double2 v = make_double2(0, 0);
    double qlen = 1;
    if (ok) {
        if (inreg) {
#pragma unroll
            for (int m = CARRY_REG - 1; m >= 0; --m)
                if (c0 + m < c1) {
                    v = cfma(q, v, uls[m]);
                    qlen *= q;
                }
        } else {
            for (int c = c1 - 1; c >= c0; --c) {
                v = cfma(q, v, at(a.ULS, c));
                qlen *= q;
            }
        }
    }
    agg[seg][kk] = v;
    qlen_s[seg][kk] = qlen;
    __syncthreads();
    double2 vin = make_double2(0, 0);
    for (int g = CARRY_SEG - 1; g > seg; --g) vin = cfma(qlen_s[g][kk], vin, agg[g][kk]);
    __syncthreads();

    double2 bsum = make_double2(0, 0);
    double wq = 1;
    v = vin;
    auto back = [&](int c, double2 wl, double2 ul) {  // UIN_c, the W aggregate term, v_c
        put(a.UIN, c, v);
        const double2 wt = cfma(gam, v, wl);
        bsum = cfma(wq, wt, bsum);
        wq *= q;
        v = cfma(q, v, ul);
    };
    if (ok) {
        if (inreg) {
#pragma unroll
            for (int m = CARRY_REG - 1; m >= 0; --m)
                if (c0 + m < c1) {
                    uin[m] = v;
                    back(c0 + m, wls[m], uls[m]);
                }
        } else {
            for (int c = c1 - 1; c >= c0; --c) back(c, at(a.WLS, c), at(a.ULS, c));
        }
    }
    if (seg == 0 && ok) {
        reinterpret_cast<double2 *>(a.rec + rec_AU(KS))[s * KS + k] = v;
        if (s == 0) {
            reinterpret_cast<double2 *>(a.rec + rec_ULS0(KS))[k] = inreg ? uls[0] : at(a.ULS, 0);
            reinterpret_cast<double2 *>(a.rec + rec_UIN0(KS))[k] = inreg ? uin[0] : at(a.UIN, 0);
        }
    }
    agg[seg][kk] = bsum;
    __syncthreads();
    double2 win = make_double2(0, 0);
    for (int g = 0; g < seg; ++g) win = cfma(qlen_s[g][kk], win, agg[g][kk]);

    double2 w = win;
    if (ok) {
        if (inreg) {
#pragma unroll
            for (int m = 0; m < CARRY_REG; ++m)
                if (c0 + m < c1) {
                    put(a.WIN, c0 + m, w);
                    w = cfma(q, w, cfma(gam, uin[m], wls[m]));
                }
        } else {
            for (int c = c0; c < c1; ++c) {
                put(a.WIN, c, w);
                w = cfma(q, w, cfma(gam, at(a.UIN, c), at(a.WLS, c)));
            }
        }
    }
    if (seg == CARRY_SEG - 1 && ok) reinterpret_cast<double2 *>(a.rec + rec_AW(KS))[s * KS + k] = w;
    if (a.fuse_pin) {  // one rank: the closure (spec_pin's work) for this workgroup's lines
        __shared__ double red2[CARRY_WAVES];
        double delta = 0;
        if (a.pinned0 && s == 0) {  // delta = -(sum of dcpart), in the extra column's order
            double d = 0;
            for (int cc = threadIdx.x; cc < Nc; cc += NT) d += a.dcpart[cc];
            d = block_sum<NT>(d, red2);
            double dd = 0;
            dd += d;
            delta = -dd;
        }
        __syncthreads();  // this workgroup's record entries (AU, AW, ULS0, UIN0) are visible
        const double part = (seg == 0 && ok) ? pin_line(a, s, k, delta) : 0.0;
        const double tot = block_sum<NT>(part, red2);
        if (threadIdx.x == 0) {
            if (s == 0) a.pinpart[blockIdx.x] = tot;
            if (s == 0 && blockIdx.x == 0) {
                a.scal[0] = delta;
                if (a.pinned0) a.scal[2] = a.scal[3] = 0;  // one rank: no cross-rank line correction
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// pin: cross-rank / periodic carries, delta, singular Poisson line, pin value.  One
// workgroup; every rank runs it redundantly on the gathered records (same order -> same
// bits everywhere).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(PIN_THREADS) void spec_pin(SpecArgs a) {
    __shared__ double red[PIN_THREADS];
    const int t = threadIdx.x;
    const int G = a.nranks, KS = a.KS, KH = a.KH;
    const int64_t Pl = a.P, Pt = a.P_total;
    const int64_t RS = a.rec_stride;
    auto rec = [&](int g) { return a.grec + (int64_t)g * RS; };

    double delta = 0;
    if (a.pinned0) {
        for (int g = 0; g < G; ++g) delta += rec(g)[rec_DSUM(KS)];
        delta = -delta;
    }

    {
        double pin_part = 0;
        const int idx = blockIdx.x * PIN_THREADS + t;
        const int s = idx / KH, k = idx - s * KH;
        if (idx < 2 * KH) pin_part = pin_line(a, s, k, delta);
        const double part = block_sum<PIN_THREADS>(pin_part, red);  // this workgroup's share of the pin
        if (t == 0) a.pinpart[blockIdx.x] = part;
        if (blockIdx.x == 0 && t == 0) {
            a.scal[0] = delta;
            if (a.pinned0) {  // affine correction of the singular line (see local_line)
                // S_j = C_g + S_loc_j on rank g, C_g = sum_{g'<g} H_g'; m = global mean of S;
                // X_j = Xs_g + j (C_g - m + m_loc) + X_loc_j with Xs_g = sum_{g'<g} (P C_g' + Q_g' - P m)
                const double P = (double)Pl;
                double C = 0, tot = 0;
                for (int g = 0; g < G; ++g) {
                    tot += P * C + rec(g)[rec_DSUM(KS) + 2];
                    C += rec(g)[rec_DSUM(KS) + 1];
                }
                const double m = tot / (double)Pt;
                double Cr = 0, Xs = 0;
                for (int g = 0; g < a.rank; ++g) {
                    Xs += (P * Cr + rec(g)[rec_DSUM(KS) + 2]) - P * m;
                    Cr += rec(g)[rec_DSUM(KS) + 1];
                }
                const double mloc = rec(a.rank)[rec_DSUM(KS) + 2] / P;
                const double scale = (a.dx * a.dx) / (double)a.M;
                a.scal[2] = scale * Xs;
                a.scal[3] = scale * ((Cr - m) + mloc);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// pass B: forward filter with carries, inverse row DFT, pin, back-projection, store
// ------------------------------------------------------------------------------------
// The pin value is the sum of the carry / pin kernels' per-workgroup parts (pinpart[0, npin)),
// in an order every pass B workgroup reproduces bit for bit.  pin_part() issues this thread's
// loads (parts t, t + T, ...; the buffer is zero-padded to PIN_PAD entries) at the top of the
// kernel; pin_total() folds them after the chunk set-up: a butterfly within the wave (both
// lanes of a pair form a + b == b + a, so every lane ends with the same bits), then the wave
// sums in wave order through LDS.  (A serial loop of dependent scalar loads here cost one
// memory round trip per eight parts in front of every workgroup's first row.)
constexpr int PIN_PAD = 1024;  // >= the widest pass B workgroup

template <int T>
__device__ __forceinline__ double pin_part(const SpecArgs &a, int t) {
    static_assert(T <= PIN_PAD, "pinpart padding");
    double p = a.pinpart[t];
    for (int b = t + T; b < a.npin; b += T) p += a.pinpart[b];
    return p;
}

template <int T>
__device__ __forceinline__ double pin_total(double p, double *pinw) {
    static_assert(T % 64 == 0, "whole waves");
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) p += __shfl_xor(p, m);
    if ((threadIdx.x & 63) == 0) pinw[threadIdx.x >> 6] = p;
    __syncthreads();
    double s = pinw[0];
#pragma unroll
    for (int w = 1; w < T / 64; ++w) s += pinw[w];
    // the same bits in every lane: keep it in scalar registers for the rows
    const unsigned long long u = (unsigned long long)__double_as_longlong(s);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ void chunk_carry(const SpecArgs &a, int s, int k, int c, double delta, bool inject,
                                            double2 &cu, double2 &w) {
    const size_t o = ((size_t)c * 2 + s) * a.KS + k;
    const Coef cf = a.coef[s * a.KS + k];
    const double2 Ue = a.EXT[(size_t)s * a.KS + k], We = a.EXT[(size_t)(2 + s) * a.KS + k];
    carry_in(a, cf, s, c, delta, inject, Ue, We, a.UIN[o], a.WIN[o], cu, w);
}

template <int N, class S>
__global__ __launch_bounds__(Geo<N>::T, Geo<N>::MINW) void spec_passB(SpecArgs a) {
    using US = typename Store<S>::C;
    using G = Geo<N>;
    constexpr int T = G::T, KQ = G::KQ, EP = G::EP, NH = N / 2;
    using Plan = FftPlan<N, T>;
    using Inv = FftFromLds<N, T, true, Plan::REG_OUT>;
    // N = 4096: the lane-exchange transform (see spec_passA): a thread's lines are k = g + q T
    // of its mirror group g; it forms Z_k and Z_(N-k) in registers q and 7 - q, the mirror
    // exchange gives every thread its whole group, and the inverse transform leaves the row in
    // the coalesced order of the stores (no LDS write of the spectrum)
    constexpr bool LX = N == lx::N && T == lx::T;
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = LX ? lds + N : (Plan::PINGPONG ? lds + LdsSize<N>::value : lds),
            *twl = LX ? lds + 2 * N : lds + (Plan::PINGPONG ? 2 : 1) * LdsSize<N>::value;
    double2 *stash = lds + 2 * N + 512;  // (LX: tw512 = twl, then the mirror stash)
    const double2 *Xb = Inv::result_in_b1 ? b1 : b0;
    // set-up loads (twiddles, the chunk's singular-line values, (r, 1/r) of k = N/2) go out
    // first and reach LDS just before pin_total's barrier (a serial head would put
    // one memory latency per load in front of the first row's loads)
    TwFill<N, T> twf;
    if constexpr (!LX) fft_twiddle_load<N, T>(twf, a.tw);
    double2 tw5 = make_double2(0, 0);
    if constexpr (LX) tw5 = a.tw[threadIdx.x];  // W^m, m < 512 (T = 512)
    const int t = threadIdx.x, c = blockIdx.x;
    const int g = LX ? lx::mirror_group(t) : t;  // lines k = g + q T
    const int L = a.L, s0 = c * L, e = s0 + L - 1;
    // the chunk's values of the singular line, staged once (a global load per row would sit
    // on every row's critical path, in front of the transform's barriers)
    __shared__ double lline[64];  // L <= 64 (pick_chunk)
    __shared__ double pinw[T / 64];
    // (r, 1/r) of the real line k = N/2, staged like lline: read in the row loop by the lane
    // that owns slot (0, 0), whose global load there would wait (in-order vmcnt) for the
    // next row's prefetch, and the whole workgroup for that wave at the next barrier
    __shared__ double2 crN[2];
    double llv = 0;
    double2 crv = make_double2(0, 0);
    if (a.pinned0 && t < L) llv = a.line[s0 + t];
    if (N < 4096 && t < 2) crv = QG_CRR(t * a.KS + NH);
    const double pinp = a.pinned0 ? pin_part<T>(a, t) : 0.0;  // (lline, twl: see pin_total)
    const int KS = a.KS;
    const int64_t Pl = a.P, ld = a.ld;
    const double delta = a.scal[0];
    const bool inject = a.pinned0 && a.rank == 0;
    const bool sing = a.pinned0;  // (s = 0, k = 0) is the singular line, served by a.line
    const double line0 = a.scal[2], line1 = a.scal[3];

    // register prefetch of the next row of u (in flight across this row's FFT).  Slot (0, t=0)
    // packs the real lines k = 0 (.x) and k = N/2 (.y).
    // (kept in the storage precision until used: converting F32 values right after the load
    // would make the load wait at once, so the prefetch would not be in flight at all)
    US upf[KQ][2];
    auto load_u = [&](int j) {
        const US *Urow = static_cast<const US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = g + q * T;
            if (NH % T == 0 || k < NH) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if constexpr (LX) {
                        upf[q][s] = Urow[s * KS + t + q * T];  // slot order (see spec_passA)
                    } else if (k == 0) {
                        upf[q][s].x = Urow[s * KS].x;
                        upf[q][s].y = Urow[s * KS + NH].x;
                    } else {
                        upf[q][s] = Urow[s * KS + k];
                    }
                }
            }
        }
    };
    constexpr bool PF = N < 8192;  // (N = 8192: no register prefetch, registers are short)
    if constexpr (PF) load_u(s0);  // first row in flight while the chunk carries are computed
    // per line: carried term cu = r^(e+1-j) u_in and forward-filter state w.  Slot (0, t = 0)
    // packs the real lines k = 0 (.x) and k = N/2 (.y).
    double2 cu[KQ][2], w[KQ][2];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const int k = g + q * T;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            cu[q][s] = make_double2(0, 0);
            w[q][s] = make_double2(0, 0);
            if (NH % T == 0 || k < NH) {
                if (k == 0) {
                    double2 c0 = make_double2(0, 0), w0 = make_double2(0, 0), cN, wN;
                    if (!(s == 0 && sing)) chunk_carry(a, s, 0, c, delta, inject, c0, w0);
                    chunk_carry(a, s, NH, c, delta, inject, cN, wN);
                    cu[q][s] = make_double2(c0.x, cN.x);
                    w[q][s] = make_double2(w0.x, wN.x);
                } else {
                    chunk_carry(a, s, k, c, delta, inject, cu[q][s], w[q][s]);
                }
            }
        }
    }
    // the recurrence coefficients (r, 1/r) of the next row, loaded after this row's transform
    // (not live across it) so their L2 latency hides behind the stores
    double2 crq[KQ][2];
    auto load_coef = [&]() {
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int k = g + q * T;
                if (NH % T == 0 || k < NH) crq[q][s] = LX ? a.scrr[s * KS + t + q * T] : QG_CRR(s * KS + k);
            }
    };
    load_coef();
#define QG_PB_R(q, s, o) crq[q][s]
    // folded after the chunk set-up, so the carries' loads are not queued behind the pin
    // parts' (folding first: 4096^2 pass B 125.9 -> 137.9 us); its barrier also publishes
    // lline and the twiddles
    if constexpr (LX) twl[t] = tw5;
    else fft_twiddle_store<N, T>(twl, twf);
    if (a.pinned0 && t < L) lline[t] = llv;
    if (N < 4096 && t < 2) crN[t] = crv;
    const double pin = pin_total<T>(pinp, pinw);
    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    for (int j = s0; j <= e; ++j) {
        if constexpr (!PF) load_u(j);
        double2 ucur[KQ][2];
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s) ucur[q][s] = d2(upf[q][s]);
        if (PF && j < e) load_u(j + 1);
        // compiler memory barrier: re-read the (L1-resident) coefficients every row instead of
        // hoisting them into registers, which would spill at this occupancy
        asm volatile("" ::: "memory");
        // LX: Z_k in register q, Z_(N-k) in register 7 - q (the partner lane's after the
        // exchange); thread 0 (group 0, its own partner) keeps Z_(512 (8 - q)) in register 8 - q
        // and Z_2048 in register 4
        double2 zr[8], zm[KQ];
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = g + q * T;
            if (NH % T == 0 || k < NH) {
                double2 X[2];
                if (k == 0) {
                    double x0[2], xN[2];
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o0 = s * KS, oN = s * KS + NH;
                        double ul0 = ucur[q][s].x, ulN = ucur[q][s].y;
                        if (s == 0 && inject && j == 0) {  // Poisson compatibility shift at row 0
                            ul0 += QG_CCS(o0) * delta;
                            ulN += QG_CCS(oN) * delta;
                        }
                        // (N = 4096: staged costs more spill than the wait: 130.3 vs 131.7 us)
                        const double2 r0 = QG_PB_R(q, s, o0), rN = N < 4096 ? crN[s] : QG_CRR(oN);
                        const double wx = r0.x * w[q][s].x + (ul0 + cu[q][s].x);
                        const double wy = rN.x * w[q][s].y + (ulN + cu[q][s].y);
                        w[q][s] = make_double2(wx, wy);
                        cu[q][s] = make_double2(cu[q][s].x * r0.y, cu[q][s].y * rN.y);
                        x0[s] = (s == 0 && sing) ? (line0 + (double)j * line1) + lline[j - s0] : wx;
                        xN[s] = wy;
                    }
                    if constexpr (LX) {
                        zr[q] = make_double2(x0[0], x0[1]);
                        zm[q] = make_double2(xN[0], xN[1]);
                    } else {
                        b0[0] = make_double2(x0[0], x0[1]);
                        b0[NH] = make_double2(xN[0], xN[1]);
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o = s * KS + k;
                        double2 ul = ucur[q][s];
                        if (s == 0 && inject && j == 0) ul.x += QG_CCS(o) * delta;
                        const double2 rr = QG_PB_R(q, s, o);
                        w[q][s] = cfma(rr.x, w[q][s], cadd(ul, cu[q][s]));
                        cu[q][s] = cscale(cu[q][s], rr.y);
                        X[s] = w[q][s];
                    }
                    const double2 zk = make_double2(X[0].x - X[1].y, X[0].y + X[1].x);
                    const double2 zn = make_double2(X[0].x + X[1].y, X[1].x - X[0].y);
                    if constexpr (LX) {
                        zr[q] = zk;
                        zm[q] = zn;
                    } else {
                        b0[k] = zk;
                        b0[N - k] = zn;
                    }
                }
            }
        }
        double2 xo[Plan::R_LAST];  // last FFT pass output in registers: element t + r*T
        if constexpr (LX) {
            static_assert(KQ == 4 && Plan::R_LAST == 8, "lane-exchange geometry");
            const bool t0 = t == 0;
            zr[4] = t0 ? zm[0] : zm[3];
            zr[5] = t0 ? zm[3] : zm[2];
            zr[6] = t0 ? zm[2] : zm[1];
            zr[7] = t0 ? zm[1] : zm[0];
            const int tt = opaque_tid();
            lx::mirror_exchange(zr, stash, tt);
            lx::fft<true, true, false>(zr, b0, b1, twl, tt);
#pragma unroll
            for (int p = 0; p < 8; ++p) xo[p] = zr[p];
        } else {
            __syncthreads();
            Inv::run(b0, b1, twl, xo);
        }
        S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
        S *row1 = out1 + (size_t)(j + 1) * ld;
        const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
        S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
        S *row2 = out2 ? out2 + (size_t)(j + 1) * ld : nullptr;
        S *grow2 = out2 ? ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows) : nullptr;
#pragma unroll
        for (int p = 0; p < EP; ++p) {
            const int i = t + p * T;
            if (N % T == 0 || i < N) {
                double2 z;
                if constexpr (Plan::REG_OUT) z = xo[p];
                else z = Xb[lay<Plan::LAST_NS>(i)];
                // the pinned unknown is exactly 0 (get_poisson_cholesky's identity row), not
                // its value minus the spectrally computed pin (a roundoff residue)
                const double x1 = (pin_row && i == 0) ? 0.0 : z.x - pin, x2 = z.y;
                store_row_with_ghosts(row1, grow1, N, i, (S)(a.pin_out[0] * x1 + a.pin_out[1] * x2));
                if (row2) store_row_with_ghosts(row2, grow2, N, i, (S)(a.pin_out[2] * x1 + a.pin_out[3] * x2));
            }
        }
        asm volatile("" ::: "memory");
        if (j < e) load_coef();
        if constexpr (!LX && Inv::b0_read_late) __syncthreads();  // the next row's recurrence writes b0
    }
#undef QG_PB_R
}

// ------------------------------------------------------------------------------------
// Wide rows (M = 8192).  Both systems' recurrence state (4 complex per wavenumber) plus a
// 8192-point transform do not fit in one CU's registers and LDS, so each workgroup serves ONE
// system of a chunk: its real row x (length M) is transformed as the half-length complex
// FFT of z_n = x_2n + i x_2n+1 (the 4096-point, 512-thread lane-exchange transform,
// qg_fft_lx.hpp) plus a split step X_k = E_k + W^k O_k, W = exp(-2 pi i / M).  The transform
// leaves a thread the elements g + 512 r of its mirror group g and, after the mirror exchange,
// the partner group's registers 4-7, so a thread's lines are
//   k_q = g + 512 q (q < 4),  k_q = (512 - g) + 512 q (q >= 4)     (thread 0: k_q = 512 q)
// and the split partner HN - k_q of line q is the thread's own line 7 - q: the split step of
// both passes runs in registers (no LDS round trip for the pairs).
// Pass A: one launch, workgroups (chunk, system) adjacent in XCD-aware order so the two
// readers of a row of zeta share an L2 and run side by side.  Pass B: two launches; system 0 leaves psi~1 rows in half_tmp
// (F64), system 1 combines them with psi~2 into the back-projection and the ghost ring.
// Recurrences, carries and the pin are the power-of-two passes' (same U / summary layout).
// ------------------------------------------------------------------------------------
constexpr int HN = 4096;           // half-length FFT
constexpr int HT = 512;            // threads per workgroup
constexpr int HK = HN / HT;        // wavenumber slots per thread (k_q above); slot (q 0, t 0)
                                   // packs the real lines k = 0 (.x) and k = HN (.y)
static_assert(HN == lx::N && HT == lx::T && HK == 8, "wide-row transform geometry");
// LDS: the transform's two row buffers, its twiddles and the mirror stash (lx::LDS_ELEMS).
// (The transforms stay F64 for F32 states too: computing pass A's in F32 saved
// 18 of 392 us at 8192^2 and pass B's 16 of 417, while the F32 error grew -- psi 2.3e-3 ->
// 5.3e-3 against the oracle at 8192 x 16, zeta 1e-4 -> 1e-3 on the smooth field with pass B's
// in F32 (r04e; qg_fft.hpp keeps the complex type a template parameter).)
constexpr size_t half_lds_bytes() { return sizeof(double2) * lx::LDS_ELEMS; }
struct HalfLds {
    double2 *b0, *b1, *tw512, *stash;
    __device__ explicit HalfLds(void *base) {
        b0 = static_cast<double2 *>(base);
        b1 = b0 + HN;
        tw512 = b1 + HN;
        stash = tw512 + 512;
    }
};
// line q of thread t (mirror group g, partner group gm = 512 - g; groups 0 and 256 are their
// own partners)
__device__ __forceinline__ int half_line(int g, int gm, int q) { return (q < HK / 2 ? g : gm) + q * HT; }
// The split step's W^k of line q, k = half_line(g, gm, q): W^(512 q) = exp(-2 pi i q / 16) is a
// constant of the unrolled line loop, so W^k = W^(g or gm) (two table entries per thread, loaded
// once) times it -- no per-row table reads (r04: 16 LDS reads per thread and row, as many as
// both of the transform's LDS transposes read)
__device__ __forceinline__ double2 half_tw_q(double2 wb, int q) {
    constexpr double C1 = 0.92387953251128674, S1 = 0.38268343236508978, H = 0.70710678118654752;
    switch (q & 7) {
    case 0: return wb;
    case 1: return cmul(wb, make_double2(C1, -S1));
    case 2: return cmul(wb, make_double2(H, -H));
    case 3: return cmul(wb, make_double2(S1, -C1));
    case 4: return make_double2(wb.y, -wb.x);  // (-i) wb
    case 5: return cmul(wb, make_double2(-S1, -C1));
    case 6: return cmul(wb, make_double2(-H, -H));
    default: return cmul(wb, make_double2(-C1, -S1));
    }
}

template <class S>
struct Pair;  // two adjacent row elements (8-byte / 4-byte alignment: rows start at element 1)
template <>
struct Pair<double> {
    typedef double V __attribute__((ext_vector_type(2), aligned(8)));
};
template <>
struct Pair<float> {
    typedef float V __attribute__((ext_vector_type(2), aligned(4)));
};

__device__ __forceinline__ void half_lds_init(const SpecArgs &a, double2 *tw512) {
    tw512[threadIdx.x] = a.tw2[threadIdx.x];  // W_4096^m, m < 512 (HT = 512)
}

template <class S>
__global__ __launch_bounds__(HT, 2) void spec_passA_half(SpecArgs a) {
    using US = typename Store<S>::C;
    using PV = typename Pair<S>::V;
    using CX = double2;
    extern __shared__ double2 lds[];
    const HalfLds hl(lds);
    double2 *b0 = hl.b0, *b1 = hl.b1, *tw512 = hl.tw512, *stash = hl.stash;
    half_lds_init(a, tw512);
    __syncthreads();
    // the two workgroups of a chunk read the same input rows: XCD-aware order puts them on
    // one XCD (one L2) side by side
    const int wg = xcd_logical_id();
    const int t = threadIdx.x, c = wg >> 1, s = wg & 1;
    const int g = lx::mirror_group(t), gm = g == 0 ? 0 : 512 - g;
    const double2 wg_tw = a.tw[g], wgm_tw = a.tw[gm];  // W^g, W^gm (see half_tw_q)
    const int s0 = c * a.L, e = s0 + a.L - 1;
    const int KS = a.KS;
    const int64_t ld = a.ld;
    const double pa = a.pin_in[2 * s], pb = a.pin_in[2 * s + 1];
    // bw = sum_j r^(e-j) u_j with the running weight om (see spec_passA): one r load per line
    double2 u[HK], bw[HK], om[HK];
#pragma unroll
    for (int q = 0; q < HK; ++q) {
        u[q] = bw[q] = make_double2(0, 0);
        om[q] = make_double2(1, 1);
    }
    double dc = 0;
    PV pf1[HK], pf2[HK];
    auto load_row = [&](int j, PV(&d1)[HK], PV(&d2)[HK]) {
        const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
        const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
#pragma unroll
        for (int p = 0; p < HK; ++p) {
            const int n = t + p * HT;
            d1[p] = *reinterpret_cast<const PV *>(r1 + 2 * n);
            d2[p] = *reinterpret_cast<const PV *>(r2 + 2 * n);
        }
    };
    const double *cr = a.cr + s * KS, *scr = a.scr + s * KS;
    const double csc = a.csc, csch = 0.5 * csc;
    // the drop-in lean mode (see spec_passA): system 0's workgroup also stores the input rows
    const bool zcopy = a.zcopy1 != nullptr && s == 0;
    auto copy_row = [&](int j, PV(&d1)[HK], PV(&d2)[HK]) {
        const int M = (int)a.M;
        auto put = [&](S *row, S *grow, int n, PV v) {  // elements 2n, 2n+1 and their ghost images
            *reinterpret_cast<PV *>(row + 1 + 2 * n) = v;
            if (n == 0) row[M + 1] = v.x;
            if (n == HN - 1) row[0] = v.y;
            if (grow) {
                *reinterpret_cast<PV *>(grow + 1 + 2 * n) = v;
                if (n == 0) grow[M + 1] = v.x;
                if (n == HN - 1) grow[0] = v.y;
            }
        };
        S *z1 = static_cast<S *>(a.zcopy1), *z2 = static_cast<S *>(a.zcopy2);
        S *g1 = ghost_row_target(z1, ld, a.P, j, true), *g2 = ghost_row_target(z2, ld, a.P, j, true);
#pragma unroll
        for (int p = 0; p < HK; ++p) {
            const int n = t + p * HT;
            put(z1 + (size_t)(j + 1) * ld, g1, n, d1[p]);
            put(z2 + (size_t)(j + 1) * ld, g2, n, d2[p]);
        }
    };
    // F32 states: r of this thread's lines loaded once -- row-invariant -- and held in
    // registers instead of re-read from L2 every row, where each row's loads queue behind the
    // next row's prefetch (vmcnt retires in order).  (F64 states: the 16 registers would spill.)
    constexpr bool RQ_HOIST = std::is_same<S, float>::value;
    double rq[HK];
    if constexpr (RQ_HOIST) {
#pragma unroll
        for (int q = 0; q < HK; ++q) rq[q] = scr[t + q * HT];
    }
    // one row: consume the prefetched row (c1, c2), refill them with row jn (< s0: none)
    auto row_step = [&](int j, PV(&c1)[HK], PV(&c2)[HK], int jn) {
        if constexpr (!RQ_HOIST) asm volatile("" ::: "memory");  // keep coefficient loads in the loop
        if (zcopy) copy_row(j, c1, c2);
        CX in[HK];
#pragma unroll
        for (int p = 0; p < HK; ++p)
            in[p] = make_double2(pa * (double)c1[p].x + pb * (double)c2[p].x,
                                 pa * (double)c1[p].y + pb * (double)c2[p].y);
        // the transform (the next row's loads issued once the first stage has left in[] in
        // LDS: fewer live registers than loading first) and the mirror exchange: in[q] =
        // Z_(k_q), in[7 - q] = Z_(HN - k_q)
        const int tt = opaque_tid();
        lx::fft<false, false, true>(in, b0, b1, tw512, tt, [&]() {
            if (jn >= s0) load_row(jn, c1, c2);
        });
        lx::mirror_exchange(in, stash, tt);
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS + (size_t)s * KS;
        double2 wb0 = wg_tw, wb1 = wgm_tw;
        asm volatile("" : "+v"(wb0.x), "+v"(wb0.y), "+v"(wb1.x), "+v"(wb1.y));  // W^k per row, not hoisted
#pragma unroll
        for (int q = 0; q < HK; ++q) {
            const int k = half_line(g, gm, q);
            const double2 Zk = in[q];
            if (k == 0) {  // X_0 = Re + Im, X_HN = Re - Im of Z_0 (both real)
                const double X0 = Zk.x + Zk.y, XN = Zk.x - Zk.y;
                if (s == 0) {
                    dc += X0;
                    a.hline[j] = X0;
                }
                const double r0 = cr[0], rN = cr[HN];
                u[q] = make_double2((r0 * csc) * X0 + r0 * u[q].x, (rN * csc) * XN + rN * u[q].y);
                st_u(Urow, Store<S>::c(u[q]));  // slot order: the pair packed in slot 0
                bw[q] = make_double2(om[q].x * u[q].x + bw[q].x, om[q].y * u[q].y + bw[q].y);
                om[q] = make_double2(om[q].x * r0, om[q].y * rN);
            } else {
                const double2 Zm = t == 0 ? in[(8 - q) & 7] : in[7 - q];  // Z_(HN - k)
                // E = (Z_k + conj Z_{HN-k}) / 2, O = (Z_k - conj Z_{HN-k}) / 2i, X = E + W^k O,
                // formed as 2E, 2O, 2X: the halves ride in the scale r (csc / 2), a power of
                // two, so u is bit for bit the halved form's
                const double2 E = make_double2(Zk.x + Zm.x, Zk.y - Zm.y);
                const double2 O = make_double2(Zk.y + Zm.y, Zm.x - Zk.x);
                const double2 X = cadd(E, cmul(half_tw_q(q < HK / 2 ? wb0 : wb1, q), O));
                const double r = RQ_HOIST ? rq[q] : scr[t + q * HT];
                u[q] = cfma(r, u[q], cscale(X, r * csch));
                st_u(Urow + t + q * HT, Store<S>::c(u[q]));
                bw[q] = cfma(om[q].x, u[q], bw[q]);
                om[q].x *= r;
            }
        }
    };
    load_row(e, pf1, pf2);
    for (int j = e; j >= s0; --j) row_step(j, pf1, pf2, j - 1);
#pragma unroll
    for (int q = 0; q < HK; ++q) {
        const int k = half_line(g, gm, q);
        const size_t o = ((size_t)c * 2 + s) * KS;
        if (k == 0) {
            a.ULS[o] = make_double2(u[q].x, 0);
            a.ULS[o + HN] = make_double2(u[q].y, 0);
            a.WLS[o] = make_double2(bw[q].x, 0);
            a.WLS[o + HN] = make_double2(bw[q].y, 0);
        } else {
            a.ULS[o + k] = u[q];
            a.WLS[o + k] = bw[q];
        }
    }
    if (t == 0 && s == 0) a.dcpart[c] = dc;
}

// SYS 0: psi~1 (pinned) -> half_tmp; SYS 1: psi~2, then psi = P_fwd (psi~1, psi~2) with ghosts
template <class S, int SYS>
__global__ __launch_bounds__(HT, 2) void spec_passB_half(SpecArgs a) {
    using US = typename Store<S>::C;
    using PV = typename Pair<S>::V;
    // half_tmp holds psi~1 in the state's precision (like u: F32 intermediates for F32 states)
    typedef S PD __attribute__((ext_vector_type(2)));  // half_tmp pair (aligned: rows of M)
    constexpr int s = SYS;
    using CX = double2;
    extern __shared__ double2 lds[];
    const HalfLds hl(lds);
    double2 *b0 = hl.b0, *b1 = hl.b1, *tw512 = hl.tw512, *stash = hl.stash;
    half_lds_init(a, tw512);
    const int t = threadIdx.x, c = blockIdx.x;
    const int g = lx::mirror_group(t), gm = g == 0 ? 0 : 512 - g;
    const double2 wg_tw = a.tw[g], wgm_tw = a.tw[gm];  // W^g, W^gm (see half_tw_q)
    const int L = a.L, s0 = c * L, e = s0 + L - 1;
    __shared__ double lline[64];  // L <= 64 (pick_chunk)
    __shared__ double pinw[HT / 64];
    __shared__ double2 crN;  // (r, 1/r) of the line k = M/2 (see spec_passB)
    const bool sing = s == 0 && a.pinned0;  // (s 0, k 0) is the singular line, served by a.line
    if (sing && t < L) lline[t] = a.line[s0 + t];
    if (t == 0) crN = a.crr[s * a.KS + HN];
    const double pinp = sing ? pin_part<HT>(a, t) : 0.0;  // (lline, twiddles: see pin_total)
    const int KS = a.KS;
    const int64_t Pl = a.P, ld = a.ld;
    const double delta = a.scal[0];
    const bool inject = a.pinned0 && a.rank == 0;
    const double line0 = a.scal[2], line1 = a.scal[3];
    const double2 *crr = a.crr + s * KS, *scrr = a.scrr + s * KS;
    const double *ccs = a.ccs + s * KS;

    US upf[HK];  // (storage precision until used: see spec_passB)
    auto load_u = [&](int j) {
        const US *Urow = static_cast<const US *>(a.U) + (size_t)j * 2 * KS + (size_t)s * KS;
#pragma unroll
        for (int q = 0; q < HK; ++q) upf[q] = Urow[t + q * HT];  // slot order (see spec_passA_half)
    };
    load_u(s0);
    // folded before the chunk set-up, whose registers are short here (the pin loads were
    // issued first, so the first row stays in flight); its barrier also publishes lline and
    // the LDS tables of half_lds_init
    const double pin = pin_total<HT>(pinp, pinw);
    if (s == 0 && blockIdx.x == 0 && t == 0) a.scal[1] = pin;  // (0 when not pinned)
    // stage 2's twiddle powers in SGPRs (lx::Stage2Tw) for B0 only: measured -4 us there, +2
    // in B1, +4 in the 4096-point pass B, +2 in the wide-row pass A (r05i, same box)
    std::conditional_t<SYS == 0, lx::Stage2Tw, lx::NoTw2> s2i{};
    if constexpr (SYS == 0) s2i = lx::stage2_powers<true>(a.tw2, t);
    double2 cu[HK], w[HK];
#pragma unroll
    for (int q = 0; q < HK; ++q) {
        const int k = half_line(g, gm, q);
        if (k == 0) {
            double2 c0 = make_double2(0, 0), w0 = make_double2(0, 0), cN, wN;
            if (!sing) chunk_carry(a, s, 0, c, delta, inject, c0, w0);
            chunk_carry(a, s, HN, c, delta, inject, cN, wN);
            cu[q] = make_double2(c0.x, cN.x);
            w[q] = make_double2(w0.x, wN.x);
        } else {
            chunk_carry(a, s, k, c, delta, inject, cu[q], w[q]);
        }
    }
    PD y1[HK];  // SYS 1: psi~1 at (2n, 2n+1), n = t + p*HT (loaded during the transform)
    auto load_y = [&](int j) {
        const S *yr = static_cast<const S *>(a.half_tmp) + (size_t)j * a.M;
#pragma unroll
        for (int p = 0; p < HK; ++p) y1[p] = *reinterpret_cast<const PD *>(yr + 2 * (t + p * HT));
    };
    // SYS 0: (r, 1/r) of the next row, loaded during this row (off the recurrence's critical
    // path; the tables do not fit in L1), as in spec_passB.  SYS 1 holds the system-0
    // rows in registers and would spill: it re-reads them at the recurrence (8192^2 F64:
    // B0 280 -> 244 us; B1 423 -> 542 us with the early loads)
    constexpr bool EARLY = SYS == 0;
    double2 crq[HK];
    auto load_coef = [&]() {
#pragma unroll
        for (int q = 0; q < HK; ++q) crq[q] = scrr[t + q * HT];
    };
    if constexpr (EARLY) load_coef();
    for (int j = s0; j <= e; ++j) {
        double2 ucur[HK];
#pragma unroll
        for (int q = 0; q < HK; ++q) ucur[q] = d2(upf[q]);
        asm volatile("" ::: "memory");  // keep coefficient loads in the loop
        double x0 = 0;  // slot (q 0, t 0): X_0 (.x of w, or the singular line)
#pragma unroll
        for (int q = 0; q < HK; ++q) {
            const int k = half_line(g, gm, q);
            if (k == 0) {
                double ul0 = ucur[q].x, ulN = ucur[q].y;
                if (s == 0 && inject && j == 0) {  // Poisson compatibility shift at row 0
                    ul0 += ccs[0] * delta;
                    ulN += ccs[HN] * delta;
                }
                const double2 r0 = EARLY ? crq[q] : crr[0], rN = crN;
                const double wx = r0.x * w[q].x + (ul0 + cu[q].x);
                const double wy = rN.x * w[q].y + (ulN + cu[q].y);
                w[q] = make_double2(wx, wy);
                cu[q] = make_double2(cu[q].x * r0.y, cu[q].y * rN.y);
                x0 = sing ? (line0 + (double)j * line1) + lline[j - s0] : wx;
            } else {
                double2 ul = ucur[q];
                if (s == 0 && inject && j == 0) ul.x += ccs[k] * delta;
                const double2 rr = EARLY ? crq[q] : scrr[t + q * HT];
                w[q] = cfma(rr.x, w[q], cadd(ul, cu[q]));
                cu[q] = cscale(cu[q], rr.y);
            }
        }
        // Z_k = (X_k + conj X_{HN-k}) + i W^-k (X_k - conj X_{HN-k}); z = IDFT(Z) = x_2n + i x_2n+1.
        // X_(HN - k_q) is this thread's line 7 - q (thread 0: line (8 - q) mod 8).  Z_(k_q) goes
        // to register q: for q >= 4 that is the partner group's register, which the mirror
        // exchange delivers.
        CX in[HK];
        double2 wb0 = wg_tw, wb1 = wgm_tw;
        asm volatile("" : "+v"(wb0.x), "+v"(wb0.y), "+v"(wb1.x), "+v"(wb1.y));  // W^k per row, not hoisted
#pragma unroll
        for (int q = 0; q < HK; ++q) {
            const int k = half_line(g, gm, q);
            if (k == 0) {
                in[q] = make_double2(x0 + w[q].y, x0 - w[q].y);
            } else {  // X_k = w[q]
                const double2 Xm = t == 0 ? w[(8 - q) & 7] : w[7 - q];
                const double2 A = make_double2(w[q].x + Xm.x, w[q].y - Xm.y);
                const double2 D = make_double2(w[q].x - Xm.x, w[q].y + Xm.y);
                const double2 B = cmul(cconj(half_tw_q(q < HK / 2 ? wb0 : wb1, q)), D);
                in[q] = make_double2(A.x - B.y, A.y + B.x);
            }
        }
        // the mirror exchange, then the transform (the next row's loads once the first stage
        // has left in[] in LDS); the output is element t + p HT of the row in register p, the
        // order of the stores below.  A row writes the LDS twice (the transform's two
        // transposes).
        const int tt = opaque_tid();
        lx::mirror_exchange(in, stash, tt);
        lx::fft<true, true, false>(in, b0, b1, tw512, tt, [&]() {
            if (j < e) load_u(j + 1);
            if constexpr (SYS == 1) load_y(j);
        }, s2i);
        const CX(&xo)[HK] = in;
        // SYS 0: the next row's (r, 1/r) before this row's stores -- vmcnt counts loads and
        // stores in order, so loaded after them the next recurrence waited for every store of
        // this row (8192^2 F32 B0: 187 -> 179 us; the 4096-point pass B, at its register
        // limit, spills and slows with the same move: 128.5 -> 145.4 us, r04c)
        if constexpr (EARLY) {
            if (j < e) load_coef();
        }
        if constexpr (SYS == 0) {
            S *yr = static_cast<S *>(a.half_tmp) + (size_t)j * a.M;
            const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
#pragma unroll
            for (int p = 0; p < HK; ++p) {
                const int n = t + p * HT;
                const double2 z = xo[p];
                PD v;
                // the pinned unknown is exactly 0 (get_poisson_cholesky's identity row)
                v.x = (S)((pin_row && n == 0) ? 0.0 : z.x - pin);
                v.y = (S)(z.y - pin);
                *reinterpret_cast<PD *>(yr + 2 * n) = v;
            }
        } else {
            S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
            S *row1 = out1 + (size_t)(j + 1) * ld;
            S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
            S *row2 = out2 ? out2 + (size_t)(j + 1) * ld : nullptr;
            S *grow2 = out2 ? ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows) : nullptr;
            const int M = (int)a.M;
            auto put = [&](S *row, S *grow, int n, PV v) {  // elements 2n, 2n+1 and their ghost images
                *reinterpret_cast<PV *>(row + 1 + 2 * n) = v;
                if (n == 0) row[M + 1] = v.x;
                if (n == HN - 1) row[0] = v.y;
                if (grow) {
                    *reinterpret_cast<PV *>(grow + 1 + 2 * n) = v;
                    if (n == 0) grow[M + 1] = v.x;
                    if (n == HN - 1) grow[0] = v.y;
                }
            };
#pragma unroll
            for (int p = 0; p < HK; ++p) {
                const int n = t + p * HT;
                const double2 z = xo[p];
                const double x1a = (double)y1[p].x, x1b = (double)y1[p].y;
                PV v1;
                v1.x = (S)(a.pin_out[0] * x1a + a.pin_out[1] * z.x);
                v1.y = (S)(a.pin_out[0] * x1b + a.pin_out[1] * z.y);
                put(row1, grow1, n, v1);
                if (row2) {
                    PV v2;
                    v2.x = (S)(a.pin_out[2] * x1a + a.pin_out[3] * z.x);
                    v2.y = (S)(a.pin_out[2] * x1b + a.pin_out[3] * z.y);
                    put(row2, grow2, n, v2);
                }
            }
        }
        // (no barrier: the transform's buffers are safe to reuse by the next row's, see
        // lx::fft)
    }
}

template <class S>
static int launch_half_t(bool passB, const SpecArgs &a, hipStream_t s) {
    const size_t lds = half_lds_bytes();
    if (passB) {
        QG_HIP(hipFuncSetAttribute((const void *)spec_passB_half<S, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        QG_HIP(hipFuncSetAttribute((const void *)spec_passB_half<S, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        spec_passB_half<S, 0><<<a.Nc, HT, lds, s>>>(a);
        QG_LAUNCH_CHECK();
        spec_passB_half<S, 1><<<a.Nc, HT, lds, s>>>(a);
    } else {
        QG_HIP(hipFuncSetAttribute((const void *)spec_passA_half<S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        spec_passA_half<S><<<2 * a.Nc, HT, lds, s>>>(a);
    }
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// ------------------------------------------------------------------------------------
// Generic rows (M not a power of two, M <= GEN_MMAX, odd or even): the same passes with the row
// transform as a run-time mixed-radix Stockham FFT in LDS (radices 8, 4, 2 and the odd primes
// up to 13, planned on the host), or, when M has a larger prime factor, a direct DFT (O(M^2)
// per row) -- for the reference's own grid sweeps (julia_bench_parts.jl:19, M = 8:8:128) and
// any other M.  Everything else (recurrences, chunk summaries, carries, pin, multi-rank
// closure) is the power-of-two code's, with the row length at run time.
// ------------------------------------------------------------------------------------
constexpr int GEN_T = 256;
constexpr int GEN_MMAX = 3200;                               // 3 row buffers of M complex in LDS
constexpr int GEN_KQ = (GEN_MMAX / 2 + GEN_T) / GEN_T;       // wavenumber slots per thread
constexpr int GEN_RMAX = 13;                                 // largest radix of a planned pass

// X_k = sum_x src[x] W^(k x), W = tw[1] (forward) or its conjugate (inverse)
template <bool INV>
__device__ __forceinline__ double2 dft_at(const double2 *src, const double2 *twl, int M, int k) {
    double2 acc = make_double2(0, 0);
    int m = 0;  // k x mod M
    for (int x = 0; x < M; ++x) {
        double2 w = twl[m];
        if (INV) w.y = -w.y;
        acc = cadd(acc, cmul(src[x], w));
        m += k;
        if (m >= M) m -= M;
    }
    return acc;
}

// One row transform by the planned passes a.rad[0..nrad): Stockham autosort between src and
// dst (one barrier per pass), twiddles and the radix-R DFT from the M-entry table twl
// (W^m = twl[m mod M], conjugated for the inverse).  Returns the buffer holding the result.
template <bool INV>
__device__ double2 *gen_fft(double2 *src, double2 *dst, const double2 *twl, const SpecArgs &a, int M) {
    const int t = threadIdx.x;
    int NS = 1;
    for (int p = 0; p < a.nrad; ++p) {
        const int R = a.rad[p], NB = M / R;
        const int tstep = M / (NS * R), rstep = NB;  // W_{NS R} = twl[tstep], W_R = twl[rstep]
        for (int b = t; b < NB; b += GEN_T) {
            const int k = b % NS;
            double2 v[GEN_RMAX];
#pragma unroll
            for (int r = 0; r < GEN_RMAX; ++r)
                if (r < R) v[r] = src[b + r * NB];
            if (NS > 1) {
                int m = 0;
                const int step = k * tstep;  // < M
#pragma unroll
                for (int r = 1; r < GEN_RMAX; ++r)
                    if (r < R) {
                        m += step;
                        if (m >= M) m -= M;
                        double2 w = twl[m];
                        if (INV) w.y = -w.y;
                        v[r] = cmul(v[r], w);
                    }
            }
            const int base = (b / NS) * NS * R + k;
            if (R == 8 || R == 4 || R == 2) {
                if (R == 8) {
                    double2 u[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) u[r] = v[r];
                    dft8<INV>(u);
#pragma unroll
                    for (int r = 0; r < 8; ++r) dst[base + r * NS] = u[r];
                } else if (R == 4) {
                    dft4<INV>(v[0], v[1], v[2], v[3]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) dst[base + r * NS] = v[r];
                } else {
                    dft2<INV>(v[0], v[1]);
                    dst[base] = v[0];
                    dst[base + NS] = v[1];
                }
            } else {  // odd prime radix: direct R-point DFT, W_R^(q r) from the table
#pragma unroll
                for (int q = 0; q < GEN_RMAX; ++q)
                    if (q < R) {
                        double2 acc = v[0];
                        int e = 0;  // q r mod R
#pragma unroll
                        for (int r = 1; r < GEN_RMAX; ++r)
                            if (r < R) {
                                e += q;
                                if (e >= R) e -= R;
                                double2 w = twl[e * rstep];
                                if (INV) w.y = -w.y;
                                acc = cadd(acc, cmul(v[r], w));
                            }
                        dst[base + q * NS] = acc;
                    }
            }
        }
        __syncthreads();
        double2 *x = src;
        src = dst;
        dst = x;
        NS *= R;
    }
    return src;
}

template <class S>
__global__ __launch_bounds__(GEN_T) void spec_passA_gen(SpecArgs a) {
    using US = typename Store<S>::C;
    constexpr int T = GEN_T, KQ = GEN_KQ;
    const int M = (int)a.M, NH = M / 2;
    // even M: slot k = 0 also carries the real line k = M/2; odd M: k = NH is a complex line
    const bool odd = M & 1;
    const int KC = odd ? NH + 1 : NH;  // slots k in [0, KC)
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + M, *twl = lds + 2 * M;
    const int t = threadIdx.x, c = blockIdx.x;
    for (int m = t; m < M; m += T) twl[m] = a.tw[m];
    const int s0 = c * a.L, e = s0 + a.L - 1;
    const int KS = a.KS;
    const int64_t ld = a.ld;
    double2 u[KQ][2], bw[KQ][2];
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            u[q][s] = make_double2(0, 0);
            bw[q][s] = make_double2(0, 0);
        }
    const double p0 = a.pin_in[0], p1 = a.pin_in[1], p2 = a.pin_in[2], p3 = a.pin_in[3];
    double dc = 0;
    for (int j = e; j >= s0; --j) {
        const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
        const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
        for (int i = t; i < M; i += T) {
            const double z1 = r1[i], z2 = r2[i];
            b0[i] = make_double2(p0 * z1 + p1 * z2, p2 * z1 + p3 * z2);
        }
        __syncthreads();
        const double2 *Zb = b1;
        if (a.nrad > 0) {
            Zb = gen_fft<false>(b0, b1, twl, a, M);
        } else {
            for (int k = t; k < M; k += T) b1[k] = dft_at<false>(b0, twl, M, k);
            __syncthreads();
        }
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = t + q * T;
            if (k < KC) {
                const double2 Zk = Zb[k];
                if (k == 0) {  // the two real lines k = 0 and k = M/2 (odd M: k = 0 only)
                    const double2 Zn = odd ? make_double2(0, 0) : Zb[NH];
                    dc += Zk.x;
                    a.hline[j] = Zk.x;
                    const double2 B[2] = {make_double2(Zk.x, Zn.x), make_double2(Zk.y, Zn.y)};
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o0 = s * KS, oN = s * KS + NH;
                        const double2 r0 = a.crr[o0], rN = a.crr[oN];
                        u[q][s] = make_double2(a.ccs[o0] * B[s].x + r0.x * u[q][s].x,
                                               a.ccs[oN] * B[s].y + rN.x * u[q][s].y);
                        Urow[s * KS] = Store<S>::c(make_double2(u[q][s].x, 0));
                        if (!odd) Urow[s * KS + NH] = Store<S>::c(make_double2(u[q][s].y, 0));
                        bw[q][s] = make_double2(bw[q][s].x * r0.y + u[q][s].x, bw[q][s].y * rN.y + u[q][s].y);
                    }
                } else {
                    const double2 Zm = Zb[M - k];
                    const double2 B[2] = {make_double2((Zk.x + Zm.x) * 0.5, (Zk.y - Zm.y) * 0.5),
                                          make_double2((Zk.y + Zm.y) * 0.5, (Zm.x - Zk.x) * 0.5)};
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o = s * KS + k;
                        const double2 rr = a.crr[o];
                        u[q][s] = cfma(rr.x, u[q][s], cscale(B[s], a.ccs[o]));
                        Urow[s * KS + k] = Store<S>::c(u[q][s]);
                        bw[q][s] = cfma(rr.y, bw[q][s], u[q][s]);
                    }
                }
            }
        }
        __syncthreads();  // the next row overwrites b0 / b1
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const int k = t + q * T;
        if (k < KC) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const size_t o = ((size_t)c * 2 + s) * KS;
                if (k == 0) {
                    const double q0 = a.coef[s * KS].qm1, qN = a.coef[s * KS + NH].qm1;
                    a.ULS[o] = make_double2(u[q][s].x, 0);
                    a.WLS[o] = make_double2(bw[q][s].x * q0, 0);
                    if (!odd) {
                        a.ULS[o + NH] = make_double2(u[q][s].y, 0);
                        a.WLS[o + NH] = make_double2(bw[q][s].y * qN, 0);
                    }
                } else {
                    a.ULS[o + k] = u[q][s];
                    a.WLS[o + k] = cscale(bw[q][s], a.coef[s * KS + k].qm1);
                }
            }
        }
    }
    if (t == 0) a.dcpart[c] = dc;
}

template <class S>
__global__ __launch_bounds__(GEN_T) void spec_passB_gen(SpecArgs a) {
    using US = typename Store<S>::C;
    constexpr int T = GEN_T, KQ = GEN_KQ;
    const int M = (int)a.M, NH = M / 2;
    const bool odd = M & 1;
    const int KC = odd ? NH + 1 : NH;  // (see spec_passA_gen)
    extern __shared__ double2 lds[];
    double2 *b0 = lds, *b1 = lds + M, *twl = lds + 2 * M;
    const int t = threadIdx.x, c = blockIdx.x;
    for (int m = t; m < M; m += T) twl[m] = a.tw[m];
    const int L = a.L, s0 = c * L, e = s0 + L - 1;
    __shared__ double lline[64];  // L <= 64 (pick_chunk)
    __shared__ double pinw[T / 64];
    if (a.pinned0 && t < L) lline[t] = a.line[s0 + t];
    const double pinp = a.pinned0 ? pin_part<T>(a, t) : 0.0;  // (lline, twl: see pin_total)
    const int KS = a.KS;
    const int64_t Pl = a.P, ld = a.ld;
    const double delta = a.scal[0];
    const bool inject = a.pinned0 && a.rank == 0;
    const bool sing = a.pinned0;
    const double line0 = a.scal[2], line1 = a.scal[3];
    double2 cu[KQ][2], w[KQ][2];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const int k = t + q * T;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            cu[q][s] = make_double2(0, 0);
            w[q][s] = make_double2(0, 0);
            if (k < KC) {
                if (k == 0) {
                    double2 c0 = make_double2(0, 0), w0 = make_double2(0, 0), cN = c0, wN = c0;
                    if (!(s == 0 && sing)) chunk_carry(a, s, 0, c, delta, inject, c0, w0);
                    if (!odd) chunk_carry(a, s, NH, c, delta, inject, cN, wN);
                    cu[q][s] = make_double2(c0.x, cN.x);
                    w[q][s] = make_double2(w0.x, wN.x);
                } else {
                    chunk_carry(a, s, k, c, delta, inject, cu[q][s], w[q][s]);
                }
            }
        }
    }
    // (its barrier also publishes lline and the twiddle table)
    const double pin = pin_total<T>(pinp, pinw);
    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    for (int j = s0; j <= e; ++j) {
        const US *Urow = static_cast<const US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            const int k = t + q * T;
            if (k < KC) {
                if (k == 0) {
                    double x0[2], xN[2];
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o0 = s * KS, oN = s * KS + NH;
                        double ul0 = d2(Urow[o0]).x, ulN = odd ? 0.0 : d2(Urow[oN]).x;
                        if (s == 0 && inject && j == 0) {  // Poisson compatibility shift at row 0
                            ul0 += a.ccs[o0] * delta;
                            ulN += a.ccs[oN] * delta;
                        }
                        const double2 r0 = a.crr[o0], rN = a.crr[oN];
                        const double wx = r0.x * w[q][s].x + (ul0 + cu[q][s].x);
                        const double wy = rN.x * w[q][s].y + (ulN + cu[q][s].y);
                        w[q][s] = make_double2(wx, wy);
                        cu[q][s] = make_double2(cu[q][s].x * r0.y, cu[q][s].y * rN.y);
                        x0[s] = (s == 0 && sing) ? (line0 + (double)j * line1) + lline[j - s0] : wx;
                        xN[s] = wy;
                    }
                    b0[0] = make_double2(x0[0], x0[1]);
                    if (!odd) b0[NH] = make_double2(xN[0], xN[1]);
                } else {
                    double2 X[2];
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int o = s * KS + k;
                        double2 ul = d2(Urow[o]);
                        if (s == 0 && inject && j == 0) ul.x += a.ccs[o] * delta;
                        const double2 rr = a.crr[o];
                        w[q][s] = cfma(rr.x, w[q][s], cadd(ul, cu[q][s]));
                        cu[q][s] = cscale(cu[q][s], rr.y);
                        X[s] = w[q][s];
                    }
                    b0[k] = make_double2(X[0].x - X[1].y, X[0].y + X[1].x);
                    b0[M - k] = make_double2(X[0].x + X[1].y, X[1].x - X[0].y);
                }
            }
        }
        __syncthreads();
        S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
        S *row1 = out1 + (size_t)(j + 1) * ld;
        const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
        S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
        S *row2 = out2 ? out2 + (size_t)(j + 1) * ld : nullptr;
        S *grow2 = out2 ? ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows) : nullptr;
        const double2 *Xb = a.nrad > 0 ? gen_fft<true>(b0, b1, twl, a, M) : nullptr;
        for (int i = t; i < M; i += T) {
            const double2 z = Xb ? Xb[i] : dft_at<true>(b0, twl, M, i);
            const double x1 = (pin_row && i == 0) ? 0.0 : z.x - pin, x2 = z.y;
            store_row_with_ghosts(row1, grow1, M, i, (S)(a.pin_out[0] * x1 + a.pin_out[1] * x2));
            if (row2) store_row_with_ghosts(row2, grow2, M, i, (S)(a.pin_out[2] * x1 + a.pin_out[3] * x2));
        }
        __syncthreads();  // the next row's recurrence writes b0
    }
}

// ------------------------------------------------------------------------------------
// Split passes: rows that are not a power of two and too wide for the generic passes
// (GEN_MMAX < M <= SPL_MMAX).  Three row buffers no longer fit in LDS, and the recurrence
// state of every wavenumber of a chunk no longer fits in one workgroup's registers, so the
// row transform and the y-recurrences become separate kernels:
//   spec_fft_split<fwd>: per row, project + M-point DFT in place in ONE LDS buffer (mixed-radix
//                        decimation-in-frequency stages, output in digit-reversed order, or a
//                        direct DFT for rows with a prime factor > 13), split into the two
//                        systems' spectra B_s(k), stored in U;
//   spec_passA_split:    one thread per (chunk, wavenumber): backward filter over the chunk's
//                        rows, u in place of B in U, chunk summaries (the generic pass A's
//                        arithmetic, in the same order);
//   spec_carry / spec_pin: unchanged;
//   spec_passB_split:    one thread per (chunk, wavenumber): carries, forward filter, X_s(k)
//                        in place of u in U (the generic pass B's arithmetic);
//   spec_fft_split<inv>: per row, rebuild the M-point spectrum from X_0, X_1, inverse DFT,
//                        pin, back-projection, store with ghosts.
// Twice the generic passes' traffic (U makes three round trips instead of one), but any
// M <= 8192 works: the capability path of laplacian.jl:60-75 (CHOLMOD factors any M x P).
// ------------------------------------------------------------------------------------
constexpr int SPL_T = 512;        // row-transform threads (256 VGPRs: a radix-13 butterfly + its roots)
constexpr int SPL_MMAX = 8192;    // one LDS buffer of M complex (128 KB)
constexpr int SPL_WMAX = 2 * SPL_MMAX;  // even rows up to here: one system at a time, half length
constexpr int SPL_KT = 256;       // recurrence kernels: wavenumbers per workgroup
// SPL_U_F64: the split pipeline keeps U in F64 for F32 states too.  Its U holds the raw row
// spectra F (and then u, X) between kernels; rounding F to F32 is a second F32 rounding of
// zeta~ whose gravest modes the solve amplifies by up to (L / 2 pi)^2 / dx^2 -- measured
// (r06, tools/r06/f32_solve_err.py): the F32 state's solve vs the F64 solve of the same zeta
// 3.4e-4 (5000 x 32), 6.1e-4 (16384 x 32), 4.1e-3 (20000 x 4: 69 000 eps_32), against
// 0.7 eps_32 in the fused passes, which store only the filtered u (no amplification).

// One decimation-in-frequency stage of radix R, in place: butterfly (block b, n) reads the R
// values n + m span of its block, does the R-point DFT, multiplies output q by W_Ls^(n q)
// (Ls = R span, the stage's sub-transform length) and writes it back to n + q span.  Every
// butterfly writes only the slots it read, so one barrier per stage and one butterfly's values
// in registers.  After all stages frequency k sits at perm[k] (mixed-radix digit reversal).
template <int R, bool INV>
__device__ void spl_stage(double2 *buf, const double2 *__restrict__ tw, int M, int span) {
    const int Ls = R * span, sc = M / Ls;  // W_Ls^e = tw[e sc]
    const int rstep = M / R;               // W_R^e = tw[e rstep]
    double2 wr[R];
    if constexpr (R != 2 && R != 4 && R != 8) {
#pragma unroll
        for (int e = 0; e < R; ++e) {
            wr[e] = tw[e * rstep];
            if (INV) wr[e].y = -wr[e].y;
        }
    }
    for (int b = threadIdx.x; b < M / R; b += SPL_T) {
        const int blk = b / span, n = b - blk * span;
        double2 *x = buf + (size_t)blk * Ls + n;
        double2 v[R];
#pragma unroll
        for (int m = 0; m < R; ++m) v[m] = x[m * span];
        if constexpr (R == 8) dft8<INV>(v);
        else if constexpr (R == 4) dft4<INV>(v[0], v[1], v[2], v[3]);
        else if constexpr (R == 2) dft2<INV>(v[0], v[1]);
        else {  // odd prime radix: direct R-point DFT
            double2 o[R];
#pragma unroll
            for (int q = 0; q < R; ++q) {
                double2 acc = v[0];
                int e = 0;
#pragma unroll
                for (int m = 1; m < R; ++m) {
                    e += q;
                    if (e >= R) e -= R;
                    acc = cadd(acc, cmul(v[m], wr[e]));
                }
                o[q] = acc;
            }
#pragma unroll
            for (int q = 0; q < R; ++q) v[q] = o[q];
        }
        x[0] = v[0];
        int e = 0;  // n q sc mod M
        const int step = n * sc;
#pragma unroll
        for (int q = 1; q < R; ++q) {
            e += step;
            if (e >= M) e -= M;
            double2 w = tw[e];
            if (INV) w.y = -w.y;
            x[q * span] = span > 1 ? cmul(v[q], w) : v[q];
        }
    }
    __syncthreads();
}

// the whole row transform in place (input synchronised in buf, natural order).  Planned rows:
// result synchronised in buf with frequency k at a.perm[k]; direct DFT: natural order.
// tw: the M-entry table of exp(-2 pi i m / M) (a.tw for the row length, a.tw2 for the
// half-length transforms of the wide split rows)
template <bool INV>
__device__ void spl_fft(double2 *buf, const SpecArgs &a, const double2 *tw, int M) {
    if (a.nrad == 0) {  // direct DFT: outputs to registers, then back in place
        constexpr int OUT = SPL_MMAX / SPL_T;
        double2 o[OUT];
#pragma unroll
        for (int q = 0; q < OUT; ++q) {
            const int k = threadIdx.x + q * SPL_T;
            if (k < M) o[q] = dft_at<INV>(buf, tw, M, k);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < OUT; ++q) {
            const int k = threadIdx.x + q * SPL_T;
            if (k < M) buf[k] = o[q];
        }
        __syncthreads();
        return;
    }
    int span = M;
    for (int p = 0; p < a.nrad; ++p) {
        const int R = a.rad[p];
        span /= R;
        switch (R) {
            case 2: spl_stage<2, INV>(buf, tw, M, span); break;
            case 3: spl_stage<3, INV>(buf, tw, M, span); break;
            case 4: spl_stage<4, INV>(buf, tw, M, span); break;
            case 5: spl_stage<5, INV>(buf, tw, M, span); break;
            case 7: spl_stage<7, INV>(buf, tw, M, span); break;
            case 8: spl_stage<8, INV>(buf, tw, M, span); break;
            case 11: spl_stage<11, INV>(buf, tw, M, span); break;
            default: spl_stage<13, INV>(buf, tw, M, span); break;
        }
    }
}

template <class S, bool INV>
__global__ __launch_bounds__(SPL_T) void spec_fft_split(SpecArgs a) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int M = (int)a.M, NH = M / 2, t = threadIdx.x;
    const bool odd = M & 1;
    const int KC = odd ? NH + 1 : NH;  // (see spec_passA_gen)
    const int KS = a.KS;
    const int64_t Pl = a.P, ld = a.ld;
    extern __shared__ double2 buf[];
    __shared__ double pinw[SPL_T / 64];
    double pin = 0;
    if constexpr (INV) {
        const double pinp = a.pinned0 ? pin_part<SPL_T>(a, t) : 0.0;
        pin = pin_total<SPL_T>(pinp, pinw);
        if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    }
    for (int64_t j = blockIdx.x; j < Pl; j += gridDim.x) {
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
        if constexpr (!INV) {
            const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
            const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
            const double p0 = a.pin_in[0], p1 = a.pin_in[1], p2 = a.pin_in[2], p3 = a.pin_in[3];
            for (int i = t; i < M; i += SPL_T) {
                const double z1 = r1[i], z2 = r2[i];
                buf[i] = make_double2(p0 * z1 + p1 * z2, p2 * z1 + p3 * z2);
            }
            __syncthreads();
            spl_fft<false>(buf, a, a.tw, M);
            auto Z = [&](int k) { return buf[a.nrad ? a.perm[k] : k]; };
            for (int k = t; k < KC; k += SPL_T) {
                const double2 Zk = Z(k);
                if (k == 0) {  // real lines k = 0 (and k = M/2 for even M)
                    Urow[0] = Store<double>::c(make_double2(Zk.x, 0));
                    Urow[KS] = Store<double>::c(make_double2(Zk.y, 0));
                    if (!odd) {
                        const double2 Zn = Z(NH);
                        Urow[NH] = Store<double>::c(make_double2(Zn.x, 0));
                        Urow[KS + NH] = Store<double>::c(make_double2(Zn.y, 0));
                    }
                } else {
                    const double2 Zm = Z(M - k);
                    Urow[k] = Store<double>::c(make_double2((Zk.x + Zm.x) * 0.5, (Zk.y - Zm.y) * 0.5));
                    Urow[KS + k] = Store<double>::c(make_double2((Zk.y + Zm.y) * 0.5, (Zm.x - Zk.x) * 0.5));
                }
            }
            __syncthreads();  // the next row overwrites buf
        } else {
            for (int k = t; k < KC; k += SPL_T) {
                if (k == 0) {
                    buf[0] = make_double2(d2(Urow[0]).x, d2(Urow[KS]).x);
                    if (!odd) buf[NH] = make_double2(d2(Urow[NH]).x, d2(Urow[KS + NH]).x);
                } else {
                    const double2 X0 = d2(Urow[k]), X1 = d2(Urow[KS + k]);
                    buf[k] = make_double2(X0.x - X1.y, X0.y + X1.x);
                    buf[M - k] = make_double2(X0.x + X1.y, X1.x - X0.y);
                }
            }
            __syncthreads();
            spl_fft<true>(buf, a, a.tw, M);
            S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
            S *row1 = out1 + (size_t)(j + 1) * ld;
            const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
            S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
            S *row2 = out2 ? out2 + (size_t)(j + 1) * ld : nullptr;
            S *grow2 = out2 ? ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows) : nullptr;
            for (int i = t; i < M; i += SPL_T) {
                const double2 z = buf[a.nrad ? a.perm[i] : i];
                const double x1 = (pin_row && i == 0) ? 0.0 : z.x - pin, x2 = z.y;
                store_row_with_ghosts(row1, grow1, M, i, (S)(a.pin_out[0] * x1 + a.pin_out[1] * x2));
                if (row2) store_row_with_ghosts(row2, grow2, M, i, (S)(a.pin_out[2] * x1 + a.pin_out[3] * x2));
            }
            __syncthreads();  // the next row overwrites buf
        }
    }
}

// Even rows wider than SPL_MMAX (up to SPL_WMAX = 16384): the M complex values of a row no
// longer fit in one LDS buffer, so each system's REAL row x is transformed on its own as the
// H = M/2-point complex transform of z_n = x_2n + i x_2n+1 (in place in H complex of LDS, the
// plan and twiddles of length H) plus a split step X_k = E_k + W^k O_k (E, O from Z_k and
// conj Z_{H-k}), as the wide-row passes do; the inverse rebuilds Z_k = (X_k + conj X_{H-k}) +
// i W^-k (X_k - conj X_{H-k}).  The inverse keeps system 0's values in registers while system
// 1 is transformed, then back-projects and stores both.  U, the recurrences, the carries and
// the closure are the split path's.  A capability path (the reference factors any M x P).
// POW2 (M = 16384): the half-length transform is the tuned 8192-point Stockham plan of the
// power-of-two passes, in place in one LDS buffer with its twiddles in LDS, natural order
// out; otherwise the planned mixed-radix DIF transform (global twiddles, digit-reversed out).
// (1024 threads: one radix-8 butterfly per thread and pass, and the inverse's held system-0
// values take 32 registers instead of 64: no spill at the 128-register cap)
constexpr int WIDE_T = 1024;
constexpr int WIDE_FT = 1024;  // forward transform threads (512 measured slower)
using WPlan = FftPlan<SPL_MMAX, WIDE_T>;
static_assert(!WPlan::PINGPONG && !FftPlan<SPL_MMAX, WIDE_FT>::PINGPONG, "the 8192-point plan runs in place");
static_assert(FftPlan<SPL_MMAX, WIDE_FT>::LDS == WPlan::LDS, "one LDS size for both directions");
template <class S, bool INV, bool POW2, int WT = POW2 ? (INV ? WIDE_T : WIDE_FT) : SPL_T>
__global__ __launch_bounds__(WT) void spec_fft_wide(SpecArgs a) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int M = POW2 ? 2 * SPL_MMAX : (int)a.M, H = M / 2, t = threadIdx.x;
    const int KS = a.KS;
    const int64_t Pl = a.P, ld = a.ld;
    const double2 *twM = a.tw, *twH = a.tw2;
    extern __shared__ double2 buf[];
    __shared__ double pinw[WT / 64];
    constexpr int PER = SPL_MMAX / WT;  // z values per thread (H <= SPL_MMAX)
    double2 *twl = buf + LdsSize<SPL_MMAX>::value;  // (POW2)
    auto Zat = [&](int k) {
        if constexpr (POW2) return buf[k];
        else return buf[a.nrad ? a.perm[k] : k];
    };
    auto xform = [&](auto inv) {
        constexpr bool I = decltype(inv)::value;
        if constexpr (POW2) {
            double2 unused[FftPlan<SPL_MMAX, WT>::R_LAST];
            FftFromLds<SPL_MMAX, WT, I, false>::run(buf, buf, twl, unused);
        } else {
            spl_fft<I>(buf, a, twH, H);
        }
    };
    if constexpr (POW2) fft_init_twiddles<SPL_MMAX, WT>(twl, twH);  // (published by the first row's barrier)
    double pin = 0;
    if constexpr (INV) {
        const double pinp = a.pinned0 ? pin_part<WT>(a, t) : 0.0;
        pin = pin_total<WT>(pinp, pinw);
        if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    }
    // POW2: the row's raw values (x1[2n], x1[2n+1], x2[2n], x2[2n+1], n = t + p WT) are loaded
    // once for both systems (a next-row prefetch spilled at the 1024-thread register cap)
    constexpr bool RAW = POW2 && !INV;
    S raw[RAW ? PER : 1][4];
    auto load_raw = [&](int64_t j, S (&d)[RAW ? PER : 1][4]) {
        if constexpr (RAW) {
            const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
            const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
#pragma unroll
            for (int p = 0; p < PER; ++p) {
                const int n = t + p * WT;
                d[p][0] = r1[2 * n];
                d[p][1] = r1[2 * n + 1];
                d[p][2] = r2[2 * n];
                d[p][3] = r2[2 * n + 1];
            }
        }
    };
    for (int64_t j = blockIdx.x; j < Pl; j += gridDim.x) {
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
        if constexpr (!INV) {
            const S *r1 = static_cast<const S *>(a.in1) + fidx(1, j + 1, ld);
            const S *r2 = static_cast<const S *>(a.in2) + fidx(1, j + 1, ld);
            if constexpr (RAW) load_raw(j, raw);
#pragma unroll 1
            for (int s = 0; s < 2; ++s) {
                const double pa = a.pin_in[2 * s], pb = a.pin_in[2 * s + 1];
                if constexpr (RAW) {
#pragma unroll
                    for (int p = 0; p < PER; ++p)
                        buf[t + p * WT] = make_double2(pa * (double)raw[p][0] + pb * (double)raw[p][2],
                                                       pa * (double)raw[p][1] + pb * (double)raw[p][3]);
                } else {
                    for (int n = t; n < H; n += WT) {
                        const double xa = pa * (double)r1[2 * n] + pb * (double)r2[2 * n];
                        const double xb = pa * (double)r1[2 * n + 1] + pb * (double)r2[2 * n + 1];
                        buf[n] = make_double2(xa, xb);
                    }
                }
                __syncthreads();
                xform(std::false_type{});
                US *Us = Urow + (size_t)s * KS;
                for (int k = t; k < H; k += WT) {
                    const double2 Zk = Zat(k);
                    if (k == 0) {  // X_0 = Re + Im, X_H = Re - Im (both real)
                        Us[0] = Store<double>::c(make_double2(Zk.x + Zk.y, 0));
                        Us[H] = Store<double>::c(make_double2(Zk.x - Zk.y, 0));
                    } else {
                        const double2 Zm = Zat(H - k);
                        const double2 E = make_double2((Zk.x + Zm.x) * 0.5, (Zk.y - Zm.y) * 0.5);
                        const double2 O = make_double2((Zk.y + Zm.y) * 0.5, (Zm.x - Zk.x) * 0.5);
                        Us[k] = Store<double>::c(cadd(E, cmul(twM[k], O)));
                    }
                }
                __syncthreads();  // the next transform overwrites buf
            }
        } else {
            double2 z1[PER];  // system 0's z_n (n = t + p WT), pin applied
#pragma unroll 1
            for (int s = 0; s < 2; ++s) {
                const US *Us = Urow + (size_t)s * KS;
                for (int k = t; k < H; k += WT) {
                    if (k == 0) {
                        const double X0 = d2(Us[0]).x, XH = d2(Us[H]).x;
                        buf[0] = make_double2(X0 + XH, X0 - XH);
                    } else {
                        const double2 Xk = d2(Us[k]), Xm = d2(Us[H - k]);
                        const double2 A = make_double2(Xk.x + Xm.x, Xk.y - Xm.y);
                        const double2 D = make_double2(Xk.x - Xm.x, Xk.y + Xm.y);
                        const double2 B = cmul(cconj(twM[k]), D);
                        buf[k] = make_double2(A.x - B.y, A.y + B.x);
                    }
                }
                __syncthreads();
                xform(std::true_type{});
                if (s == 0) {
                    const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
#pragma unroll
                    for (int p = 0; p < PER; ++p) {
                        const int n = t + p * WT;
                        if (n < H) {
                            const double2 z = Zat(n);
                            // the pinned unknown is exactly 0 (see spec_passB)
                            z1[p] = make_double2((pin_row && n == 0) ? 0.0 : z.x - pin, z.y - pin);
                        }
                    }
                    __syncthreads();  // system 1 overwrites buf
                } else {
                    S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
                    S *row1 = out1 + (size_t)(j + 1) * ld;
                    S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
                    S *row2 = out2 ? out2 + (size_t)(j + 1) * ld : nullptr;
                    S *grow2 = out2 ? ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows) : nullptr;
#pragma unroll
                    for (int p = 0; p < PER; ++p) {
                        const int n = t + p * WT;
                        if (n < H) {
                            const double2 z2 = Zat(n);
                            const double x1a = z1[p].x, x1b = z1[p].y;
                            store_row_with_ghosts(row1, grow1, M, 2 * n, (S)(a.pin_out[0] * x1a + a.pin_out[1] * z2.x));
                            store_row_with_ghosts(row1, grow1, M, 2 * n + 1, (S)(a.pin_out[0] * x1b + a.pin_out[1] * z2.y));
                            if (row2) {
                                store_row_with_ghosts(row2, grow2, M, 2 * n, (S)(a.pin_out[2] * x1a + a.pin_out[3] * z2.x));
                                store_row_with_ghosts(row2, grow2, M, 2 * n + 1,
                                                      (S)(a.pin_out[2] * x1b + a.pin_out[3] * z2.y));
                            }
                        }
                    }
                    __syncthreads();  // the next row overwrites buf
                }
            }
        }
    }
}

// lines k of (chunk blockIdx.x): the generic pass A's backward filter and summaries
template <class S>
__global__ __launch_bounds__(SPL_KT) void spec_passA_split(SpecArgs a) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int c = blockIdx.x, k = blockIdx.y * SPL_KT + threadIdx.x;
    if (k >= a.KH) return;
    const int KS = a.KS, s0 = c * a.L, e = s0 + a.L - 1;
    double2 u[2] = {make_double2(0, 0), make_double2(0, 0)}, bw[2] = {u[0], u[1]};
    double2 rr[2];
    double cs[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        rr[s] = a.crr[s * KS + k];
        cs[s] = a.ccs[s * KS + k];
    }
    double dc = 0;
    for (int j = e; j >= s0; --j) {
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const double2 B = d2(Urow[s * KS + k]);
            if (s == 0 && k == 0) {
                dc += B.x;
                a.hline[j] = B.x;
            }
            u[s] = cfma(rr[s].x, u[s], cscale(B, cs[s]));
            Urow[s * KS + k] = Store<double>::c(u[s]);
            bw[s] = cfma(rr[s].y, bw[s], u[s]);
        }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const size_t o = ((size_t)c * 2 + s) * KS + k;
        a.ULS[o] = u[s];
        a.WLS[o] = cscale(bw[s], a.coef[s * KS + k].qm1);
    }
    if (k == 0) a.dcpart[c] = dc;
}

// lines k of (chunk blockIdx.x): carries, the generic pass B's forward filter, X in place
template <class S>
__global__ __launch_bounds__(SPL_KT) void spec_passB_split(SpecArgs a) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int c = blockIdx.x, k = blockIdx.y * SPL_KT + threadIdx.x;
    if (k >= a.KH) return;
    const int KS = a.KS, L = a.L, s0 = c * L, e = s0 + L - 1;
    const double delta = a.scal[0];
    const bool inject = a.pinned0 && a.rank == 0;
    const bool sing = a.pinned0 && k == 0;  // (s = 0, k = 0): the singular line, from a.line
    const double line0 = a.scal[2], line1 = a.scal[3];
    double2 cu[2], w[2], rr[2];
    double cs[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        cu[s] = w[s] = make_double2(0, 0);
        if (!(s == 0 && sing)) chunk_carry(a, s, k, c, delta, inject, cu[s], w[s]);
        rr[s] = a.crr[s * KS + k];
        cs[s] = a.ccs[s * KS + k];
    }
    for (int j = s0; j <= e; ++j) {
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            double2 ul = d2(Urow[s * KS + k]);
            if (s == 0 && inject && j == 0) ul.x += cs[s] * delta;  // Poisson compatibility shift
            w[s] = cfma(rr[s].x, w[s], cadd(ul, cu[s]));
            cu[s] = cscale(cu[s], rr[s].y);
            const double2 X = (s == 0 && sing) ? make_double2((line0 + (double)j * line1) + a.line[j], 0) : w[s];
            Urow[s * KS + k] = Store<double>::c(X);
        }
    }
}

// ------------------------------------------------------------------------------------
// Bluestein rows: any row length the transforms above do not take (odd M > 8192, M > 16384),
// as the reference's CHOLMOD factors any M x P (laplacian.jl:60-75).  The M-point DFT of a
// row is a chirp-z convolution (nk = (n^2 + k^2 - (k - n)^2) / 2):
//   X_k = c_k sum_n (x_n c_n) b_(k-n),   c_n = exp(-pi i n^2 / M),  b_m = exp(+pi i m^2 / M),
// evaluated cyclically with power-of-two FFTs of length L >= 2M - 1 (the filter's transform
// is a host table); the inverse DFT is the conjugate of the forward DFT of the conjugate.  The
// transforms are Stockham passes in global memory (radix 8, then 4 / 2), over batches of
// rows.  The spectra feed the split pipeline's recurrence kernels (spec_passA_split /
// spec_passB_split): the same U contract as spec_fft_split.  A capability path, exact to
// roundoff.
// ------------------------------------------------------------------------------------
constexpr int BL_T = 256;
constexpr int64_t BL_MMAX = 1 << 18;           // rows up to 262144 points (L <= 2^19)
constexpr size_t BL_BUF_BYTES = (size_t)1 << 28;  // per ping-pong buffer (rows per batch)

template <int R, bool INV>
__global__ __launch_bounds__(BL_T) void bl_pass(const double2 *__restrict__ src, double2 *__restrict__ dst,
                                                const double2 *__restrict__ tw, int L, int NS, int rows) {
    const int NB = L / R;
    const int64_t total = (int64_t)rows * NB;
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T) {
        const int row = (int)(gi / NB), j = (int)(gi - (int64_t)row * NB);
        const double2 *x = src + (size_t)row * L;
        double2 *y = dst + (size_t)row * L;
        const int k = j % NS;
        double2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = x[j + r * NB];
        if (NS > 1) {  // W_(NS R)^(r k) = W_L^(r k L / (NS R)), exact table entries (< L)
            const int step = k * (L / (NS * R));
            int e = 0;
#pragma unroll
            for (int r = 1; r < R; ++r) {
                e += step;
                double2 w = tw[e];
                if (INV) w.y = -w.y;
                v[r] = cmul(v[r], w);
            }
        }
        dftR<R, INV>(v);
        const int base = (j / NS) * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) y[base + r * NS] = v[r];
    }
}

__global__ __launch_bounds__(BL_T) void bl_mul(double2 *x, const double2 *__restrict__ bhat, int L, int rows) {
    const int64_t total = (int64_t)rows * L;
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T)
        x[gi] = cmul(x[gi], bhat[gi % L]);
}

// rows [r0, r0 + rows): A_n = z_n c_n (n < M), 0 beyond; z = the projected pair of inputs
template <class S>
__global__ __launch_bounds__(BL_T) void bl_load_fwd(SpecArgs a, int64_t r0, int rows, double2 *A) {
    const int M = (int)a.M, L = a.bl_L;
    const int64_t total = (int64_t)rows * L, ld = a.ld;
    const double p0 = a.pin_in[0], p1 = a.pin_in[1], p2 = a.pin_in[2], p3 = a.pin_in[3];
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T) {
        const int64_t r = gi / L, j = r0 + r;
        const int n = (int)(gi - r * L);
        double2 v = make_double2(0, 0);
        if (n < M) {
            const double z1 = static_cast<const S *>(a.in1)[fidx(1 + n, j + 1, ld)];
            const double z2 = static_cast<const S *>(a.in2)[fidx(1 + n, j + 1, ld)];
            v = cmul(make_double2(p0 * z1 + p1 * z2, p2 * z1 + p3 * z2), a.bl_chirp[n]);
        }
        A[gi] = v;
    }
}

// Z_k = c_k Y_k, split into the two systems' spectra B_s(k) in U (spec_fft_split's forward)
template <class S>
__global__ __launch_bounds__(BL_T) void bl_store_fwd(SpecArgs a, int64_t r0, int rows, const double2 *Y) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int M = (int)a.M, NH = M / 2, L = a.bl_L, KS = a.KS;
    const bool odd = M & 1;
    const int KC = odd ? NH + 1 : NH;
    const int64_t total = (int64_t)rows * KC;
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T) {
        const int64_t r = gi / KC, j = r0 + r;
        const int k = (int)(gi - r * KC);
        const double2 *y = Y + (size_t)r * L;
        US *Urow = static_cast<US *>(a.U) + (size_t)j * 2 * KS;
        auto Z = [&](int q) { return cmul(a.bl_chirp[q], y[q]); };
        const double2 Zk = Z(k);
        if (k == 0) {  // real lines k = 0 (and k = M/2 for even M)
            Urow[0] = Store<double>::c(make_double2(Zk.x, 0));
            Urow[KS] = Store<double>::c(make_double2(Zk.y, 0));
            if (!odd) {
                const double2 Zn = Z(NH);
                Urow[NH] = Store<double>::c(make_double2(Zn.x, 0));
                Urow[KS + NH] = Store<double>::c(make_double2(Zn.y, 0));
            }
        } else {
            const double2 Zm = Z(M - k);
            Urow[k] = Store<double>::c(make_double2((Zk.x + Zm.x) * 0.5, (Zk.y - Zm.y) * 0.5));
            Urow[KS + k] = Store<double>::c(make_double2((Zk.y + Zm.y) * 0.5, (Zm.x - Zk.x) * 0.5));
        }
    }
}

// inverse, first half: rebuild Z from the systems' X in U (spec_fft_split's inverse) and load
// A_n = conj(Z_n) c_n, 0 beyond M
template <class S>
__global__ __launch_bounds__(BL_T) void bl_load_inv(SpecArgs a, int64_t r0, int rows, double2 *A) {
    using US = double2;  // (F64 whatever the state: see SPL_U_F64)
    const int M = (int)a.M, NH = M / 2, L = a.bl_L, KS = a.KS;
    const bool odd = M & 1;
    const int KC = odd ? NH + 1 : NH;
    const int64_t total = (int64_t)rows * KC;
    auto put = [&](double2 *x, int n, double2 z) { x[n] = cmul(cconj(z), a.bl_chirp[n]); };
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T) {
        const int64_t r = gi / KC, j = r0 + r;
        const int k = (int)(gi - r * KC);
        const US *Urow = static_cast<const US *>(a.U) + (size_t)j * 2 * KS;
        double2 *x = A + (size_t)r * L;
        if (k == 0) {
            put(x, 0, make_double2(d2(Urow[0]).x, d2(Urow[KS]).x));
            if (!odd) put(x, NH, make_double2(d2(Urow[NH]).x, d2(Urow[KS + NH]).x));
        } else {
            const double2 X0 = d2(Urow[k]), X1 = d2(Urow[KS + k]);
            put(x, k, make_double2(X0.x - X1.y, X0.y + X1.x));
            put(x, M - k, make_double2(X0.x + X1.y, X1.x - X0.y));
        }
    }
    const int64_t tail = (int64_t)rows * (L - M);
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < tail; gi += (int64_t)gridDim.x * BL_T) {
        const int64_t r = gi / (L - M);
        A[(size_t)r * L + M + (gi - r * (L - M))] = make_double2(0, 0);
    }
}

// inverse, second half: z_n = conj(c_n Y_n); pin, back-projection, store with the ghost ring
// (spec_fft_split's inverse)
template <class S>
__global__ __launch_bounds__(BL_T) void bl_store_inv(SpecArgs a, int64_t r0, int rows, const double2 *Y) {
    const int M = (int)a.M, L = a.bl_L;
    const int64_t Pl = a.P, ld = a.ld;
    __shared__ double pinw[BL_T / 64];
    const double pinp = a.pinned0 ? pin_part<BL_T>(a, threadIdx.x) : 0.0;
    const double pin = pin_total<BL_T>(pinp, pinw);
    if (blockIdx.x == 0 && threadIdx.x == 0 && r0 == 0) a.scal[1] = pin;
    const int64_t total = (int64_t)rows * M;
    S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
    for (int64_t gi = (int64_t)blockIdx.x * BL_T + threadIdx.x; gi < total; gi += (int64_t)gridDim.x * BL_T) {
        const int64_t r = gi / M, j = r0 + r;
        const int i = (int)(gi - r * M);
        const double2 z = cconj(cmul(a.bl_chirp[i], Y[(size_t)r * L + i]));
        const bool pin_row = a.pinned0 && a.rank == 0 && j == 0;
        S *row1 = out1 + (size_t)(j + 1) * ld;
        S *grow1 = ghost_row_target(out1, ld, Pl, j, a.write_ghost_rows);
        const double x1 = (pin_row && i == 0) ? 0.0 : z.x - pin, x2 = z.y;
        store_row_with_ghosts(row1, grow1, M, i, (S)(a.pin_out[0] * x1 + a.pin_out[1] * x2));
        if (out2) {
            S *row2 = out2 + (size_t)(j + 1) * ld;
            S *grow2 = ghost_row_target(out2, ld, Pl, j, a.write_ghost_rows);
            store_row_with_ghosts(row2, grow2, M, i, (S)(a.pin_out[2] * x1 + a.pin_out[3] * x2));
        }
    }
}

static unsigned bl_grid(int64_t work) {
    return (unsigned)std::min<int64_t>((work + BL_T - 1) / BL_T, 2048);
}

// length-L transforms of `rows` rows: x (input, natural order) -> the returned buffer
template <bool INV>
static int bl_fft(const SpecArgs &a, double2 *x, double2 *other, int rows, hipStream_t s, double2 **out) {
    const int L = a.bl_L;
    double2 *src = x, *dst = other;
    for (int NS = 1; NS < L;) {
        const int rem = L / NS, R = rem % 8 == 0 ? 8 : (rem % 4 == 0 ? 4 : 2);
        const unsigned g = bl_grid((int64_t)rows * (L / R));
        if (R == 8) bl_pass<8, INV><<<g, BL_T, 0, s>>>(src, dst, a.bl_tw, L, NS, rows);
        else if (R == 4) bl_pass<4, INV><<<g, BL_T, 0, s>>>(src, dst, a.bl_tw, L, NS, rows);
        else bl_pass<2, INV><<<g, BL_T, 0, s>>>(src, dst, a.bl_tw, L, NS, rows);
        QG_LAUNCH_CHECK();
        std::swap(src, dst);
        NS *= R;
    }
    *out = src;
    return QG_OK;
}

// the row transforms of every row, forward (rows -> U) or inverse (U -> rows)
template <class S>
static int bl_rows(bool inv, const SpecArgs &a, hipStream_t s) {
    const int L = a.bl_L;
    for (int64_t r0 = 0; r0 < a.P; r0 += a.bl_rows) {
        const int rows = (int)std::min<int64_t>(a.bl_rows, a.P - r0);
        double2 *y = nullptr, *z = nullptr;
        if (!inv) bl_load_fwd<S><<<bl_grid((int64_t)rows * L), BL_T, 0, s>>>(a, r0, rows, a.bl_buf0);
        else bl_load_inv<S><<<bl_grid((int64_t)rows * L), BL_T, 0, s>>>(a, r0, rows, a.bl_buf0);
        QG_LAUNCH_CHECK();
        QG_CHECK(bl_fft<false>(a, a.bl_buf0, a.bl_buf1, rows, s, &y));
        bl_mul<<<bl_grid((int64_t)rows * L), BL_T, 0, s>>>(y, a.bl_bhat, L, rows);
        QG_LAUNCH_CHECK();
        QG_CHECK(bl_fft<true>(a, y, y == a.bl_buf0 ? a.bl_buf1 : a.bl_buf0, rows, s, &z));
        if (!inv) bl_store_fwd<S><<<bl_grid((int64_t)rows * (a.M / 2 + 1)), BL_T, 0, s>>>(a, r0, rows, z);
        else bl_store_inv<S><<<bl_grid((int64_t)rows * a.M), BL_T, 0, s>>>(a, r0, rows, z);
        QG_LAUNCH_CHECK();
    }
    return QG_OK;
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
template <int N, class S>
static int launch_pass_t(bool passB, const SpecArgs &a, hipStream_t s) {
    constexpr bool LX = N == lx::N && Geo<N>::T == lx::T;  // (the lane-exchange transform)
    const size_t lds = sizeof(double2) * (LX ? (size_t)lx::LDS_ELEMS : (size_t)FftPlan<N, Geo<N>::T>::LDS);
    if (passB) {
        QG_HIP(hipFuncSetAttribute((const void *)spec_passB<N, S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        spec_passB<N, S><<<a.Nc, Geo<N>::T, lds, s>>>(a);
    } else {
        QG_HIP(hipFuncSetAttribute((const void *)spec_passA<N, S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        spec_passA<N, S><<<a.Nc, Geo<N>::T, lds, s>>>(a);
    }
    QG_LAUNCH_CHECK();
    return QG_OK;
}

template <int N>
static int launch_pass(bool passB, const SpecArgs &a, hipStream_t s) {
    return a.f32 ? launch_pass_t<N, float>(passB, a, s) : launch_pass_t<N, double>(passB, a, s);
}

static int dispatch_pass(bool passB, const SpecArgs &a, hipStream_t s) {
    switch (a.M) {
        case 8: return launch_pass<8>(passB, a, s);
        case 16: return launch_pass<16>(passB, a, s);
        case 32: return launch_pass<32>(passB, a, s);
        case 64: return launch_pass<64>(passB, a, s);
        case 128: return launch_pass<128>(passB, a, s);
        case 256: return launch_pass<256>(passB, a, s);
        case 512: return launch_pass<512>(passB, a, s);
        case 1024: return launch_pass<1024>(passB, a, s);
        case 2048: return launch_pass<2048>(passB, a, s);
        case 4096: return launch_pass<4096>(passB, a, s);
        case 8192: return a.f32 ? launch_half_t<float>(passB, a, s) : launch_half_t<double>(passB, a, s);
        default: break;
    }
    if (a.bl_L) {  // Bluestein rows: their transforms around the split pipeline's recurrences
        const dim3 rgrid((unsigned)a.Nc, (unsigned)((a.KH + SPL_KT - 1) / SPL_KT));
        if (!passB) {
            QG_CHECK(a.f32 ? bl_rows<float>(false, a, s) : bl_rows<double>(false, a, s));
            if (a.f32) spec_passA_split<float><<<rgrid, SPL_KT, 0, s>>>(a);
            else spec_passA_split<double><<<rgrid, SPL_KT, 0, s>>>(a);
            QG_LAUNCH_CHECK();
        } else {
            if (a.f32) spec_passB_split<float><<<rgrid, SPL_KT, 0, s>>>(a);
            else spec_passB_split<double><<<rgrid, SPL_KT, 0, s>>>(a);
            QG_LAUNCH_CHECK();
            QG_CHECK(a.f32 ? bl_rows<float>(true, a, s) : bl_rows<double>(true, a, s));
        }
        return QG_OK;
    }
    // (qg_set_form(QG_FORM_ROW_SPLIT, 1): generic-size rows through the split passes too)
    if (a.M > GEN_MMAX || form(QG_FORM_ROW_SPLIT)) {
        if (a.M > SPL_WMAX || (a.M > SPL_MMAX && a.M % 2 != 0)) return QG_ERR_UNSUPPORTED;
        const bool wsplit = a.M > SPL_MMAX;  // half-length transforms, one system at a time
        const bool wpow2 = a.M == 2 * SPL_MMAX;  // (the tuned 8192-point plan)
        const size_t lds = sizeof(double2) * (wpow2 ? (size_t)WPlan::LDS : (size_t)(wsplit ? a.M / 2 : a.M));
        const unsigned rows = (unsigned)std::min<int64_t>(a.P, 1024);
        const dim3 rgrid((unsigned)a.Nc, (unsigned)((a.KH + SPL_KT - 1) / SPL_KT));
        auto fft = [&](const void *fn, auto kernel) -> int {
            QG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            kernel<<<rows, wpow2 ? (passB ? WIDE_T : WIDE_FT) : SPL_T, lds, s>>>(a);
            QG_LAUNCH_CHECK();
            return QG_OK;
        };
        if (!passB) {
            if (wpow2)
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_wide<float, false, true>, spec_fft_wide<float, false, true>)
                               : fft((const void *)spec_fft_wide<double, false, true>, spec_fft_wide<double, false, true>));
            else if (wsplit)
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_wide<float, false, false>, spec_fft_wide<float, false, false>)
                               : fft((const void *)spec_fft_wide<double, false, false>, spec_fft_wide<double, false, false>));
            else
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_split<float, false>, spec_fft_split<float, false>)
                               : fft((const void *)spec_fft_split<double, false>, spec_fft_split<double, false>));
            if (a.f32) spec_passA_split<float><<<rgrid, SPL_KT, 0, s>>>(a);
            else spec_passA_split<double><<<rgrid, SPL_KT, 0, s>>>(a);
            QG_LAUNCH_CHECK();
        } else {
            if (a.f32) spec_passB_split<float><<<rgrid, SPL_KT, 0, s>>>(a);
            else spec_passB_split<double><<<rgrid, SPL_KT, 0, s>>>(a);
            QG_LAUNCH_CHECK();
            if (wpow2)
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_wide<float, true, true>, spec_fft_wide<float, true, true>)
                               : fft((const void *)spec_fft_wide<double, true, true>, spec_fft_wide<double, true, true>));
            else if (wsplit)
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_wide<float, true, false>, spec_fft_wide<float, true, false>)
                               : fft((const void *)spec_fft_wide<double, true, false>, spec_fft_wide<double, true, false>));
            else
                QG_CHECK(a.f32 ? fft((const void *)spec_fft_split<float, true>, spec_fft_split<float, true>)
                               : fft((const void *)spec_fft_split<double, true>, spec_fft_split<double, true>));
        }
        return QG_OK;
    }
    const size_t lds = sizeof(double2) * 3 * (size_t)a.M;  // row, transform, twiddles
    auto go = [&](const void *fn, auto kernel) -> int {
        QG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        kernel<<<a.Nc, GEN_T, lds, s>>>(a);
        return QG_OK;
    };
    if (passB) {
        QG_CHECK(a.f32 ? go((const void *)spec_passB_gen<float>, spec_passB_gen<float>)
                       : go((const void *)spec_passB_gen<double>, spec_passB_gen<double>));
    } else {
        QG_CHECK(a.f32 ? go((const void *)spec_passA_gen<float>, spec_passA_gen<float>)
                       : go((const void *)spec_passA_gen<double>, spec_passA_gen<double>));
    }
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// power-of-two rows 8 .. 8192 (FFT passes), any other rows 3 .. GEN_MMAX (generic passes)
// and GEN_MMAX .. SPL_MMAX (split passes), even rows to SPL_WMAX (wide split passes), any row
// ---- two-point domains (global M = 2 or P = 2, one rank) --------------------------------
// The reference's 1-D periodic operator is laplacian_1d with the wrap entries written over it
// (laplacian.jl:40-45).  For N = 2 the wrap entries ARE the neighbour entries, so its D_2 is
// [-2 1; 1 -2] -- eigenvalue -1 on (1, 1), -3 on (1, -1) -- not the periodic 5-point operator's
// [-2 2; 2 -2] that the FACR passes diagonalise.  Solved here as the reference builds it
// (construct_spA, laplacian.jl:54-58): in the modes q of the two-point direction
// (X_q = x_a + x_b, x_a - x_b) the system (L + alpha dx^2) x = dx^2 zeta~ separates into one
// line along the other direction per (system, mode), (D_N + c_q) X_q = R_q with
// c_q = lambda_q + alpha dx^2 <= -1: cyclic tridiagonal (diagonal a = -(r + 1/r), both
// neighbours 1) for N >= 3, solved exactly as X = -r (1 - r S+)^-1 (1 - r S-)^-1 R with the
// periodic closures of the two first-order filters, or the 2 x 2 [a 1; 1 a] for N = 2.  Both
// systems are nonsingular, so the pinned Poisson system of get_poisson_cholesky (row and column
// of point 1 -> identity, b[1] = 0; laplacian.jl:66-75, model.jl:185) is the unpinned solution y
// plus the multiple of z = A0^-1 e_1 that zeroes point 1: x = y - (y_1 / z_1) z (only the first
// equation is dropped, so A x = b + mu e_1 with x_1 = 0).  z is solved once at init by the same
// kernel (unit = 1).  One workgroup: all threads stage the right-hand sides, four threads run the
// lines, then all threads combine the modes, pin, back-project and write the ghost ring.  No performance at stake (a test domain).
template <class S>
__global__ __launch_bounds__(256) void spec_twopoint(SpecArgs a, int unit) {
    const int64_t M = a.M, P = a.P, ld = a.ld, N = a.two_N;
    const double dx2 = a.dx * a.dx;
    // line point n, two-point index t -> interior (i, j)
    auto idx = [&](int64_t n, int t) -> int64_t {
        return a.two_yline ? fidx(1 + t, n + 1, ld) : fidx(n + 1, 1 + t, ld);
    };
    const S *in1 = static_cast<const S *>(a.in1), *in2 = static_cast<const S *>(a.in2);
    // the four right-hand sides, staged by the whole workgroup (coalesced): line (s, q) gets
    // dx^2 (zeta~_a +- zeta~_b) of mode q; unit: -dx^2 e_1 in both modes of system 0
    for (int64_t e = threadIdx.x; e < 4 * N; e += blockDim.x) {
        const int sq = (int)(e / N), s = sq >> 1, q = sq & 1;
        const int64_t n = e - (int64_t)sq * N;
        double v = 0.0;
        if (unit) {
            v = n == 0 ? -dx2 : 0.0;
        } else {
            const double pa = a.pin_in[2 * s], pb = a.pin_in[2 * s + 1];
            const int64_t o0 = idx(n, 0), o1 = idx(n, 1);
            // b[1] = 0: system 0's pinned point drops out of its right-hand side
            const double v0 = (s == 0 && a.pinned0 && n == 0) ? 0.0 : pa * (double)in1[o0] + pb * (double)in2[o0];
            const double v1 = pa * (double)in1[o1] + pb * (double)in2[o1];
            v = dx2 * (q == 0 ? v0 + v1 : v0 - v1);
        }
        a.two_X[e] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {  // the line solves, in place over the staged right-hand sides
        const int s = threadIdx.x >> 1, q = threadIdx.x & 1;
        double *X = a.two_X + (size_t)(2 * s + q) * N;
        if (!unit || s == 0) {
            const double r = a.two_r[s][q];
            if (N == 2) {  // [a 1; 1 a]^-1 = [a -1; -1 a] / (a^2 - 1), a = two_r
                const double r0 = X[0], r1 = X[1], den = r * r - 1.0;
                X[0] = (r * r0 - r1) / den;
                X[1] = (r * r1 - r0) / den;
            } else {
                // w = (1 - r S-)^-1 R: w_n = R_n + r w_{n-1}, w_0 = sum_m r^m R_{-m} / (1 - r^N)
                double acc = 0.0, pw = 1.0;
                for (int64_t m = 0; m < N && pw != 0.0; ++m) {
                    acc += pw * X[(N - m) % N];
                    pw *= r;
                }
                double w = acc * a.two_inv1mrN[s][q];
                X[0] = w;
#pragma unroll 8
                for (int64_t n = 1; n < N; ++n) {
                    w = X[n] + r * w;
                    X[n] = w;
                }
                // v = (1 - r S+)^-1 w: v_n = w_n + r v_{n+1}, v_{N-1} = sum_m r^m w_{N-1+m} / (1 - r^N)
                acc = 0.0;
                pw = 1.0;
                for (int64_t m = 0; m < N && pw != 0.0; ++m) {
                    acc += pw * X[(N - 1 + m) % N];
                    pw *= r;
                }
                double v = acc * a.two_inv1mrN[s][q];
                X[N - 1] = -r * v;
#pragma unroll 8
                for (int64_t n = N - 2; n >= 0; --n) {
                    v = X[n] + r * v;
                    X[n] = -r * v;
                }
            }
        }
    }
    __syncthreads();
    const double *X = a.two_X;
    auto sol = [&](int s, int64_t n, int t) -> double {
        const double p = X[(size_t)(2 * s) * N + n], m = X[(size_t)(2 * s + 1) * N + n];
        return 0.5 * (t == 0 ? p + m : p - m);
    };
    if (unit) {
        for (int64_t e = threadIdx.x; e < 2 * N; e += blockDim.x) a.two_z[e] = sol(0, e >> 1, (int)(e & 1));
        return;
    }
    const double y1 = sol(0, 0, 0);
    const double mu = a.pinned0 ? y1 / a.two_z[0] : 0.0;
    if (threadIdx.x == 0) {
        a.scal[0] = 0.0;  // no compatibility shift: both systems are nonsingular
        a.scal[1] = y1;   // the unpinned solution at point 1, removed by the pin
    }
    S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
    const int64_t tot = (M + 2) * (P + 2);
    for (int64_t e = threadIdx.x; e < tot; e += blockDim.x) {
        const int64_t gi = e % (M + 2), gj = e / (M + 2);
        const int64_t i = ((gi - 1) % M + M) % M, j = ((gj - 1) % P + P) % P;  // periodic ghosts
        const int64_t n = a.two_yline ? j : i;
        const int t = (int)(a.two_yline ? i : j);
        double x0 = sol(0, n, t);
        if (a.pinned0) x0 -= mu * a.two_z[2 * n + t];
        const double x1 = sol(1, n, t);
        out1[gi + ld * gj] = (S)(a.pin_out[0] * x0 + a.pin_out[1] * x1);
        if (out2) out2[gi + ld * gj] = (S)(a.pin_out[2] * x0 + a.pin_out[3] * x1);
    }
}

// beyond (odd above SPL_MMAX, or above SPL_WMAX) up to BL_MMAX (Bluestein rows)
static bool bluestein_rows(int64_t M) { return M > SPL_WMAX || (M > SPL_MMAX && M % 2 != 0); }
bool SpectralSolver::supports(int64_t M, int64_t P) {
    if (P < 2) return false;
    if (M >= 8 && M <= 8192 && (M & (M - 1)) == 0) return true;
    if (M > SPL_MMAX) return M <= BL_MMAX;
    return M >= 2 && M <= SPL_MMAX;  // (M = 2: the two-point path, one rank)
}

// Bluestein tables (long double on the host): the chirp, and the filter's length-L transform
// (an iterative radix-2 FFT in long double, scaled by 1/L)
static void bl_tables(int64_t M, int L, std::vector<double2> &chirp, std::vector<double2> &bhat,
                      std::vector<double2> &twL) {
    const long double pi = 3.141592653589793238462643383279503L;
    chirp.resize(M);
    std::vector<long double> br(L, 0.0L), bi(L, 0.0L);
    for (int64_t n = 0; n < M; ++n) {
        const int64_t q = (n * n) % (2 * M);  // exp(-+ pi i n^2 / M) has period 2M in n^2
        const long double ang = pi * (long double)q / (long double)M;
        chirp[n] = make_double2((double)cosl(ang), (double)-sinl(ang));
        br[n] = cosl(ang);
        bi[n] = sinl(ang);
        if (n > 0) {
            br[L - n] = br[n];
            bi[L - n] = bi[n];
        }
    }
    for (int i = 1, j = 0; i < L; ++i) {  // bit reversal
        int bit = L >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            std::swap(br[i], br[j]);
            std::swap(bi[i], bi[j]);
        }
    }
    for (int len = 2; len <= L; len <<= 1) {
        for (int k = 0; k < len / 2; ++k) {
            const long double a = -2 * pi * (long double)k / (long double)len;
            const long double wr = cosl(a), wi = sinl(a);
            for (int i = 0; i < L; i += len) {
                const int u = i + k, v = i + k + len / 2;
                const long double xr = br[v] * wr - bi[v] * wi, xi = br[v] * wi + bi[v] * wr;
                br[v] = br[u] - xr;
                bi[v] = bi[u] - xi;
                br[u] += xr;
                bi[u] += xi;
            }
        }
    }
    bhat.resize(L);
    twL.resize(L);
    for (int m = 0; m < L; ++m) {
        bhat[m] = make_double2((double)(br[m] / L), (double)(bi[m] / L));
        const long double a = 2 * pi * (long double)m / (long double)L;
        twL[m] = make_double2((double)cosl(a), (double)-sinl(a));
    }
}

// Rows per chunk: at most 16 (chunk summaries stay a small fraction of the traffic; 32 for
// the wide rows, whose passes run two workgroups per chunk and whose summaries are twice as
// long), small enough that the P / L workgroups of passes A and B cover the 256 CUs, and
// dividing P.
static int pick_chunk(int64_t M, int64_t P, int req) {
    if (req > 0) return (P % req == 0 && req <= 64) ? req : -1;
    int cap = M >= 2 * HN ? 32 : 16;
    while (cap > 1 && P / cap < 256) cap >>= 1;
    for (int L = cap; L >= 1; L >>= 1)
        if (P % L == 0) return L;
    return 1;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

int SpectralSolver::init(int64_t M, int64_t P, int64_t P_total, int rank, int nranks, double dx,
                         const double alpha[2], int pinned0, const double pin_in[4], const double pin_out[4],
                         int chunk_rows, int f32) {
    if (!supports(M, P)) return QG_ERR_UNSUPPORTED;
    if (!(dx > 0) || nranks < 1 || rank < 0 || rank >= nranks || P_total != P * nranks) return QG_ERR_INVALID_ARG;
    // two points in a direction (global): the reference's laplacian_1d_periodic
    // (laplacian.jl:40-45) writes its wrap entry over the neighbour entry, so its matrix is not
    // the periodic 5-point operator the passes below diagonalise -- solved as the reference
    // builds it by spec_twopoint (one rank: a two-row domain split over ranks has one-row slabs)
    if (M == 2 || P_total == 2) return init_twopoint(M, P, nranks, dx, alpha, pinned0, pin_in, pin_out, f32);
    const int L = pick_chunk(M, P, chunk_rows);
    if (L < 1) return QG_ERR_INVALID_ARG;
    SpecArgs &a = a_;
    a.M = M;
    a.P = P;
    a.ld = M + 2;
    a.P_total = P_total;
    a.rank = rank;
    a.nranks = nranks;
    a.L = L;
    a.Nc = (int)(P / L);
    a.f32 = f32;
    a.KH = (int)(M / 2 + 1);
    a.KS = (a.KH + 63) & ~63;
    a.nrad = 0;
    // generic rows: mixed-radix plan, or none (direct DFT: rows with a prime factor > 13, and
    // short rows, where the direct DFT measured no slower -- 120^2: 15 600-17 200 vs 15 000 steps/s)
    const bool blue = bluestein_rows(M);
    const bool wsplit = M > SPL_MMAX && !blue;  // (planned at the half length H = M/2)
    if (!blue && (wsplit || ((M & (M - 1)) != 0 && M > 128))) {
        int64_t m = wsplit ? M / 2 : M, n = 0;
        int rad[16];
        while (m % 8 == 0) { rad[n++] = 8; m /= 8; }
        if (m % 4 == 0) { rad[n++] = 4; m /= 4; }
        if (m % 2 == 0) { rad[n++] = 2; m /= 2; }
        for (int p = 3; p <= GEN_RMAX && m > 1; p += 2)
            while (m % p == 0 && n < 16) { rad[n++] = p; m /= p; }
        if (m == 1) {
            a.nrad = (int)n;
            for (int i = 0; i < n; ++i) a.rad[i] = rad[i];
        }
    }
    a.dx = dx;
    a.pinned0 = pinned0 ? 1 : 0;
    std::memcpy(a.pin_in, pin_in, sizeof(a.pin_in));
    std::memcpy(a.pin_out, pin_out, sizeof(a.pin_out));
    const int KS = a.KS;

    // ---- tables (long double) --------------------------------------------------------
    std::vector<double2> tw(M);
    const long double twopi = 6.283185307179586476925286766559L;
    for (int64_t m = 0; m < M; ++m) {
        const long double ang = twopi * (long double)m / (long double)M;
        tw[m] = make_double2((double)cosl(ang), (double)-sinl(ang));
    }
    std::vector<Coef> coef(2 * (size_t)KS);
    std::memset(coef.data(), 0, sizeof(Coef) * coef.size());
    for (int s = 0; s < 2; ++s)
        for (int k = 0; k < a.KH; ++k) {
            Coef &cf = coef[s * KS + k];
            if (s == 0 && pinned0 && k == 0) continue;  // singular line, r = 0 marker
            const long double th = twopi * (long double)k / (long double)M;
            const long double sh = sinl(th / 2);
            const long double d = 2 * sh * sh - (long double)alpha[s] * (long double)dx * (long double)dx / 2;
            if (!(d > 0)) return QG_ERR_UNSUPPORTED;  // singular (alpha = 0 unpinned) or alpha > 0
            // r = rho - sqrt(rho^2 - 1) with rho = 1 + d, in cancellation-free form
            const long double sq = sqrtl(d * (d + 2));
            const long double r = 1 / ((1 + d) + sq);
            const long double lr = -log1pl(d + sq);
            if (!(r > 1e-300L)) return QG_ERR_UNSUPPORTED;  // |alpha| dx^2 beyond double range
            cf.r = (double)r;
            cf.rinv = (double)(1 / r);
            cf.lr = (double)lr;
            cf.q = (double)expl(L * lr);
            cf.qm1 = (double)expl((L - 1) * lr);
            if (-(L - 1) * lr > 600) return QG_ERR_UNSUPPORTED;  // r^-(L-1) scaling would overflow
            cf.gam = (double)(r * expm1l(2 * L * lr) / expm1l(2 * lr));
            cf.rP = (double)expl((long double)P * lr);
            cf.gamP = (double)(r * expm1l(2 * (long double)P * lr) / expm1l(2 * lr));
            cf.cs = (double)(-r * (long double)dx * (long double)dx / (long double)M);
            cf.inv1mrPt = (double)(-1 / expm1l((long double)P_total * lr));
        }

    // ---- device memory ---------------------------------------------------------------
    const size_t n_tw = align_up(sizeof(double2) * M);
    const size_t n_coef = align_up(sizeof(Coef) * coef.size());
    const size_t n_hot = align_up(sizeof(double) * 14 * (size_t)KS);
    const size_t n_U = align_up(sizeof(double2) * (size_t)P * 2 * KS);
    const size_t n_S = align_up(sizeof(double2) * (size_t)a.Nc * 2 * KS);
    const size_t n_dc = align_up(sizeof(double) * a.Nc);
    const int64_t RS = rec_size(KS, P);
    const size_t n_rec = align_up(sizeof(double) * RS);
    const size_t n_grec = align_up(sizeof(double) * RS * nranks);  // gather target (also 1-rank ring)
    const size_t n_ext = align_up(sizeof(double2) * 4 * KS);
    const size_t n_line = align_up(sizeof(double) * P);  // (hline and line)
    const size_t n_scal = align_up(sizeof(double) * 8);
    const int nkb = (a.KH + CARRY_KB - 1) / CARRY_KB;  // carry k-blocks (fused pin parts)
    // zero-padded to PIN_PAD parts: every pass B thread loads one unconditionally (pin_part)
    const size_t n_pinpart = align_up(sizeof(double) * (std::max({pin_kblocks(a.KH), nkb, PIN_PAD}) + 1));
    const bool wide = M == 2 * HN;  // wide-row passes: half-length twiddles + system-0 rows
    const size_t n_tw2 = (wide || wsplit) ? align_up(sizeof(double2) * (size_t)(M / 2)) : 0;
    const size_t n_half = wide ? align_up((f32 ? sizeof(float) : sizeof(double)) * (size_t)P * M) : 0;
    // split passes with a plan: where the DIF stages leave frequency k (digit reversal)
    const int64_t MP = wsplit ? M / 2 : M;  // length of the planned transform
    const size_t n_perm = a.nrad > 0 ? align_up(sizeof(int) * MP) : 0;
    std::vector<double2> bl_chirp, bl_bhat, bl_twL;
    int BL = 0, brows = 0;
    if (blue) {
        BL = 1;
        while (BL < 2 * M - 1) BL <<= 1;
        brows = (int)std::max<int64_t>(1, std::min<int64_t>(P, (int64_t)(BL_BUF_BYTES / (sizeof(double2) * BL))));
        bl_tables(M, BL, bl_chirp, bl_bhat, bl_twL);
    }
    const size_t n_bl = blue ? align_up(sizeof(double2) * M) + 2 * align_up(sizeof(double2) * BL) +
                                   2 * align_up(sizeof(double2) * (size_t)BL * brows)
                             : 0;
    bytes_ = n_tw + n_coef + n_hot + n_U + 4 * n_S + n_dc + n_rec + n_grec + n_ext + 2 * n_line + n_scal + n_pinpart +
             n_tw2 + n_half + n_perm + n_bl;
    if (hipMalloc(&mem_, bytes_) != hipSuccess) {
        mem_ = nullptr;
        return QG_ERR_ALLOC;
    }
    char *p = static_cast<char *>(mem_);
    auto take = [&](size_t n) { char *r = p; p += n; return r; };
    double2 *d_tw = (double2 *)take(n_tw);
    Coef *d_coef = (Coef *)take(n_coef);
    double *d_hot = (double *)take(n_hot);
    a.U = take(n_U);  // double2 (F64 states) or float2 (F32) per element
    a.ULS = (double2 *)take(n_S);
    a.WLS = (double2 *)take(n_S);
    a.UIN = (double2 *)take(n_S);
    a.WIN = (double2 *)take(n_S);
    a.dcpart = (double *)take(n_dc);
    a.rec = (double *)take(n_rec);
    grec_buf_ = (double *)take(n_grec);
    a.grec = nranks > 1 ? grec_buf_ : a.rec;
    a.rec_stride = RS;
    a.EXT = (double2 *)take(n_ext);
    a.line = (double *)take(n_line);
    a.hline = (double *)take(n_line);
    a.scal = (double *)take(n_scal);
    a.pinpart = (double *)take(n_pinpart);
    a.tw2 = (wide || wsplit) ? (const double2 *)take(n_tw2) : nullptr;
    a.half_tmp = wide ? (void *)take(n_half) : nullptr;
    a.perm = nullptr;
    if (a.nrad > 0) {
        int *d_perm = (int *)take(n_perm);
        std::vector<int> perm(MP);
        for (int64_t k = 0; k < MP; ++k) {
            int64_t rem = k, span = MP, pos = 0;
            for (int q = 0; q < a.nrad; ++q) {
                span /= a.rad[q];
                pos += (rem % a.rad[q]) * span;
                rem /= a.rad[q];
            }
            perm[k] = (int)pos;
        }
        QG_HIP(hipMemcpy(d_perm, perm.data(), sizeof(int) * MP, hipMemcpyHostToDevice));
        a.perm = d_perm;
    }
    a.bl_L = 0;
    if (blue) {
        double2 *ch = (double2 *)take(align_up(sizeof(double2) * M));
        double2 *bh = (double2 *)take(align_up(sizeof(double2) * BL));
        double2 *tl = (double2 *)take(align_up(sizeof(double2) * BL));
        a.bl_buf0 = (double2 *)take(align_up(sizeof(double2) * (size_t)BL * brows));
        a.bl_buf1 = (double2 *)take(align_up(sizeof(double2) * (size_t)BL * brows));
        QG_HIP(hipMemcpy(ch, bl_chirp.data(), sizeof(double2) * M, hipMemcpyHostToDevice));
        QG_HIP(hipMemcpy(bh, bl_bhat.data(), sizeof(double2) * BL, hipMemcpyHostToDevice));
        QG_HIP(hipMemcpy(tl, bl_twL.data(), sizeof(double2) * BL, hipMemcpyHostToDevice));
        a.bl_chirp = ch;
        a.bl_bhat = bh;
        a.bl_tw = tl;
        a.bl_L = BL;
        a.bl_rows = brows;
    }
    a.tw = d_tw;
    a.coef = d_coef;
    QG_HIP(hipMemcpy(d_tw, tw.data(), sizeof(double2) * M, hipMemcpyHostToDevice));
    if (wide || wsplit) {  // exp(-2 pi i m / (M/2)) = tw[2m]
        const int64_t H = M / 2;
        std::vector<double2> tw2(H);
        for (int64_t m = 0; m < H; ++m) tw2[m] = tw[2 * m];
        QG_HIP(hipMemcpy((void *)a.tw2, tw2.data(), sizeof(double2) * H, hipMemcpyHostToDevice));
    }
    QG_HIP(hipMemcpy(d_coef, coef.data(), sizeof(Coef) * coef.size(), hipMemcpyHostToDevice));
    {
        // [2][KS] (r, 1/r) pairs, [2][KS] cs, [2][KS] r; slot order: [2][KS] (r, 1/r), [2][KS] r
        std::vector<double> hot(14 * (size_t)KS);
        for (size_t i = 0; i < 2 * (size_t)KS; ++i) {
            hot[2 * i] = coef[i].r;
            hot[2 * i + 1] = coef[i].rinv;
            hot[4 * KS + i] = coef[i].cs;
            hot[6 * KS + i] = coef[i].r;
        }
        if (M == lx::N || M == 2 * lx::N) {
            const int lines = M == lx::N ? 4 : 8;  // per thread and system
            for (int s = 0; s < 2; ++s)
                for (int t = 0; t < lx::T; ++t)
                    for (int q = 0; q < lines; ++q) {
                        const int g = lx::mirror_group(t), gm = g == 0 ? 0 : 512 - g;
                        const size_t k = (size_t)((q < 4 ? g : gm) + 512 * q), slot = (size_t)(t + 512 * q);
                        const Coef &cf = coef[(size_t)s * KS + k];
                        hot[8 * KS + 2 * (s * KS + slot)] = cf.r;
                        hot[8 * KS + 2 * (s * KS + slot) + 1] = cf.rinv;
                        hot[12 * KS + s * KS + slot] = cf.r;
                    }
        }
        QG_HIP(hipMemcpy(d_hot, hot.data(), sizeof(double) * hot.size(), hipMemcpyHostToDevice));
        a.crr = reinterpret_cast<const double2 *>(d_hot);
        a.ccs = d_hot + 4 * KS;
        a.cr = d_hot + 6 * KS;
        a.scrr = reinterpret_cast<const double2 *>(d_hot + 8 * KS);
        a.scr = d_hot + 12 * KS;
        a.csc = -(dx * dx) / (double)M;
    }
    QG_HIP(hipMemset(a.rec, 0, n_rec));
    QG_HIP(hipMemset(a.scal, 0, n_scal));
    QG_HIP(hipMemset(a.line, 0, n_line));
    QG_HIP(hipMemset(a.pinpart, 0, n_pinpart));
    return QG_OK;
}

int SpectralSolver::init_twopoint(int64_t M, int64_t P, int nranks, double dx, const double alpha[2], int pinned0,
                                  const double pin_in[4], const double pin_out[4], int f32) {
    if (nranks != 1) return QG_ERR_UNSUPPORTED;
    SpecArgs &a = a_;
    a.M = M;
    a.P = P;
    a.ld = M + 2;
    a.P_total = P;
    a.rank = 0;
    a.nranks = 1;
    a.f32 = f32;
    a.dx = dx;
    a.pinned0 = pinned0 ? 1 : 0;
    std::memcpy(a.pin_in, pin_in, sizeof(a.pin_in));
    std::memcpy(a.pin_out, pin_out, sizeof(a.pin_out));
    a.two = 1;
    a.two_yline = P != 2 ? 1 : 0;  // (M = P = 2: the line along x, of two points)
    const int64_t N = a.two_yline ? P : M;
    a.two_N = N;
    const long double lam[2] = {-1.0L, -3.0L};  // D_2 on (1, 1) and (1, -1)
    for (int s = 0; s < 2; ++s)
        for (int q = 0; q < 2; ++q) {
            const long double c = lam[q] + (long double)alpha[s] * (long double)dx * (long double)dx;
            if (!(c < 0)) return QG_ERR_UNSUPPORTED;  // (alpha > 0: not the reference's systems)
            if (N == 2) {
                a.two_r[s][q] = (double)(c - 2);  // the diagonal a of [a 1; 1 a]
                a.two_inv1mrN[s][q] = 0;
            } else {
                const long double rho = 1 - c / 2;  // > 1
                const long double r = 1 / (rho + sqrtl((rho - 1) * (rho + 1)));
                a.two_r[s][q] = (double)r;
                a.two_inv1mrN[s][q] = (double)(-1 / expm1l((long double)N * logl(r)));
            }
        }
    const size_t n_X = align_up(sizeof(double) * 4 * (size_t)N), n_z = align_up(sizeof(double) * 2 * (size_t)N);
    const size_t n_scal = align_up(sizeof(double) * 8);
    bytes_ = n_X + n_z + n_scal;
    if (hipMalloc(&mem_, bytes_) != hipSuccess) {
        mem_ = nullptr;
        return QG_ERR_ALLOC;
    }
    char *p = static_cast<char *>(mem_);
    a.two_X = (double *)p;
    a.two_z = (double *)(p + n_X);
    a.scal = (double *)(p + n_X + n_z);
    QG_HIP(hipMemset(mem_, 0, bytes_));
    if (a.pinned0) {  // z = A0^-1 e_1, once
        spec_twopoint<double><<<1, 256, 0, nullptr>>>(a, 1);
        QG_LAUNCH_CHECK();
        QG_HIP(hipStreamSynchronize(nullptr));
    }
    return QG_OK;
}

SpectralSolver::~SpectralSolver() {
    if (mem_) (void)hipFree(mem_);
}

int SpectralSolver::solve(const void *in1, const void *in2, void *out1, void *out2, int write_ghost_rows,
                          hipStream_t s, GatherFn gather, void *user, const double *pin_in, const double *pin_out,
                          void *zcopy1, void *zcopy2) {
    if (!mem_) return QG_ERR_NOT_BOUND;
    if ((zcopy1 || zcopy2) && (!fuses_input_copy() || !zcopy1 || !zcopy2 || a_.nranks > 1)) return QG_ERR_INVALID_ARG;
    SpecArgs a = a_;
    a.zcopy1 = zcopy1;
    a.zcopy2 = zcopy2;
    if (pin_in) std::memcpy(a.pin_in, pin_in, sizeof(a.pin_in));
    if (pin_out) std::memcpy(a.pin_out, pin_out, sizeof(a.pin_out));
    a.in1 = in1;
    a.in2 = in2 ? in2 : in1;
    a.out1 = out1;
    a.out2 = out2;
    a.write_ghost_rows = write_ghost_rows;
    if (a.two) {
        if (a.f32) spec_twopoint<float><<<1, 256, 0, s>>>(a, 0);
        else spec_twopoint<double><<<1, 256, 0, s>>>(a, 0);
        QG_LAUNCH_CHECK();
        return QG_OK;
    }
    // one rank: the carry kernel closes the lines itself (no spec_pin), with or without a
    // transport -- a 1-rank ring's record all-gather would only copy the record onto itself
    // (grec aliases rec), so none is posted (r04: RCCL's one-rank all-gather was a 6 us copy
    // kernel and spec_pin another launch on the 1-rank ring's critical path)
    a.fuse_pin = a.nranks == 1 ? 1 : 0;
    a.npin = a.fuse_pin ? (a.KH + CARRY_KB - 1) / CARRY_KB : pin_kblocks(a.KH);
    QG_CHECK(dispatch_pass(false, a, s));
    {
        const unsigned nkb = (unsigned)((a.KH + CARRY_KB - 1) / CARRY_KB) + 1;
        static int cus = 0;
        if (cus == 0) {
            int dev = 0;
            QG_HIP(hipGetDevice(&dev));
            QG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        }
        if (2 * (int)nkb > cus) spec_carry<4><<<dim3(nkb, 2), 64 * CARRY_WAVES, 0, s>>>(a);
        else spec_carry<1><<<dim3(nkb, 2), 64 * CARRY_WAVES, 0, s>>>(a);
    }
    QG_LAUNCH_CHECK();
    if (a.nranks > 1) {
        if (!gather) return QG_ERR_RCCL;
        QG_CHECK(gather(user, a.rec, grec_buf_, a.rec_stride, s));
    }
    if (!a.fuse_pin) {
        spec_pin<<<pin_kblocks(a.KH), PIN_THREADS, 0, s>>>(a);
        QG_LAUNCH_CHECK();
    }
    QG_CHECK(dispatch_pass(true, a, s));
    return QG_OK;
}

}  // namespace qg
