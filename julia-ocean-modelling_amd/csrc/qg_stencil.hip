// Stencil kernels for gfx950: the Arakawa-Jacobian tendency + Euler/AB3 update, the
// stand-alone laplace_5p / cd / J / ghost-fill operators and the seeded initialisation.
//
// Arithmetic follows the reference term by term and this file is compiled with
// -ffp-contract=off, so results are bit-identical to oracle/qg_oracle.c:
//   laplace_5p            src/schemes/laplacian.jl:15-27
//   cd                    src/model.jl:68-80
//   j_pp, j_pt, j_tp, J   src/schemes/arakawa.jl:7-62
//   zeta_f1 / zeta_f2     src/model.jl:139-153
//   eulers_method / AB3   src/model.jl:123-136
//   ghost ring            src/schemes/boundary_conditions.jl:2-13
//   initialise_model      src/model.jl:37-62
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "qg_common.hpp"

namespace qg {

// ------------------------------------------------------------------------------------
// Stand-alone operators on (M+2, P+2) fields (reference semantics: interior from the
// input's ghost ring, output ghosts refreshed).
// ------------------------------------------------------------------------------------
__global__ void laplace_kernel(const double *__restrict__ u, double *__restrict__ out, int64_t M,
                               int64_t P, double idx2) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i >= M) return;
    const int64_t ld = M + 2, mi = i + 1, mj = j + 1;
    const double v = ((((u[fidx(mi - 1, mj, ld)] + u[fidx(mi + 1, mj, ld)]) - 4 * u[fidx(mi, mj, ld)]) +
                       u[fidx(mi, mj - 1, ld)]) + u[fidx(mi, mj + 1, ld)]) * idx2;
    store_with_ghosts(out, ld, M, P, i, j, v, true);
}

__global__ void cd_kernel(const double *__restrict__ u, double *__restrict__ out, int64_t M, int64_t P,
                          double c) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i >= M) return;
    const int64_t ld = M + 2, mi = i + 1, mj = j + 1;
    store_with_ghosts(out, ld, M, P, i, j, c * (u[fidx(mi + 1, mj, ld)] - u[fidx(mi - 1, mj, ld)]), true);
}

// J at one point from accessors Z(a,b), S(a,b) (arakawa.jl:7-62, same evaluation order)
template <class V, class ZF, class SF>
__device__ __forceinline__ V arakawa_point(ZF Z, SF S, V den) {
    const V jpp = (Z(1, 0) - Z(-1, 0)) * (S(0, 1) - S(0, -1)) - (Z(0, 1) - Z(0, -1)) * (S(1, 0) - S(-1, 0));
    const V jpt = ((Z(1, 0) * (S(1, 1) - S(1, -1)) - Z(-1, 0) * (S(-1, 1) - S(-1, -1))) -
                        Z(0, 1) * (S(1, 1) - S(-1, 1))) +
                       Z(0, -1) * (S(1, -1) - S(-1, -1));
    const V jtp = ((Z(1, 1) * (S(0, 1) - S(1, 0)) - Z(-1, -1) * (S(-1, 0) - S(0, -1))) -
                        Z(-1, 1) * (S(0, 1) - S(-1, 0))) +
                       Z(1, -1) * (S(1, 0) - S(0, -1));
    return ((jpp + jpt) + jtp) / den;
}

__global__ void arakawa_kernel(const double *__restrict__ z, const double *__restrict__ p,
                               double *__restrict__ out, int64_t M, int64_t P, double den) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i >= M) return;
    const int64_t ld = M + 2, mi = i + 1, mj = j + 1;
    auto Z = [&](int a, int b) { return z[fidx(mi + a, mj + b, ld)]; };
    auto S = [&](int a, int b) { return p[fidx(mi + a, mj + b, ld)]; };
    store_with_ghosts(out, ld, M, P, i, j, arakawa_point<double>(Z, S, den), true);
}

// update_doubly_periodic_bc! (boundary_conditions.jl:2-13)
__global__ void fill_ghosts_kernel(double *b, int64_t M, int64_t P, int rows_too) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t ld = M + 2;
    if (rows_too && t < M) {  // ghost columns j = 0 and j = P+1 (i interior)
        b[fidx(t + 1, 0, ld)] = b[fidx(t + 1, P, ld)];
        b[fidx(t + 1, P + 1, ld)] = b[fidx(t + 1, 1, ld)];
    }
    if (t < P) {  // ghost rows i = 0 and i = M+1 (j interior)
        b[fidx(0, t + 1, ld)] = b[fidx(M, t + 1, ld)];
        b[fidx(M + 1, t + 1, ld)] = b[fidx(1, t + 1, ld)];
    }
    if (rows_too && t == 0) {
        b[fidx(0, 0, ld)] = b[fidx(M, P, ld)];
        b[fidx(0, P + 1, ld)] = b[fidx(M, 1, ld)];
        b[fidx(M + 1, P + 1, ld)] = b[fidx(1, 1, ld)];
        b[fidx(M + 1, 0, ld)] = b[fidx(1, P, ld)];
    }
}

// Workgroup -> (strip, row block, layer), XCD-aware: workgroups are dealt round-robin to the
// 8 XCDs (each with its own L2), so the linear id is remapped (xcd_logical_id) to give each
// XCD a contiguous range of logical workgroups -- whole row blocks of adjacent strips.  The
// cache line two neighbouring strips share (rows start at element 1: strip edges are not line
// aligned) is then fetched into one L2 instead of two: 4096^2 tendency reads 1.18 -> 1.11 GB,
// 378 -> 364 us.  QG_TEND_NO_XCD restores the hardware order (A/B builds).
struct TendBlock {
    int x, y, z;
};
__device__ __forceinline__ TendBlock tend_block() {
    const int b = xcd_logical_id();
    const int x = b % gridDim.x, r = b / gridDim.x;
    return {x, r % (int)gridDim.y, r / (int)gridDim.y};
}

// ------------------------------------------------------------------------------------
// Fused tendency + Euler/AB3 update (evolve_zeta!, model.jl:155-170), one layer per
// blockIdx.z.  Each block owns TX columns (one per thread) and marches down a strip of
// rows.  Rolling LDS rings hold psi (6 rows, x-halo 2), zeta (5 rows, x-halo 1) and
// lap(psi) (4 rows, x-halo 1); the ring depths let one barrier per row suffice.  Row j+3 of
// psi, row j+2 of zeta and F(t-1), F(t-2) of row j+1 are fetched into registers while row
// j is computed (software pipeline), so HBM latency hides behind the stencil arithmetic.
// Per interior point: read zeta, psi, [F(t-1), F(t-2)], write zeta+, F (+ ghost images).
// ------------------------------------------------------------------------------------
//
// CERT (F64 PCG, one rank): the workgroup holds BOTH layers (threads [0, TX) layer 0, [TX, 2TX)
// layer 1, each with its own rings) and also certifies the solve that produced psi from zeta:
// per point and system, b_s = -(proj_in zeta)_s and r_s = b_s + (A_s psi~)_s with psi~ =
// P_fwd^-1 psi, A_s psi~ = sum_l P_fwd^-1[s][l] (lap(psi_l) + alpha_s psi_l) (lap(psi_l) is
// the ring's own), summed over the two layers through LDS; (b,b), (r,r) per workgroup.
// One strip (see tendency_pair_strip for EDGE: false = the x-halo inside the row, so no
// periodic wraps and no ghost-column stores in the row loop).  IN_ROWS: every row the strip
// reads (jb0-2 .. jb1+1) is a local row and no output row is a ghost-row image (2 <= jb0,
// jb1 + 2 <= P): the row pointers then advance by ld per row, with no range checks.
//
// Scalar work per row.  The loop's addressing is wave-uniform, so it runs on the CU's one
// scalar ALU, which all resident waves share: with ring slots as (j + 2R) % R per access (a
// signed division by 6 / 5 / 4 each), row pointers as (j + 1) * ld products and the kernel
// arguments re-read after the asm barrier below, the 4096^2 F64 tendency issued 2.1 scalar
// instructions per vector one -- 1.36e8 per launch, 529 k per CU in 809 k cycles
// (SQ_INSTS_SALU, r04k).  Now the ring slots are pointer arrays rotated once per row, the row
// pointers induction variables, and the arguments read once.
template <int TX, int PF, class T, bool CERT, bool EDGE, bool IN_ROWS>
__device__ __forceinline__ void tendency_strip(const TendArgsT<T> &a, int layer, int t, int x0, int jb0, int jb1,
                                               T (*sp)[TX + 4], T (*sz)[TX + 2], T (*sl)[TX + 2],
                                               double (*xch)[4][CERT ? TX : 1]) {
    constexpr int RP = 6, RZ = 5, RL = 4;  // ring depths
    const int M = (int)a.M, P = (int)a.P;
    const int64_t ld = a.ld;
    const int i = x0 + t;
    double cv[4] = {0, 0, 0, 0};  // (b0,b0), (r0,r0), (b1,b1), (r1,r1)
    double pend[4] = {0, 0, 0, 0};
    int pend_j = -1;
    auto cert_fold = [&]() {  // layer 0: both layers' contributions of row pend_j
        if (pend_j < 0) return;
        const double *x = &xch[pend_j & 1][0][0];
        double bs[2], rs[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bs[s] = pend[2 * s] + x[(2 * s) * TX + t];
            rs[s] = pend[2 * s + 1] + x[(2 * s + 1) * TX + t];
        }
        if (a.cert_pin && i == 0 && pend_j == 0) bs[0] = rs[0] = 0.0;  // identity row: b = x = 0
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            cv[2 * s] += bs[s] * bs[s];
            cv[2 * s + 1] += rs[s] * rs[s];
        }
        pend_j = -1;
    };

    const T *psi = a.psi[layer];
    const T *zeta = a.zeta[layer];
    const RowSrcT<T> &prs = a.psi_rows[layer];
    const RowSrcT<T> &zrs = a.zeta_rows[layer];
    // the arguments the row loop uses, read once
    const T *const fp1 = a.fprev1[layer], *const fp2 = a.fprev2[layer];
    T *const zo = a.zeta_out[layer], *const fo = a.f_out[layer];
    T *const fs1 = a.fshift1[layer], *const fs2 = a.fshift2[layer];
    const double *const wind = layer == 0 ? a.wind : nullptr;  // wind extension (off: nullptr)
    const bool gr = a.write_ghost_rows != 0;
    // model constants in the state's precision (the same expressions as the F64 path)
    const T dx = (T)a.dx, idx = T(1) / dx, idx2 = idx * idx;
    const T cdc = T(0.5) * idx;
    const T den = T(12) * (dx * dx);
    const T visc = (T)a.visc, dtT = (T)a.dt, Ut = (T)a.U, rt = (T)a.r;
    const bool small = M < TX + 4;

    auto wx = [&](int x) -> int {  // periodic wrap of an interior column index
        if constexpr (!EDGE) return x;
        if (small) return ((x % M) + M) % M;
        return x < 0 ? x + M : (x >= M ? x - M : x);
    };
    auto rowp = [&](const T *base, const RowSrcT<T> &rs, int j) -> const T * {
        if (IN_ROWS || (j >= 0 && j < P)) return base + fidx(1, j + 1, ld);
        return rs.halo[j < 0 ? j + 2 : (j - P) + 2];
    };
    // per-thread column positions: psi LDS position t+2 (own) and the halo position
    const int ph_q = t < 2 ? t : (t >= TX - 2 ? t + 4 : -1);   // psi halo slot or none
    const int zh_q = t == 0 ? 0 : (t == TX - 1 ? TX + 1 : -1);  // zeta halo slot or none
    const int xo = wx(i);
    const int xph = ph_q >= 0 ? wx(x0 - 2 + ph_q) : 0;
    const int xzh = zh_q >= 0 ? wx(x0 - 1 + zh_q) : 0;
    const bool has_out = !EDGE || i < M;
    const bool ab3 = a.ab3 != 0;

    // prefetch pipeline PF rows deep: slot 0 is consumed next
    T pc[PF], ph[PF], zc[PF], zh[PF], f1[PF], f2[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) pc[k] = ph[k] = zc[k] = zh[k] = f1[k] = f2[k] = 0;
    auto fetch_psi = [&](const T *r, T &c, T &h) {  // r: interior element 0 of the row
        c = r[xo];
        if (ph_q >= 0) h = r[xph];
    };
    auto fetch_zeta = [&](const T *r, T &c, T &h) {
        c = r[xo];
        if (zh_q >= 0) h = r[xzh];
    };
    auto fetch_f = [&](size_t o, T &g1, T &g2) {  // o: element offset of the row's interior element 0
        if (ab3 && has_out) {
            g1 = ld_stream(fp1 + o + i);
            g2 = ld_stream(fp2 + o + i);
        }
    };
    auto commit_psi = [&](auto d, T c, T h) {
        d[t + 2] = c;
        if (ph_q >= 0) d[ph_q] = h;
    };
    auto commit_zeta = [&](auto d, T c, T h) {
        d[t + 1] = c;
        if (zh_q >= 0) d[zh_q] = h;
    };
    // lap(psi) of the row whose psi rows below / at / above are pm, p0, pp: LDS positions
    // 0..TX+1 (x0-1 .. x0+TX)
    auto lap_row = [&](auto pm, auto p0, auto pp, auto dst) {
        for (int q = t; q < TX + 2; q += TX) {
            const int c = q + 1;
            dst[q] = ((((p0[c - 1] + p0[c + 1]) - T(4) * p0[c]) + pm[c]) + pp[c]) * idx2;
        }
    };
    // ring slots of the rows the iteration j uses: rP[k] = psi row j-2+k, rZ[k] = zeta row
    // j-1+k, rL[k] = lap row j-1+k; rotated by one at the end of every row
    // (LDS-typed: 32-bit addresses, one scalar register per slot)
    typedef __attribute__((address_space(3))) T *LT;
    LT rP[RP], rZ[RZ], rL[RL];
#pragma unroll
    for (int k = 0; k < RP; ++k) rP[k] = (LT)sp[(jb0 - 2 + k + 2 * RP) % RP];
#pragma unroll
    for (int k = 0; k < RZ; ++k) rZ[k] = (LT)sz[(jb0 - 1 + k + 2 * RZ) % RZ];
#pragma unroll
    for (int k = 0; k < RL; ++k) rL[k] = (LT)sl[(jb0 - 1 + k + 2 * RL) % RL];

    // prologue: psi rows jb0-2..jb0+2, zeta rows jb0-1..jb0+1 into LDS.  All eight rows' loads
    // are issued before the first LDS write (a fetch-commit loop waited one full memory latency
    // per row: eight round trips in front of every strip, while the workgroups of a chip-full,
    // which start together, all sat in them).
    {
        T p0c[5], p0h[5], z0c[3], z0h[3];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            p0c[k] = p0h[k] = 0;
            fetch_psi(rowp(psi, prs, jb0 - 2 + k), p0c[k], p0h[k]);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            z0c[k] = z0h[k] = 0;
            fetch_zeta(rowp(zeta, zrs, jb0 - 1 + k), z0c[k], z0h[k]);
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) commit_psi(rP[k], p0c[k], p0h[k]);
#pragma unroll
        for (int k = 0; k < 3; ++k) commit_zeta(rZ[k], z0c[k], z0h[k]);
    }
    // prefetch for iterations jb0 .. jb0+PF-1: psi row j+3, zeta row j+2 (committed while
    // rows are still needed, i.e. j+2 <= jb1) and F of row j
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int j = jb0 + k;
        if (j + 2 <= jb1) {
            fetch_psi(rowp(psi, prs, j + 3), pc[k], ph[k]);
            fetch_zeta(rowp(zeta, zrs, j + 2), zc[k], zh[k]);
        }
        if (j < jb1) fetch_f((size_t)(j + 1) * ld + 1, f1[k], f2[k]);
    }
    __syncthreads();
    lap_row(rP[0], rP[1], rP[2], rL[0]);
    lap_row(rP[1], rP[2], rP[3], rL[1]);
    lap_row(rP[2], rP[3], rP[4], rL[2]);

    // IN_ROWS row pointers: the next fetch (iteration j + PF) and this row's outputs
    const T *nP = psi + fidx(1, jb0 + PF + 3 + 1, ld), *nZ = zeta + fidx(1, jb0 + PF + 2 + 1, ld);
    size_t nF = (size_t)(jb0 + PF + 1) * ld + 1;
    size_t oRow = (size_t)(jb0 + 1) * ld;

    const T bl = (T)a.beta[layer];
    for (int j = jb0; j < jb1; ++j) {
        const bool more = j + 2 <= jb1;  // psi row j+3 / zeta row j+2 / lap row j+2 needed
        if (more) {
            commit_psi(rP[5], pc[0], ph[0]);
            commit_zeta(rZ[3], zc[0], zh[0]);
        }
        const T f1c = f1[0], f2c = f2[0];
        // land this row's F(t-1), F(t-2) (issued last iteration) before the next row's loads
        // go out: loads complete in order (vmcnt), and with f1c / f2c first read after the
        // new loads the compiler waited for those too (vmcnt(0)) on every row
        asm volatile("" : : "v"(f1c), "v"(f2c) : "memory");
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) {
            pc[k] = pc[k + 1];
            ph[k] = ph[k + 1];
            zc[k] = zc[k + 1];
            zh[k] = zh[k + 1];
            f1[k] = f1[k + 1];
            f2[k] = f2[k + 1];
        }
        {
            const int jn = j + PF;  // iteration whose inputs are fetched now
            if (jn + 2 <= jb1) {
                fetch_psi(IN_ROWS ? nP : rowp(psi, prs, jn + 3), pc[PF - 1], ph[PF - 1]);
                fetch_zeta(IN_ROWS ? nZ : rowp(zeta, zrs, jn + 2), zc[PF - 1], zh[PF - 1]);
            }
            if (jn < jb1) fetch_f(IN_ROWS ? nF : (size_t)(jn + 1) * ld + 1, f1[PF - 1], f2[PF - 1]);
        }
        __syncthreads();
        if constexpr (CERT) {
            if (layer == 0) cert_fold();  // row j-1: layer 1 wrote its part before this barrier
        }
        if (more) lap_row(rP[3], rP[4], rP[5], rL[3]);
        if (has_out) {
            const LT Lm = rL[0], L0 = rL[1], Lp = rL[2];
            const LT Pm = rP[1], P0 = rP[2], Pp = rP[3];
            const LT Zm = rZ[0], Z0 = rZ[1], Zp = rZ[2];
            const int cl = t + 1;  // centre in sl / sz (x-halo 1)
            const int cp = t + 2;  // centre in sp (x-halo 2)
            const T biharm = ((((L0[cl - 1] + L0[cl + 1]) - T(4) * L0[cl]) + Lm[cl]) + Lp[cl]) * idx2;
            const T v_term = visc * biharm;
            auto Z = [&](int da, int db) {
                const LT r = db < 0 ? Zm : (db > 0 ? Zp : Z0);
                return r[cl + da];
            };
            auto S = [&](int da, int db) {
                const LT r = db < 0 ? Pm : (db > 0 ? Pp : P0);
                return r[cp + da];
            };
            const T J_term = arakawa_point<T>(Z, S, den);
            const T beta_term = bl * (cdc * (P0[cp + 1] - P0[cp - 1]));
            T last;
            if (layer == 0) last = Ut * (cdc * (Z0[cl + 1] - Z0[cl - 1]));  // U * cd(zeta)
            else last = rt * L0[cl];                                         // r * lap(psi)
            T F = ((v_term - J_term) - beta_term) - last;
            if (wind) F = F + (T)wind[j];
            const T zcen = Z0[cl];
            const T zn = ab3 ? zcen + dtT * ((((T)(23.0 / 12.0) * F) - ((T)(16.0 / 12.0) * f1c)) + ((T)(5.0 / 12.0) * f2c))
                             : zcen + (dtT * F);
            const size_t orow = IN_ROWS ? oRow : (size_t)(j + 1) * ld;
            store_row_with_ghosts<T, EDGE>(zo + orow, IN_ROWS ? nullptr : ghost_row_target(zo, ld, P, j, gr), M, i, zn);
            store_row_with_ghosts<T, EDGE>(fo + orow, IN_ROWS ? nullptr : ghost_row_target(fo, ld, P, j, gr), M, i, F);
            if (ab3 && fs1) {  // (see TendArgsT::fshift1)
                store_row_with_ghosts<T, EDGE>(fs1 + orow, IN_ROWS ? nullptr : ghost_row_target(fs1, ld, P, j, gr), M, i, f1c);
                store_row_with_ghosts<T, EDGE>(fs2 + orow, IN_ROWS ? nullptr : ghost_row_target(fs2, ld, P, j, gr), M, i, f2c);
            }
            if constexpr (CERT) {  // this layer's parts of b_s and r_s at (i, j)
                double part[4];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const double b = -(a.cert_in[2 * s + layer] * (double)zcen);
                    part[2 * s] = b;
                    part[2 * s + 1] = b + a.cert_pinv[2 * s + layer] * ((double)L0[cl] + a.cert_alpha[s] * (double)P0[cp]);
                }
                if (layer == 1) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) xch[j & 1][k][t] = part[k];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) pend[k] = part[k];
                    pend_j = j;
                }
            }
        }
        // the next row: ring slots rotate by one, row pointers advance by one row
        {
            const LT p0 = rP[0], z0 = rZ[0], l0 = rL[0];
#pragma unroll
            for (int k = 0; k + 1 < RP; ++k) rP[k] = rP[k + 1];
#pragma unroll
            for (int k = 0; k + 1 < RZ; ++k) rZ[k] = rZ[k + 1];
#pragma unroll
            for (int k = 0; k + 1 < RL; ++k) rL[k] = rL[k + 1];
            rP[RP - 1] = p0;
            rZ[RZ - 1] = z0;
            rL[RL - 1] = l0;
        }
        nP += ld;
        nZ += ld;
        nF += ld;
        oRow += ld;
    }
    if constexpr (CERT) {
        __syncthreads();
        if (layer == 0) cert_fold();
        // workgroup sums (layer-1 waves add zeros), fixed order
        __shared__ double sv[4][2 * TX / 64];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double v = cv[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == 0) sv[k][w] = v;
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            double v = 0;
            for (int g = 0; g < 2 * TX / 64; ++g) v += sv[threadIdx.x][g];
            a.cert[4 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) + threadIdx.x] = v;
        }
    }
}

template <int TX, int PF, class T, bool CERT = false>
__global__ __launch_bounds__(CERT ? 2 * TX : TX, (CERT || TX >= 512) ? 4 : 5) void tendency_kernel(TendArgsT<T> a, int nyA, int nyB) {
    constexpr int RP = 6, RZ = 5, RL = 4;  // ring depths
    constexpr int NL = CERT ? 2 : 1;       // layers per workgroup
    const TendBlock tb = tend_block();
    // (wave-uniform: TX is a whole number of waves; in an SGPR the per-layer pointers stay
    // scalar loads -- a per-lane index made them vector loads, re-issued every row)
    const int layer = CERT ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x / TX)) : tb.z;
    const int t = CERT ? (int)(threadIdx.x % TX) : (int)threadIdx.x;
    const int M = (int)a.M;
    const int x0 = tb.x * TX;
    // strip rows: range A = [j0, j1) split evenly over nyA workgroups along y, then range B
    const int y = tb.y;
    const bool second = y >= nyA;
    const int r0 = second ? a.j2 : a.j0, nr = second ? a.j3 - a.j2 : a.j1 - a.j0;
    const int yy = second ? y - nyA : y, ny = second ? nyB : nyA;
    const int jb0 = r0 + (int)(((int64_t)yy * nr) / ny);
    const int jb1 = r0 + (int)(((int64_t)(yy + 1) * nr) / ny);
    if (jb0 >= jb1) {  // uniform over the block
        if constexpr (CERT) {
            if (threadIdx.x < 4) a.cert[4 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) + threadIdx.x] = 0;
        }
        return;
    }
    __shared__ T sp_[NL][RP][TX + 4];
    __shared__ T sz_[NL][RZ][TX + 2];
    __shared__ T sl_[NL][RL][TX + 2];
    // CERT: layer 1's (b0, r0, b1, r1) contributions of row j, read by layer 0 after the next
    // barrier (double-buffered by row parity); layer 0 keeps its own for that row meanwhile
    __shared__ double xch[CERT ? 2 : 1][4][CERT ? TX : 1];
    const int L = CERT ? layer : 0;
    const bool in_rows = jb0 >= 2 && jb1 + 2 <= (int)a.P;  // (uniform) see tendency_strip
    if (x0 >= 2 && x0 + TX + 2 <= M) {  // (uniform) the x-halo inside the row
        if (in_rows) tendency_strip<TX, PF, T, CERT, false, true>(a, layer, t, x0, jb0, jb1, sp_[L], sz_[L], sl_[L], xch);
        else tendency_strip<TX, PF, T, CERT, false, false>(a, layer, t, x0, jb0, jb1, sp_[L], sz_[L], sl_[L], xch);
    } else {
        tendency_strip<TX, PF, T, CERT, true, false>(a, layer, t, x0, jb0, jb1, sp_[L], sz_[L], sl_[L], xch);
    }
}

// ------------------------------------------------------------------------------------
// Float32 tendency, two points per thread (register blocking).  With F32 fields the kernel
// above moves half the bytes but keeps its per-point LDS reads and per-row barrier, and is
// bound by those, not by HBM.  Here each thread owns the adjacent pair
// (x0 + 2t, x0 + 2t + 1): one 8-byte access per row and field (global and LDS), and the
// stencil neighbours of both points come from 4-wide register windows of each ring row.
// The arithmetic per point is tendency_kernel's, in the same order: bit-identical results.
// All rings carry an x-halo of 2, so every pair sits at an even (8-byte aligned) LDS index.
// ------------------------------------------------------------------------------------
// pair types: V = 2 elements at an LDS pair (aligned to 2 elements), VU = 2 elements in a
// field row (interior rows start at element 1: aligned to one element only)
template <class T>
struct PairT;
template <>
struct PairT<float> {
    typedef float V __attribute__((ext_vector_type(2)));
    typedef float VU __attribute__((ext_vector_type(2), aligned(4)));
};
template <>
struct PairT<double> {
    typedef double V __attribute__((ext_vector_type(2)));
    typedef double VU __attribute__((ext_vector_type(2), aligned(8)));
};

// store the pair (xa, xa+1) of row j with its periodic images (store_row_with_ghosts x 2);
// EDGE = false: a pair of an interior strip (both points in range, neither column 0 nor M-1)
template <class T, bool EDGE = true>
__device__ __forceinline__ void store_pair_with_ghosts(T *row, T *grow, int M, int xa, T v0, T v1, bool has_b) {
    using VU = typename PairT<T>::VU;
    auto put = [&](T *r) {
        if constexpr (!EDGE) {
            *(VU *)(r + xa + 1) = VU{v0, v1};
            return;
        }
        if (has_b) {
            *(VU *)(r + xa + 1) = VU{v0, v1};
            if (xa + 1 == M - 1) r[0] = v1;
        } else {
            r[xa + 1] = v0;
            if (xa == M - 1) r[0] = v0;
        }
        if (xa == 0) r[M + 1] = v0;
    };
    put(row);
    if (grow) put(grow);
}

// One strip of the pair kernel.  EDGE = false (every strip whose x-halo lies inside the row:
// all but the first and the last): no periodic wrap of column indices, every pair in range,
// no ghost-column stores -- the interior strips' row loop is straight-line code except for
// the halo lanes.  EDGE = true: the general form (wraps, partial pairs, ghost columns).
// IN_ROWS and the scalar bookkeeping (rotated ring slots, induction row pointers, arguments
// read once): see tendency_strip.
template <int TX, class T, int PF, bool EDGE, bool IN_ROWS>
__device__ __forceinline__ void tendency_pair_strip(const TendArgsT<T> &a, int layer, int x0, int jb0, int jb1,
                                                    T (*sp)[2 * TX + 4], T (*sz)[2 * TX + 4], T (*sl)[2 * TX + 4]) {
    using V = typename PairT<T>::V;
    using VU = typename PairT<T>::VU;
    constexpr int RP = 6, RZ = 5, RL = 4, W = 2 * TX;
    const int t = threadIdx.x;
    const int M = (int)a.M, P = (int)a.P;
    const int64_t ld = a.ld;
    const int xa = x0 + 2 * t;  // own points xa, xa + 1

    const T *psi = a.psi[layer];
    const T *zeta = a.zeta[layer];
    const RowSrcT<T> &prs = a.psi_rows[layer];
    const RowSrcT<T> &zrs = a.zeta_rows[layer];
    // the arguments the row loop uses, read once
    const T *const fp1 = a.fprev1[layer], *const fp2 = a.fprev2[layer];
    T *const zo = a.zeta_out[layer], *const fo = a.f_out[layer];
    T *const fs1 = a.fshift1[layer], *const fs2 = a.fshift2[layer];
    const double *const wind = layer == 0 ? a.wind : nullptr;  // wind extension (off: nullptr)
    const bool gr = a.write_ghost_rows != 0;
    const T dx = (T)a.dx, idx = T(1) / dx, idx2 = idx * idx;
    const T cdc = T(0.5) * idx;
    const T den = T(12) * (dx * dx);
    const T visc = (T)a.visc, dtT = (T)a.dt, Ut = (T)a.U, rt = (T)a.r;
    const bool small = M < W + 4;

    auto wx = [&](int x) -> int {
        if constexpr (!EDGE) return x;
        if (small) return ((x % M) + M) % M;
        return x < 0 ? x + M : (x >= M ? x - M : x);
    };
    auto rowp = [&](const T *base, const RowSrcT<T> &rs, int j) -> const T * {
        if (IN_ROWS || (j >= 0 && j < P)) return base + fidx(1, j + 1, ld);
        return rs.halo[j < 0 ? j + 2 : (j - P) + 2];
    };
    const int hq = t == 0 ? 0 : (t == TX - 1 ? W + 2 : -1);  // halo pair LDS index, or none
    const int xh = t == 0 ? x0 - 2 : x0 + W;
    const bool has_a = !EDGE || xa < M, has_b = !EDGE || xa + 1 < M;
    const bool ab3 = a.ab3 != 0;
    const int c0 = 2 * t + 2;  // LDS index of xa

    auto load_pair = [&](const T *r, V &c) {
        if (has_b) {
            const VU v = *(const VU *)(r + xa);
            c = V{v.x, v.y};
        } else {
            c = V{r[wx(xa)], r[wx(xa + 1)]};
        }
    };
    auto load_halo = [&](const T *r, V &h) {
        if constexpr (EDGE) {
            if (hq >= 0) h = V{r[wx(xh)], r[wx(xh + 1)]};
        } else if (hq >= 0) {
            const VU v = *(const VU *)(r + xh);
            h = V{v.x, v.y};
        }
    };
    // ring slots of the rows the iteration j uses (LDS-typed: 32-bit addresses): rP[k] = psi
    // row j-2+k, rZ[k] = zeta row j-1+k, rL[k] = lap row j-1+k; rotated by one every row
    typedef __attribute__((address_space(3))) T *LT;
    LT rP[RP], rZ[RZ], rL[RL];
#pragma unroll
    for (int k = 0; k < RP; ++k) rP[k] = (LT)sp[(jb0 - 2 + k + 2 * RP) % RP];
#pragma unroll
    for (int k = 0; k < RZ; ++k) rZ[k] = (LT)sz[(jb0 - 1 + k + 2 * RZ) % RZ];
#pragma unroll
    for (int k = 0; k < RL; ++k) rL[k] = (LT)sl[(jb0 - 1 + k + 2 * RL) % RL];
    // Ring rows of interior strips 16 B per lane: threads [0, TX/2) read the psi row, [TX/2, TX)
    // the zeta row, each as (W + 4) / Q vectors of Q elements (x0-2 .. x0+W+1); threads 0 and
    // TX/2 take the one vector left over each.  One 16-byte load and LDS store per lane and row
    // instead of two 8-byte ones (a wave's row access touches 9 cache lines per KB instead of
    // 10 at the rows' element-1 offset): 8192^2 F32 738 -> 725 us (r04h, same box; the walk
    // alone 0.320 -> 0.311 ms, tools/microbench/strip_width.hip).  The same form for the F64
    // one-point kernel measured 334.5 -> 336.7 us and is not used.  Ring contents unchanged.
    constexpr int Q = 16 / sizeof(T);
    constexpr bool R16 = !EDGE && (W + 4) % Q == 0 && (W + 4) / Q == TX / 2 + 1;
    typedef T VQ __attribute__((ext_vector_type(Q)));                         // LDS (16-B aligned)
    typedef T VQU __attribute__((ext_vector_type(Q), aligned(sizeof(T))));  // row (element-1 offset)
    const bool is_psi = t < TX / 2;  // (wave-uniform for TX % 128 == 0)
    const int vq = is_psi ? t : t - TX / 2;
    const bool xtra = t == 0 || t == TX / 2;  // vector TX/2 of its row
    auto fetch16 = [&](const T *rp, const T *rz, VQ &c, VQ &e) {  // (rows' interior element 0)
        const T *r = (is_psi ? rp : rz) + (x0 - 2);
        c = *(const VQU *)(r + Q * vq);
        if (xtra) e = *(const VQU *)(r + Q * (TX / 2));
    };
    auto commit16 = [&](LT dp, LT dz, VQ c, VQ e) {
        const LT d = is_psi ? dp : dz;
        *(__attribute__((address_space(3))) VQ *)(d + Q * vq) = c;
        if (xtra) *(__attribute__((address_space(3))) VQ *)(d + Q * (TX / 2)) = e;
    };

    // prefetch pipeline PF rows deep: slot 0 is consumed next
    V pc[PF], ph[PF], zc[PF], zh[PF], f1[PF], f2[PF];
    VQ rc[PF], re[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        pc[k] = ph[k] = zc[k] = zh[k] = f1[k] = f2[k] = V{0, 0};
        rc[k] = re[k] = VQ{};
    }
    auto fetch_pair_row = [&](const T *r, V &c, V &h) {
        load_pair(r, c);
        load_halo(r, h);
    };
    auto fetch_f = [&](size_t o, V &g1, V &g2) {  // o: element offset of the row's interior element 0
        if (ab3 && has_a) {
            const T *p1 = fp1 + o, *p2 = fp2 + o;
            if (has_b) {
                const VU u1 = *(const VU *)(p1 + xa), u2 = *(const VU *)(p2 + xa);
                g1 = V{u1.x, u1.y};
                g2 = V{u2.x, u2.y};
            } else {
                g1.x = p1[xa];
                g2.x = p2[xa];
            }
        }
    };
    auto commit = [&](LT d, V c, V h) {
        *(__attribute__((address_space(3))) V *)(d + c0) = c;
        if (hq >= 0) *(__attribute__((address_space(3))) V *)(d + hq) = h;
    };
    auto lap_row = [&](LT pm, LT p0, LT pp, LT dst) {  // lap(psi) at x0-1 .. x0+W (LDS 1 .. W+2)
        typedef __attribute__((address_space(3))) V *LV;
        const V a0 = *(LV)(p0 + c0 - 2), a1 = *(LV)(p0 + c0), a2 = *(LV)(p0 + c0 + 2);
        const V m = *(LV)(pm + c0), p = *(LV)(pp + c0);
        V r;
        r.x = ((((a0.y + a1.y) - T(4) * a1.x) + m.x) + p.x) * idx2;
        r.y = ((((a1.x + a2.x) - T(4) * a1.y) + m.y) + p.y) * idx2;
        *(LV)(dst + c0) = r;
        if (t == 0) dst[1] = ((((p0[0] + p0[2]) - T(4) * p0[1]) + pm[1]) + pp[1]) * idx2;
        if (t == TX - 1)
            dst[W + 2] = ((((p0[W + 1] + p0[W + 3]) - T(4) * p0[W + 2]) + pm[W + 2]) + pp[W + 2]) * idx2;
    };

    // prologue: psi rows jb0-2..jb0+2, zeta rows jb0-1..jb0+1 into LDS, every load issued
    // before the first LDS write (see tendency_kernel)
    if constexpr (R16) {
        VQ q0c[5], q0e[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            q0c[k] = q0e[k] = VQ{};
            if (is_psi || k < 3) fetch16(rowp(psi, prs, jb0 - 2 + k), rowp(zeta, zrs, jb0 - 1 + k), q0c[k], q0e[k]);
        }
#pragma unroll
        for (int k = 0; k < 5; ++k)
            if (is_psi || k < 3) commit16(rP[k], rZ[k], q0c[k], q0e[k]);
    } else {
        V p0c[5], p0h[5], z0c[3], z0h[3];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            p0c[k] = p0h[k] = V{0, 0};
            fetch_pair_row(rowp(psi, prs, jb0 - 2 + k), p0c[k], p0h[k]);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            z0c[k] = z0h[k] = V{0, 0};
            fetch_pair_row(rowp(zeta, zrs, jb0 - 1 + k), z0c[k], z0h[k]);
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) commit(rP[k], p0c[k], p0h[k]);
#pragma unroll
        for (int k = 0; k < 3; ++k) commit(rZ[k], z0c[k], z0h[k]);
    }
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int j = jb0 + k;
        if (j + 2 <= jb1) {
            if constexpr (R16) {
                fetch16(rowp(psi, prs, j + 3), rowp(zeta, zrs, j + 2), rc[k], re[k]);
            } else {
                fetch_pair_row(rowp(psi, prs, j + 3), pc[k], ph[k]);
                fetch_pair_row(rowp(zeta, zrs, j + 2), zc[k], zh[k]);
            }
        }
        if (j < jb1) fetch_f((size_t)(j + 1) * ld + 1, f1[k], f2[k]);
    }
    __syncthreads();
    lap_row(rP[0], rP[1], rP[2], rL[0]);
    lap_row(rP[1], rP[2], rP[3], rL[1]);
    lap_row(rP[2], rP[3], rP[4], rL[2]);

    // IN_ROWS row pointers: the next fetch (iteration j + PF) and this row's outputs
    const T *nP = psi + fidx(1, jb0 + PF + 3 + 1, ld), *nZ = zeta + fidx(1, jb0 + PF + 2 + 1, ld);
    size_t nF = (size_t)(jb0 + PF + 1) * ld + 1;
    size_t oRow = (size_t)(jb0 + 1) * ld;

    const T bl = (T)a.beta[layer];
    for (int j = jb0; j < jb1; ++j) {
        const bool more = j + 2 <= jb1;
        if (more) {
            if constexpr (R16) {
                commit16(rP[5], rZ[3], rc[0], re[0]);
            } else {
                commit(rP[5], pc[0], ph[0]);
                commit(rZ[3], zc[0], zh[0]);
            }
        }
        const V f1c = f1[0], f2c = f2[0];
        asm volatile("" : : "v"(f1c), "v"(f2c) : "memory");  // (see tendency_kernel)
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) {
            pc[k] = pc[k + 1];
            ph[k] = ph[k + 1];
            zc[k] = zc[k + 1];
            zh[k] = zh[k + 1];
            rc[k] = rc[k + 1];
            re[k] = re[k + 1];
            f1[k] = f1[k + 1];
            f2[k] = f2[k + 1];
        }
        {
            const int jn = j + PF;  // iteration whose inputs are fetched now
            if (jn + 2 <= jb1) {
                const T *rp = IN_ROWS ? nP : rowp(psi, prs, jn + 3), *rz = IN_ROWS ? nZ : rowp(zeta, zrs, jn + 2);
                if constexpr (R16) {
                    fetch16(rp, rz, rc[PF - 1], re[PF - 1]);
                } else {
                    fetch_pair_row(rp, pc[PF - 1], ph[PF - 1]);
                    fetch_pair_row(rz, zc[PF - 1], zh[PF - 1]);
                }
            }
            if (jn < jb1) fetch_f(IN_ROWS ? nF : (size_t)(jn + 1) * ld + 1, f1[PF - 1], f2[PF - 1]);
        }
        __syncthreads();
        if (more) lap_row(rP[3], rP[4], rP[5], rL[3]);
        if (has_a) {
            typedef __attribute__((address_space(3))) V *LV;
            // 4-wide windows (LDS c0-1 .. c0+2) of the zeta / psi rows j-1, j, j+1 and lap row j;
            // lap rows j-1, j+1 at the pair only
            T Zw[3][4], Sw[3][4], L0w[4];
            const LT zr[3] = {rZ[0], rZ[1], rZ[2]};
            const LT pr[3] = {rP[1], rP[2], rP[3]};
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const V u0 = *(LV)(zr[r] + c0 - 2), u1 = *(LV)(zr[r] + c0), u2 = *(LV)(zr[r] + c0 + 2);
                Zw[r][0] = u0.y; Zw[r][1] = u1.x; Zw[r][2] = u1.y; Zw[r][3] = u2.x;
                const V s0 = *(LV)(pr[r] + c0 - 2), s1 = *(LV)(pr[r] + c0), s2 = *(LV)(pr[r] + c0 + 2);
                Sw[r][0] = s0.y; Sw[r][1] = s1.x; Sw[r][2] = s1.y; Sw[r][3] = s2.x;
            }
            const LT l0 = rL[1];
            {
                const V u0 = *(LV)(l0 + c0 - 2), u1 = *(LV)(l0 + c0), u2 = *(LV)(l0 + c0 + 2);
                L0w[0] = u0.y; L0w[1] = u1.x; L0w[2] = u1.y; L0w[3] = u2.x;
            }
            const V Lm = *(LV)(rL[0] + c0), Lp = *(LV)(rL[2] + c0);
            T out_z[2], out_f[2];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int w = 1 + v;  // window index of the point
                const T lm = v ? Lm.y : Lm.x, lp = v ? Lp.y : Lp.x;
                const T biharm = ((((L0w[w - 1] + L0w[w + 1]) - T(4) * L0w[w]) + lm) + lp) * idx2;
                const T v_term = visc * biharm;
                auto Z = [&](int da, int db) { return Zw[db + 1][w + da]; };
                auto S = [&](int da, int db) { return Sw[db + 1][w + da]; };
                const T J_term = arakawa_point<T>(Z, S, den);
                const T beta_term = bl * (cdc * (Sw[1][w + 1] - Sw[1][w - 1]));
                T last;
                if (layer == 0) last = Ut * (cdc * (Zw[1][w + 1] - Zw[1][w - 1]));
                else last = rt * L0w[w];
                T F = ((v_term - J_term) - beta_term) - last;
                if (wind) F = F + (T)wind[j];
                const T zcen = Zw[1][w];
                const T g1 = v ? f1c.y : f1c.x, g2 = v ? f2c.y : f2c.x;
                out_z[v] = ab3 ? zcen + dtT * ((((T)(23.0 / 12.0) * F) - ((T)(16.0 / 12.0) * g1)) + ((T)(5.0 / 12.0) * g2))
                               : zcen + (dtT * F);
                out_f[v] = F;
            }
            const size_t orow = IN_ROWS ? oRow : (size_t)(j + 1) * ld;
            store_pair_with_ghosts<T, EDGE>(zo + orow, IN_ROWS ? nullptr : ghost_row_target(zo, ld, P, j, gr), M, xa,
                                            out_z[0], out_z[1], has_b);
            store_pair_with_ghosts<T, EDGE>(fo + orow, IN_ROWS ? nullptr : ghost_row_target(fo, ld, P, j, gr), M, xa,
                                            out_f[0], out_f[1], has_b);
            if (ab3 && fs1) {  // (see TendArgsT::fshift1)
                store_pair_with_ghosts<T, EDGE>(fs1 + orow, IN_ROWS ? nullptr : ghost_row_target(fs1, ld, P, j, gr), M,
                                                xa, f1c.x, f1c.y, has_b);
                store_pair_with_ghosts<T, EDGE>(fs2 + orow, IN_ROWS ? nullptr : ghost_row_target(fs2, ld, P, j, gr), M,
                                                xa, f2c.x, f2c.y, has_b);
            }
        }
        // the next row: ring slots rotate by one, row pointers advance by one row
        {
            const LT p0 = rP[0], z0 = rZ[0], l0 = rL[0];
#pragma unroll
            for (int k = 0; k + 1 < RP; ++k) rP[k] = rP[k + 1];
#pragma unroll
            for (int k = 0; k + 1 < RZ; ++k) rZ[k] = rZ[k + 1];
#pragma unroll
            for (int k = 0; k + 1 < RL; ++k) rL[k] = rL[k + 1];
            rP[RP - 1] = p0;
            rZ[RZ - 1] = z0;
            rL[RL - 1] = l0;
        }
        nP += ld;
        nZ += ld;
        nF += ld;
        oRow += ld;
    }
}

// PF: register prefetch depth in rows (as tendency_kernel's)
template <int TX, class T, int PF = 1>
__global__ __launch_bounds__(TX) void tendency_pair_kernel(TendArgsT<T> a, int nyA, int nyB) {
    constexpr int RP = 6, RZ = 5, RL = 4, W = 2 * TX, WL = W + 4;
    const TendBlock tb = tend_block();
    const int M = (int)a.M;
    const int x0 = tb.x * W;
    const int y = tb.y;
    const bool second = y >= nyA;
    const int r0 = second ? a.j2 : a.j0, nr = second ? a.j3 - a.j2 : a.j1 - a.j0;
    const int yy = second ? y - nyA : y, ny = second ? nyB : nyA;
    const int jb0 = r0 + (int)(((int64_t)yy * nr) / ny);
    const int jb1 = r0 + (int)(((int64_t)(yy + 1) * nr) / ny);
    if (jb0 >= jb1) return;  // uniform over the block
    __shared__ __attribute__((aligned(16))) T sp[RP][WL];
    __shared__ __attribute__((aligned(16))) T sz[RZ][WL];
    __shared__ __attribute__((aligned(16))) T sl[RL][WL];
    const bool in_rows = jb0 >= 2 && jb1 + 2 <= (int)a.P;  // (uniform) see tendency_strip
    if (x0 >= 2 && x0 + W + 2 <= M) {  // (uniform) the x-halo inside the row
        if (in_rows) tendency_pair_strip<TX, T, PF, false, true>(a, tb.z, x0, jb0, jb1, sp, sz, sl);
        else tendency_pair_strip<TX, T, PF, false, false>(a, tb.z, x0, jb0, jb1, sp, sz, sl);
    } else {
        tendency_pair_strip<TX, T, PF, true, false>(a, tb.z, x0, jb0, jb1, sp, sz, sl);
    }
}

// ------------------------------------------------------------------------------------
// Seeded initialise_model: psi and zeta of slot 0, ghosts included, computed directly at
// the wrapped GLOBAL index (so slabs need no communication).  model.jl:37-62.
// ------------------------------------------------------------------------------------
template <class T>  // computed in F64 (the reference's values), stored as T
__global__ void initialise_kernel(T *zeta, T *psi, int64_t M, int64_t P, int64_t P_total,
                                  int64_t j_offset, double amp, double S1, double S2, double idx2,
                                  uint64_t seed1, uint64_t seed2) {
    const int64_t mi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // memory index incl ghosts
    const int64_t mj = blockIdx.y;
    if (mi >= M + 2) return;
    const int64_t ld = M + 2;
    auto gi = [&](int64_t x) { return ((x % M) + M) % M; };
    auto gj = [&](int64_t y) { return ((y % P_total) + P_total) % P_total; };
    auto psi_at = [&](uint64_t seed, int64_t x, int64_t y) {  // interior coords, wrapped
        return amp * u01(seed, (uint64_t)gi(x) + (uint64_t)M * (uint64_t)gj(y));
    };
    const int64_t x = mi - 1, y = mj - 1 + j_offset;
    const double p1 = psi_at(seed1, x, y), p2 = psi_at(seed2, x, y);
    auto lap = [&](uint64_t seed) {
        return ((((psi_at(seed, x - 1, y) + psi_at(seed, x + 1, y)) - 4 * psi_at(seed, x, y)) +
                 psi_at(seed, x, y - 1)) + psi_at(seed, x, y + 1)) * idx2;
    };
    const size_t o = fidx(mi, mj, ld);
    const size_t F = (size_t)(M + 2) * (size_t)(P + 2);
    psi[o] = (T)p1;
    psi[F + o] = (T)p2;
    zeta[o] = (T)(lap(seed1) + S1 * (p2 - p1));
    zeta[F + o] = (T)(lap(seed2) + S2 * (p1 - p2));
}

// ------------------------------------------------------------------------------------
// Slot moves of up to three (M+2, P+2, 2, 3) history arrays in one launch (blockIdx.y =
// array), in place: new slot s <- old slot src[s] (-1: slot s is left alone).  Slots are
// contiguous blocks of `n16` 16-byte vectors (2 layers x (M+2)(P+2) elements: a multiple of
// 16 B for F64, and for F32 since M is even).  Each element's sources are read into
// registers before any of its destinations is written, by the same thread, so any
// permutation of the three slots is safe.  Two uses:
//   store_new_state!'s shift (model.jl:102-106: X[:,:,:,3] .= X[:,:,:,2]; X[:,:,:,2] .=
//     X[:,:,:,1]): src = {-1, 0, 1}, 2 reads + 2 writes per element, slot 1 left for the
//     new values;
//   qg_canonicalize's rotation of a field whose newest slot is physical h: src = {h, h+1,
//     h+2} mod 3, each slot read once and written once.
// ------------------------------------------------------------------------------------
struct SlotMoveArgs {
    uint4 *base[3];
    int src[3][3];
    int64_t n16;
};

// One vector per thread and slot, non-temporal stores (tools/microbench/slot_shift.hip, two
// 4096^2 F64 arrays shifted: 5.7 TB/s of reads + writes; 4 vectors per thread with all loads
// first 4.5, grid-stride loops 4.7-5.2, plain stores 5.5, hipMemcpyAsync pairs 5.4)
typedef unsigned int SlotVec __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void slot_move_kernel(SlotMoveArgs a) {
    const int k = blockIdx.y;
    SlotVec *b = reinterpret_cast<SlotVec *>(a.base[k]);
    const int s0 = a.src[k][0], s1 = a.src[k][1], s2 = a.src[k][2];
    const int64_t n = a.n16;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    SlotVec v[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
        if (s0 == q || s1 == q || s2 == q) v[q] = b[q * n + i];
    if (s0 >= 0) __builtin_nontemporal_store(v[s0], b + i);
    if (s1 >= 0) __builtin_nontemporal_store(v[s1], b + n + i);
    if (s2 >= 0) __builtin_nontemporal_store(v[s2], b + 2 * n + i);
}

int launch_slot_move(void *const *arrays, const int (*src)[3], int narrays, size_t slot_bytes, hipStream_t s) {
    if (narrays < 1 || narrays > 3 || slot_bytes % 16 != 0) return QG_ERR_INVALID_ARG;
    SlotMoveArgs a{};
    for (int k = 0; k < narrays; ++k) {
        if (reinterpret_cast<uintptr_t>(arrays[k]) % 16 != 0) return QG_ERR_INVALID_ARG;
        a.base[k] = static_cast<uint4 *>(arrays[k]);
        for (int q = 0; q < 3; ++q) {
            if (src[k][q] < -1 || src[k][q] > 2) return QG_ERR_INVALID_ARG;
            a.src[k][q] = src[k][q];
        }
    }
    a.n16 = (int64_t)(slot_bytes / 16);
    const int64_t gx = (a.n16 + 255) / 256;
    if (gx > 0x7fffffff) return QG_ERR_UNSUPPORTED;
    slot_move_kernel<<<dim3((unsigned)std::max<int64_t>(gx, 1), (unsigned)narrays), 256, 0, s>>>(a);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static dim3 grid_rows(int64_t M, int64_t P, int bs) { return dim3((unsigned)((M + bs - 1) / bs), (unsigned)P); }

int launch_laplace(const double *u, double *out, int64_t M, int64_t P, double dx, hipStream_t s) {
    const double i = 1.0 / dx;
    laplace_kernel<<<grid_rows(M, P, 256), 256, 0, s>>>(u, out, M, P, i * i);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

int launch_cd(const double *u, double *out, int64_t M, int64_t P, double dx, hipStream_t s) {
    cd_kernel<<<grid_rows(M, P, 256), 256, 0, s>>>(u, out, M, P, 0.5 * (1.0 / dx));
    QG_LAUNCH_CHECK();
    return QG_OK;
}

int launch_arakawa(const double *z, const double *p, double *out, int64_t M, int64_t P, double dx,
                   hipStream_t s) {
    arakawa_kernel<<<grid_rows(M, P, 256), 256, 0, s>>>(z, p, out, M, P, 12 * (dx * dx));
    QG_LAUNCH_CHECK();
    return QG_OK;
}

int launch_fill_ghosts(double *b, int64_t M, int64_t P, hipStream_t s) {
    const int64_t n = M > P ? M : P;
    fill_ghosts_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(b, M, P, 1);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

int launch_fill_ghost_cols(double *b, int64_t M, int64_t P, hipStream_t s) {
    fill_ghosts_kernel<<<(unsigned)((P + 255) / 256), 256, 0, s>>>(b, M, P, 0);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// ------------------------------------------------------------------------------------
// Cache-resident tendency (small grids).  When every field of the step fits in the 256 MB
// MALL, the LDS-ring kernel above spends most of its time in the ring prologue and the
// per-row barriers of short strips.  Here each thread computes one output point straight
// from global memory: the 13-point psi diamond, the 3x3 zeta block and F(t-1), F(t-2), the
// neighbours' re-reads served by L1/L2/MALL; no LDS, no barriers.  Same expressions in the
// same order as tendency_kernel (lap at the five points, then the biharmonic), so the two
// kernels are bit-identical.  Block: 64 x-points (one wave) x 4 rows.
// ------------------------------------------------------------------------------------
// one point (i, j) of one layer: loads, tendency, AB3 update, stores; returns the centre
// values the certification uses (zeta, lap(psi), psi)
template <class T>
__device__ __forceinline__ void direct_point(const TendArgsT<T> &a, int layer, int i, int j, T &zc_out, T &L0_out,
                                             T &P0_out) {
    const int M = (int)a.M, P = (int)a.P;
    const int64_t ld = a.ld;
    const T *psi = a.psi[layer], *zeta = a.zeta[layer];
    const RowSrcT<T> &prs = a.psi_rows[layer];
    const RowSrcT<T> &zrs = a.zeta_rows[layer];
    const T dx = (T)a.dx, idx = T(1) / dx, idx2 = idx * idx;
    const T cdc = T(0.5) * idx;
    const T den = T(12) * (dx * dx);
    const T visc = (T)a.visc, dtT = (T)a.dt, Ut = (T)a.U, rt = (T)a.r;
    const bool small = M < 8;
    auto wx = [&](int x) -> int {
        if (small) return ((x % M) + M) % M;
        return x < 0 ? x + M : (x >= M ? x - M : x);
    };
    auto rowp = [&](const T *base, const RowSrcT<T> &rs, int jj) -> const T * {
        if (jj >= 0 && jj < P) return base + fidx(1, jj + 1, ld);
        return rs.halo[jj < 0 ? jj + 2 : (jj - P) + 2];
    };
    const T *pr[5], *zr[3];
#pragma unroll
    for (int d = 0; d < 5; ++d) pr[d] = rowp(psi, prs, j - 2 + d);
#pragma unroll
    for (int d = 0; d < 3; ++d) zr[d] = rowp(zeta, zrs, j - 1 + d);
    const int xm2 = wx(i - 2), xm1 = wx(i - 1), xp1 = wx(i + 1), xp2 = wx(i + 2);
    auto X = [&](int da) { return da == -2 ? xm2 : da == -1 ? xm1 : da == 0 ? i : da == 1 ? xp1 : xp2; };
    auto S = [&](int da, int db) { return pr[db + 2][X(da)]; };
    auto Z = [&](int da, int db) { return zr[db + 1][X(da)]; };
    auto lap = [&](int da, int db) {  // lap_row's expression at (i + da, j + db)
        return ((((S(da - 1, db) + S(da + 1, db)) - T(4) * S(da, db)) + S(da, db - 1)) + S(da, db + 1)) * idx2;
    };
    const T L0 = lap(0, 0);
    const T biharm = ((((lap(-1, 0) + lap(1, 0)) - T(4) * L0) + lap(0, -1)) + lap(0, 1)) * idx2;
    const T v_term = visc * biharm;
    const T J_term = arakawa_point<T>(Z, S, den);
    const T bl = (T)a.beta[layer];
    const T beta_term = bl * (cdc * (S(1, 0) - S(-1, 0)));
    T last;
    if (layer == 0) last = Ut * (cdc * (Z(1, 0) - Z(-1, 0)));
    else last = rt * L0;
    T F = ((v_term - J_term) - beta_term) - last;
    if (layer == 0 && a.wind) F = F + (T)a.wind[j];
    const T zcen = Z(0, 0);
    T zn, f1c = 0, f2c = 0;
    if (a.ab3) {
        const size_t o = (size_t)(j + 1) * ld + i + 1;
        f1c = ld_stream(a.fprev1[layer] + o);
        f2c = ld_stream(a.fprev2[layer] + o);
        zn = zcen + dtT * ((((T)(23.0 / 12.0) * F) - ((T)(16.0 / 12.0) * f1c)) + ((T)(5.0 / 12.0) * f2c));
    } else {
        zn = zcen + (dtT * F);
    }
    T *zo = a.zeta_out[layer], *fo = a.f_out[layer];
    const bool gr = a.write_ghost_rows;
    store_row_with_ghosts(zo + (size_t)(j + 1) * ld, ghost_row_target(zo, ld, P, j, gr), M, i, zn);
    store_row_with_ghosts(fo + (size_t)(j + 1) * ld, ghost_row_target(fo, ld, P, j, gr), M, i, F);
    if (a.ab3 && a.fshift1[layer]) {  // (see TendArgsT::fshift1)
        T *s1 = a.fshift1[layer], *s2 = a.fshift2[layer];
        store_row_with_ghosts(s1 + (size_t)(j + 1) * ld, ghost_row_target(s1, ld, P, j, gr), M, i, f1c);
        store_row_with_ghosts(s2 + (size_t)(j + 1) * ld, ghost_row_target(s2, ld, P, j, gr), M, i, f2c);
    }
    zc_out = zcen;
    L0_out = L0;
    P0_out = S(0, 0);
}

template <class T>
__global__ __launch_bounds__(256) void tendency_direct_kernel(TendArgsT<T> a, int nyA, int nyB) {
    const TendBlock tb = tend_block();
    const int layer = tb.z;
    const int M = (int)a.M;
    const int i = tb.x * 64 + (int)(threadIdx.x & 63);
    const int w = (int)(threadIdx.x >> 6);
    const int y = tb.y;
    const bool second = y >= nyA;
    const int r0 = second ? a.j2 : a.j0, r1 = second ? a.j3 : a.j1;
    const int j = r0 + 4 * (second ? y - nyA : y) + w;
    if (i >= M || j >= r1) return;  // no barriers below
    T zc, L0, P0;
    direct_point(a, layer, i, j, zc, L0, P0);
}

// The certifying form of the cache-resident kernel (PCG, one rank, small grids): each thread
// steps both layers of its point and forms the previous solve's residual terms there
// (tendency_kernel<CERT>'s per-point parts, layer 0's first); (b,b), (r,r) per block.
__global__ __launch_bounds__(256) void tendency_direct_cert_kernel(TendArgsT<double> a, int nyA, int nyB) {
    const TendBlock tb = tend_block();
    const int M = (int)a.M;
    const int i = tb.x * 64 + (int)(threadIdx.x & 63);
    const int w = (int)(threadIdx.x >> 6);
    const int y = tb.y;
    const bool second = y >= nyA;
    const int r0 = second ? a.j2 : a.j0, r1 = second ? a.j3 : a.j1;
    const int j = r0 + 4 * (second ? y - nyA : y) + w;
    double cv[4] = {0, 0, 0, 0};
    if (i < M && j < r1) {
        double part[2][4];
#pragma unroll
        for (int layer = 0; layer < 2; ++layer) {
            double zc, L0, P0;
            direct_point(a, layer, i, j, zc, L0, P0);
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const double b = -(a.cert_in[2 * s + layer] * zc);
                part[layer][2 * s] = b;
                part[layer][2 * s + 1] = b + a.cert_pinv[2 * s + layer] * (L0 + a.cert_alpha[s] * P0);
            }
        }
        double bs[2], rs[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bs[s] = part[0][2 * s] + part[1][2 * s];
            rs[s] = part[0][2 * s + 1] + part[1][2 * s + 1];
        }
        if (a.cert_pin && i == 0 && j == 0) bs[0] = rs[0] = 0.0;  // identity row: b = x = 0
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            cv[2 * s] = bs[s] * bs[s];
            cv[2 * s + 1] = rs[s] * rs[s];
        }
    }
    // block sums, fixed order (wave shuffles, then the four wave totals in order)
    __shared__ double sv[4][4];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double v = cv[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) sv[k][w] = v;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const double v = ((sv[threadIdx.x][0] + sv[threadIdx.x][1]) + sv[threadIdx.x][2]) + sv[threadIdx.x][3];
        a.cert[4 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) + threadIdx.x] = v;
    }
}

template <int TX, int PF, class T>
static int launch_tend_variant(const TendArgsT<T> &a, int rows, hipStream_t s) {
    const int nA = (a.j1 - a.j0 + rows - 1) / rows, nB = a.j3 > a.j2 ? (a.j3 - a.j2 + rows - 1) / rows : 0;
    dim3 grid((unsigned)((a.M + TX - 1) / TX), (unsigned)(nA + nB), 2);
    tendency_kernel<TX, PF, T><<<grid, TX, 0, s>>>(a, nA, nB);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// Resident workgroups per chip (CUs x per-CU occupancy) of a tendency kernel
template <class K>
static int tend_slots(K kernel, int threads, int &sl) {
    if (sl) return QG_OK;
    int dev = 0, cus = 0, per = 0;
    QG_HIP(hipGetDevice(&dev));
    QG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    QG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0));
    sl = cus * (per > 0 ? per : 1);
    return QG_OK;
}

// Default geometry: a whole number of chip-fulls of strips (CUs x resident workgroups per
// CU, from the occupancy API) -- a grid that is not a multiple leaves
// a partly idle last "wave" of workgroups -- with rows split evenly over the strips and at
// least 4 rows per strip.  (4096^2: 0.380 ms vs 0.385 for fixed 64-row strips; 1024^2: 33 vs
// 38 us.)
template <class T>
static int launch_tend_balanced(const TendArgsT<T> &a, hipStream_t s) {
    constexpr int TX = 256, PF = 1;  // register prefetch depth (rows)
    static int sl = 0;
    QG_CHECK(tend_slots(tendency_kernel<TX, PF, T>, TX, sl));
    const int nx = (int)((a.M + TX - 1) / TX);
    const int rA = a.j1 - a.j0, rB = a.j3 > a.j2 ? a.j3 - a.j2 : 0;
    // one chip-full of longer strips from ~1750^2 to ~3500^2 points: the ring prologue (6 rows
    // read before the first output row) then costs less than the idle tail of a second wave
    // (tile sweep, profiles/r01/tile_sweep_*.json: 2048^2 106 vs 111 us)
    const double pts = (double)a.M * (rA + rB);
    // six chip-fulls from ~3500^2 up: with the batched ring prologue a strip's start costs one
    // memory latency, and shorter strips keep the chip's concurrent accesses closer together
    // (tools/waves_sweep.sh, profiles/r02/prologue: 4096^2 3 -> 6 chip-fulls 341.7 -> 335 us,
    // 8192^2 4 -> 6 1 237-1 257 -> 1 230-1 241 us; before the prologue fix three and four).
    // Since the scalar-unit cuts (r04) a strip's start costs less and shorter walks pay:
    // 4096^2 6 -> 9 chip-fulls 328 -> 323 us, 8192^2 12 -> 16 1 339 -> 1 317 us (6: 1 300 vs
    // 12: 1 267 on another box; tools/r04_p.sh, profiles/r04/waves/)
    const int waves = pts >= 40.0e6 ? 16 : (pts >= 12.0e6 ? 9 : (pts >= 3.0e6 ? 1 : 2));
    const int target = std::max(1, waves * sl / (2 * nx));  // row workgroups per column strip
    auto split = [&](int rows) { return rows <= 0 ? 0 : std::max(1, std::min(rows / 4, (int)((int64_t)target * rows / (rA + rB)))); };
    const int nyA = split(rA), nyB = split(rB);
    dim3 grid((unsigned)nx, (unsigned)(nyA + nyB), 2);
    tendency_kernel<TX, PF, T><<<grid, TX, 0, s>>>(a, nyA, nyB);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// The certifying variant (PCG, one rank): both layers per workgroup, 128-point strips (256:
// 401 vs 398 us at 4096^2, same call), chip-fulls as above.
template <int TX>
static int launch_tendency_cert_t(const TendArgsT<double> &a, int64_t cap, int *nblk, hipStream_t s) {
    constexpr int PF = 1;
    static int sl = 0;
    if (sl == 0) {
        int dev = 0, cus = 0, per = 0;
        QG_HIP(hipGetDevice(&dev));
        QG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        QG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, tendency_kernel<TX, PF, double, true>, 2 * TX, 0));
        sl = cus * (per > 0 ? per : 1);
    }
    const int nx = (int)((a.M + TX - 1) / TX);
    const int rA = a.j1 - a.j0, rB = a.j3 > a.j2 ? a.j3 - a.j2 : 0;
    // three chip-fulls (tools/sweep_r02g.sh, 4096^2 with the batched prologue: 2 -> 3
    // 388.8 -> 385.1 us, 2 to 8 within 2 %; before it 2 was best, tools/cert_sweep.sh)
    const int waves = 3;
    const int target = std::max(1, waves * sl / nx);
    auto split = [&](int rows) { return rows <= 0 ? 0 : std::max(1, std::min(rows / 4, (int)((int64_t)target * rows / (rA + rB)))); };
    const int nyA = split(rA), nyB = split(rB);
    if (nyA + nyB == 0) {
        *nblk = 0;
        return QG_OK;
    }
    dim3 grid((unsigned)nx, (unsigned)(nyA + nyB), 1);
    if ((int64_t)grid.x * grid.y > cap) return QG_ERR_INVALID_ARG;
    tendency_kernel<TX, PF, double, true><<<grid, 2 * TX, 0, s>>>(a, nyA, nyB);
    QG_LAUNCH_CHECK();
    *nblk = (int)(grid.x * grid.y);
    return QG_OK;
}

// up to ~1100^2 (128^2 13.6 -> 7.4 us, 1024^2 33.2 -> 31.2; 1536^2 slower)
constexpr double TEND_DIRECT_PTS = 1.2e6;

// below this many points per layer the certifying tendency is the cache-resident one-point
// form (both layers per thread): 256^2 17.7 -> 13.9 us, 512^2 20.7 -> 18.7 us; at 1024^2 the
// two-layer ring form is faster (40.6 vs 43.1 us), so the cut sits below the plain
// tendency's TEND_DIRECT_PTS.  qg_set_form(QG_FORM_TENDENCY, ...) forces either form.
constexpr double CERT_DIRECT_PTS = 0.5e6;
int launch_tendency_cert(const TendArgsT<double> &a, int64_t cap, int *nblk, hipStream_t s) {
    const double pts = (double)a.M * ((a.j1 - a.j0) + (a.j3 > a.j2 ? a.j3 - a.j2 : 0));
    const int f = form(QG_FORM_TENDENCY);
    if (f == QG_TEND_DIRECT || (f != QG_TEND_RING && pts < CERT_DIRECT_PTS)) {
        const int nA = (a.j1 - a.j0 + 3) / 4, nB = a.j3 > a.j2 ? (a.j3 - a.j2 + 3) / 4 : 0;
        if (nA + nB == 0) {
            *nblk = 0;
            return QG_OK;
        }
        dim3 grid((unsigned)((a.M + 63) / 64), (unsigned)(nA + nB), 1);
        if ((int64_t)grid.x * grid.y > cap) return QG_ERR_INVALID_ARG;
        tendency_direct_cert_kernel<<<grid, 256, 0, s>>>(a, nA, nB);
        QG_LAUNCH_CHECK();
        *nblk = (int)(grid.x * grid.y);
        return QG_OK;
    }
    return launch_tendency_cert_t<128>(a, cap, nblk, s);
}

// Float32 default: the pair kernel over whole chip-fulls of 512-point strips (as above);
// qg_set_form(QG_FORM_TENDENCY, QG_TEND_ONE_POINT) selects the one-point kernel instead.
template <int TX, class T>
static int launch_tend_pair(const TendArgsT<T> &a, hipStream_t s) {
    constexpr int W = 2 * TX, PF = 1;
    static int sl = 0;
    QG_CHECK(tend_slots(tendency_pair_kernel<TX, T, PF>, TX, sl));
    const int nx = (int)((a.M + W - 1) / W);
    const double pts = (double)a.M * ((a.j1 - a.j0) + (a.j3 > a.j2 ? a.j3 - a.j2 : 0));
    // (tools/sweep_r02g.sh with the batched prologue: 8192^2 4 -> 6 chip-fulls 773 -> 764 us;
    // 4096^2 keeps 2: 209 vs 213-230 us.  r04, after the scalar-unit cuts: 8192^2 6 -> 12 -> 20
    // chip-fulls 652-719 -> 613-670 -> 646-652 us (12 -> 20 on one box: 663-668 -> 646-652),
    // tools/r04_p.sh, profiles/r04/waves/)
    const int waves = pts >= 40.0e6 ? 20 : 2;
    const int rA = a.j1 - a.j0, rB = a.j3 > a.j2 ? a.j3 - a.j2 : 0;
    const int target = std::max(1, waves * sl / (2 * nx));
    auto split = [&](int rows) { return rows <= 0 ? 0 : std::max(1, std::min(rows / 4, (int)((int64_t)target * rows / (rA + rB)))); };
    const int nyA = split(rA), nyB = split(rB);
    dim3 grid((unsigned)nx, (unsigned)(nyA + nyB), 2);
    tendency_pair_kernel<TX, T, PF><<<grid, TX, 0, s>>>(a, nyA, nyB);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// the strip tile of qg_set_form(QG_FORM_TENDENCY_TILE, (W << 16) | R): strips W points wide
// (one thread per point, W in {64, 128, 256, 512}) and about R rows per workgroup -- BASELINE
// config 3's LDS tile sweep.  w = 0: the default geometry.
static void tend_tile(int &w, int &r) {
    const int v = form(QG_FORM_TENDENCY_TILE);
    w = v >> 16;
    r = v & 0xffff;
    if ((w != 64 && w != 128 && w != 256 && w != 512) || r < 1) w = 0;
}

template <class T>
static int launch_tend_direct(const TendArgsT<T> &a, hipStream_t s) {
    const int nA = (a.j1 - a.j0 + 3) / 4, nB = a.j3 > a.j2 ? (a.j3 - a.j2 + 3) / 4 : 0;
    dim3 grid((unsigned)((a.M + 63) / 64), (unsigned)(nA + nB), 2);
    tendency_direct_kernel<T><<<grid, 256, 0, s>>>(a, nA, nB);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

template <class T>
static int launch_tendency_t(const TendArgsT<T> &a, hipStream_t s) {
    if (a.j1 - a.j0 <= 0 && a.j3 - a.j2 <= 0) return QG_OK;
    int tw, tr;
    tend_tile(tw, tr);
    switch (tw) {
        case 64: return launch_tend_variant<64, 1, T>(a, tr, s);
        case 128: return launch_tend_variant<128, 1, T>(a, tr, s);
        case 256: return launch_tend_variant<256, 1, T>(a, tr, s);
        case 512: return launch_tend_variant<512, 1, T>(a, tr, s);
        default: break;
    }
    const int f = form(QG_FORM_TENDENCY);
    if constexpr (sizeof(T) == 4) {
        if (f == QG_TEND_AUTO && a.M % 2 == 0) return launch_tend_pair<256>(a, s);
    }  // (F64 pair kernel measured slower: 0.41-0.43 vs 0.386 ms at 4096^2 -- HBM-bound already)
    const double pts = (double)a.M * ((a.j1 - a.j0) + (a.j3 > a.j2 ? a.j3 - a.j2 : 0));
    if (f == QG_TEND_DIRECT || (f != QG_TEND_RING && pts < TEND_DIRECT_PTS)) return launch_tend_direct(a, s);
    // ~870^2 .. ~1750^2 points: 128-wide strips of 8 rows (tile sweep: 1024^2 35 vs 38 us)
    if (pts >= 0.75e6 && pts < 3.0e6) return launch_tend_variant<128, 1, T>(a, 8, s);
    return launch_tend_balanced(a, s);
}

int launch_tendency(const TendArgsT<double> &a, hipStream_t s) { return launch_tendency_t(a, s); }
int launch_tendency(const TendArgsT<float> &a, hipStream_t s) { return launch_tendency_t(a, s); }

// seeded initialise_model; P = local rows, P_total / j_offset place the slab in the global grid
int launch_initialise_global(void *zeta, void *psi, void *f_store, int esize, int64_t M, int64_t P,
                             int64_t P_total, int64_t j_offset, double amp, double S1, double S2,
                             double dx, uint64_t seed1, uint64_t seed2, hipStream_t s) {
    const size_t F = (size_t)(M + 2) * (size_t)(P + 2);
    QG_HIP(hipMemsetAsync(zeta, 0, esize * F * 6, s));
    QG_HIP(hipMemsetAsync(psi, 0, esize * F * 6, s));
    QG_HIP(hipMemsetAsync(f_store, 0, esize * F * 6, s));
    const double i = 1.0 / dx;
    dim3 grid((unsigned)((M + 2 + 255) / 256), (unsigned)(P + 2));
    if (esize == 8)
        initialise_kernel<double><<<grid, 256, 0, s>>>((double *)zeta, (double *)psi, M, P, P_total, j_offset, amp,
                                                       S1, S2, i * i, seed1, seed2);
    else
        initialise_kernel<float><<<grid, 256, 0, s>>>((float *)zeta, (float *)psi, M, P, P_total, j_offset, amp,
                                                      S1, S2, i * i, seed1, seed2);
    QG_LAUNCH_CHECK();
    return QG_OK;
}
}  // namespace qg
