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
template <class ZF, class SF>
__device__ __forceinline__ double arakawa_point(ZF Z, SF S, double den) {
    const double jpp = (Z(1, 0) - Z(-1, 0)) * (S(0, 1) - S(0, -1)) - (Z(0, 1) - Z(0, -1)) * (S(1, 0) - S(-1, 0));
    const double jpt = ((Z(1, 0) * (S(1, 1) - S(1, -1)) - Z(-1, 0) * (S(-1, 1) - S(-1, -1))) -
                        Z(0, 1) * (S(1, 1) - S(-1, 1))) +
                       Z(0, -1) * (S(1, -1) - S(-1, -1));
    const double jtp = ((Z(1, 1) * (S(0, 1) - S(1, 0)) - Z(-1, -1) * (S(-1, 0) - S(0, -1))) -
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
    store_with_ghosts(out, ld, M, P, i, j, arakawa_point(Z, S, den), true);
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

// ------------------------------------------------------------------------------------
// Fused tendency + Euler/AB3 update (evolve_zeta!, model.jl:155-170), one layer per
// blockIdx.z.  Each block owns TX columns and marches down a strip of rows keeping rolling
// LDS rings: psi (5 rows, x-halo 2), zeta (4 rows, x-halo 1), lap(psi) (3 rows, x-halo 1).
// Every psi / zeta row is read from HBM once per strip (plus the strip's 4 / 2 halo rows).
// Per interior point the kernel reads zeta, psi, [F(t-1), F(t-2)] and writes zeta+, F.
// ------------------------------------------------------------------------------------
template <int TX>
__global__ __launch_bounds__(TX) void tendency_kernel(TendArgs a, int rows_per_block) {
    const int layer = blockIdx.z;
    const int t = threadIdx.x;
    const int64_t M = a.M, P = a.P, ld = a.ld;
    const int64_t x0 = (int64_t)blockIdx.x * TX;
    const int64_t i = x0 + t;
    const int jb0 = a.j0 + blockIdx.y * rows_per_block;
    const int jb1 = min(jb0 + rows_per_block, a.j1);
    if (jb0 >= jb1) return;  // uniform over the block

    __shared__ double sp[5][TX + 4];
    __shared__ double sz[4][TX + 2];
    __shared__ double sl[3][TX + 2];

    const double *psi = a.psi[layer];
    const double *zeta = a.zeta[layer];
    const RowSrc &prs = a.psi_rows[layer];
    const RowSrc &zrs = a.zeta_rows[layer];
    const double idx = 1.0 / a.dx, idx2 = idx * idx;
    const double cdc = 0.5 * idx;
    const double den = 12 * (a.dx * a.dx);
    const int Mi = (int)M;

    auto rowp = [&](const double *base, const RowSrc &rs, int j) -> const double * {
        if (j >= 0 && j < P) return base + fidx(1, j + 1, ld);
        return rs.halo[j < 0 ? j + 2 : (int)(j - P) + 2];
    };
    auto xw = [&](int64_t x) -> int64_t {
        int xi = (int)(x % Mi);
        return xi < 0 ? xi + Mi : xi;
    };
    auto load_psi = [&](int j) {
        const double *r = rowp(psi, prs, j);
        double *dst = sp[(j + 10) % 5];
        for (int q = t; q < TX + 4; q += TX) dst[q] = r[xw(x0 - 2 + q)];
    };
    auto load_zeta = [&](int j) {
        const double *r = rowp(zeta, zrs, j);
        double *dst = sz[(j + 8) % 4];
        for (int q = t; q < TX + 2; q += TX) dst[q] = r[xw(x0 - 1 + q)];
    };
    auto lap_row = [&](int j) {  // lap(psi) at row j, positions x0-1 .. x0+TX
        const double *pm = sp[(j - 1 + 10) % 5], *p0 = sp[(j + 10) % 5], *pp = sp[(j + 1 + 10) % 5];
        double *dst = sl[(j + 3) % 3];
        for (int q = t; q < TX + 2; q += TX) {
            const int c = q + 1;
            dst[q] = ((((p0[c - 1] + p0[c + 1]) - 4 * p0[c]) + pm[c]) + pp[c]) * idx2;
        }
    };

    // prologue: psi rows jb0-2..jb0+1, zeta rows jb0-1..jb0, lap rows jb0-1, jb0
    for (int j = jb0 - 2; j <= jb0 + 1; ++j) load_psi(j);
    load_zeta(jb0 - 1);
    load_zeta(jb0);
    __syncthreads();
    lap_row(jb0 - 1);
    lap_row(jb0);

    const double bl = a.beta[layer];
    for (int j = jb0; j < jb1; ++j) {
        load_psi(j + 2);
        load_zeta(j + 1);
        __syncthreads();
        lap_row(j + 1);
        __syncthreads();
        if (i < M) {
            const double *Lm = sl[(j - 1 + 3) % 3], *L0 = sl[(j + 3) % 3], *Lp = sl[(j + 1 + 3) % 3];
            const double *Pm = sp[(j - 1 + 10) % 5], *P0 = sp[(j + 10) % 5], *Pp = sp[(j + 1 + 10) % 5];
            const double *Zm = sz[(j - 1 + 8) % 4], *Z0 = sz[(j + 8) % 4], *Zp = sz[(j + 1 + 8) % 4];
            const int cl = t + 1;  // centre in sl / sz (x-halo 1)
            const int cp = t + 2;  // centre in sp (x-halo 2)
            const double biharm = ((((L0[cl - 1] + L0[cl + 1]) - 4 * L0[cl]) + Lm[cl]) + Lp[cl]) * idx2;
            const double v_term = a.visc * biharm;
            auto Z = [&](int da, int db) {
                const double *r = db < 0 ? Zm : (db > 0 ? Zp : Z0);
                return r[cl + da];
            };
            auto S = [&](int da, int db) {
                const double *r = db < 0 ? Pm : (db > 0 ? Pp : P0);
                return r[cp + da];
            };
            const double J_term = arakawa_point(Z, S, den);
            const double beta_term = bl * (cdc * (P0[cp + 1] - P0[cp - 1]));
            double last;
            if (layer == 0) last = a.U * (cdc * (Z0[cl + 1] - Z0[cl - 1]));  // U * cd(zeta)
            else last = a.r * L0[cl];                                         // r * lap(psi)
            const double F = ((v_term - J_term) - beta_term) - last;
            const double zc = Z0[cl];
            double zn;
            const size_t o = fidx(i + 1, j + 1, ld);
            if (!a.ab3) {
                zn = zc + (a.dt * F);
            } else {
                const double f2 = a.fprev1[layer][o], f3 = a.fprev2[layer][o];
                zn = zc + a.dt * ((((23.0 / 12.0) * F) - ((16.0 / 12.0) * f2)) + ((5.0 / 12.0) * f3));
            }
            store_with_ghosts(a.zeta_out[layer], ld, M, P, i, j, zn, a.write_ghost_rows);
            store_with_ghosts(a.f_out[layer], ld, M, P, i, j, F, a.write_ghost_rows);
        }
    }
}

// ------------------------------------------------------------------------------------
// Seeded initialise_model: psi and zeta of slot 0, ghosts included, computed directly at
// the wrapped GLOBAL index (so slabs need no communication).  model.jl:37-62.
// ------------------------------------------------------------------------------------
__global__ void initialise_kernel(double *zeta, double *psi, int64_t M, int64_t P, int64_t P_total,
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
    psi[o] = p1;
    psi[F + o] = p2;
    zeta[o] = lap(seed1) + S1 * (p2 - p1);
    zeta[F + o] = lap(seed2) + S2 * (p1 - p2);
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

int launch_tendency(const TendArgs &a, hipStream_t s) {
    constexpr int TX = 128;
    const int rows = 32;
    const int nrows = a.j1 - a.j0;
    if (nrows <= 0) return QG_OK;
    dim3 grid((unsigned)((a.M + TX - 1) / TX), (unsigned)((nrows + rows - 1) / rows), 2);
    tendency_kernel<TX><<<grid, TX, 0, s>>>(a, rows);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// seeded initialise_model; P = local rows, P_total / j_offset place the slab in the global grid
int launch_initialise_global(double *zeta, double *psi, double *f_store, int64_t M, int64_t P,
                             int64_t P_total, int64_t j_offset, double amp, double S1, double S2,
                             double dx, uint64_t seed1, uint64_t seed2, hipStream_t s) {
    const size_t F = (size_t)(M + 2) * (size_t)(P + 2);
    QG_HIP(hipMemsetAsync(zeta, 0, sizeof(double) * F * 6, s));
    QG_HIP(hipMemsetAsync(psi, 0, sizeof(double) * F * 6, s));
    QG_HIP(hipMemsetAsync(f_store, 0, sizeof(double) * F * 6, s));
    const double i = 1.0 / dx;
    dim3 grid((unsigned)((M + 2 + 255) / 256), (unsigned)(P + 2));
    initialise_kernel<<<grid, 256, 0, s>>>(zeta, psi, M, P, P_total, j_offset, amp, S1, S2, i * i, seed1,
                                           seed2);
    QG_LAUNCH_CHECK();
    return QG_OK;
}
}  // namespace qg
