// Geometric multigrid V-cycle as the PCG preconditioner (QG_PRECOND_MULTIGRID; SURVEY 7
// step 5: "geometric multigrid V-cycle on the periodic grid -- all bandwidth-bound stencils").
//
// Operator per level and system: B_s = -(cx (E + W - 2) + cy (N + S - 2) + alpha_s), the
// 5-point form of construct_spA (src/schemes/laplacian.jl:54-75) with hx, hy of the level,
// periodic in x and y.  The Poisson system's pin (laplacian.jl:70-73) is handled around the
// cycle by PCG (qg_pcg.hip, mg_precond): z = T^T V T r, T moving the compatibility residue
// sum(r) to the pin, T^T shifting z to vanish there -- the pinned inverse's exact form.
//
// V(2,2): two damped-Jacobi sweeps from zero (one fused pass), the residual restricted by
// full weighting (R = c P^T in every direction that coarsens, so the cycle is symmetric), the
// coarse problem rediscretised at 2h, bilinear prolongation, two sweeps; the coarsest grid
// (<= MG_COARSE_MAX points) gets Jacobi sweeps inside one workgroup's LDS.  A dimension
// coarsens while it is even and >= 8 (semi-coarsening when only one does), down to <= 64
// points.
//
// Across y-slabs the cycle is the same global one: a slab level takes its y neighbours from
// ghost rows the transport refreshes before every stencil pass that reads them (comm_halo),
// and once a slab level is down to MG_AGG_POINTS points (or cannot halve its rows) its
// right-hand side is all-gathered into the global grid (one contiguous block of rows per
// rank), which every rank then cycles redundantly and identically; each rank takes its own
// rows of the result back.
//
// Every stage is a stencil pass over rows: HBM-bound, one thread per point of a row segment,
// rows strided over the grid's y workgroups.  Sums run in a fixed order: deterministic.
#include <algorithm>
#include <cstring>

#include "qg_mg.hpp"

namespace qg {

constexpr int MG_T = 256;
constexpr int MG_ROWB = 256;
constexpr double MG_OMEGA = 0.8;  // damped Jacobi: optimal smoothing factor of the 2-D 5-point stencil

struct MgOp {
    int64_t M, P, ld;
    double cx, cy, alpha[2], wd[2];  // wd = omega / diag(B_s)
    int slab;                         // y neighbours beyond the rows: ghost rows (1) or wrap (0)
};

// f(i, j), i wrapping; j in [-1, P] on a slab level (rows -1 and P: the refreshed ghost rows)
__device__ __forceinline__ double mg_at(const MgOp &o, const double *f, int64_t i, int64_t j) {
    if (i < 0) i += o.M;
    else if (i >= o.M) i -= o.M;
    if (!o.slab) {
        if (j < 0) j += o.P;
        else if (j >= o.P) j -= o.P;
    }
    return f[fidx(i + 1, j + 1, o.ld)];
}

__device__ __forceinline__ double mg_apply(const MgOp &o, int s, const double *f, int64_t i, int64_t j) {
    const double c = mg_at(o, f, i, j);
    const double lap = o.cx * ((mg_at(o, f, i - 1, j) + mg_at(o, f, i + 1, j)) - 2 * c) +
                       o.cy * ((mg_at(o, f, i, j - 1) + mg_at(o, f, i, j + 1)) - 2 * c);
    return -(lap + o.alpha[s] * c);
}

// zout = zin + omega D^-1 (r - B zin)
struct MgJac {
    MgOp o;
    const double *r[2], *zin[2];
    double *zout[2];
};
__global__ __launch_bounds__(MG_T) void mg_jacobi(MgJac a) {
    const int s = blockIdx.z;
    const int64_t i = blockIdx.x * (int64_t)MG_T + threadIdx.x;
    if (i >= a.o.M) return;
    const double wd = a.o.wd[s];
    const double *r = a.r[s], *zin = a.zin[s];
    double *zout = a.zout[s];
    for (int64_t j = blockIdx.y; j < a.o.P; j += gridDim.y) {
        const size_t o = fidx(i + 1, j + 1, a.o.ld);
        zout[o] = zin[o] + wd * (r[o] - mg_apply(a.o, s, zin, i, j));
    }
}

// the two pre-smoothing sweeps from zero in one pass: t = omega D^-1 r, z = t + omega D^-1 (r - B t)
// = omega D^-1 (2 r - omega D^-1 B r) (D is constant on a level); r's neighbours on a slab level
// from its refreshed ghost rows
struct MgPre {
    MgOp o;
    const double *r[2];
    double *z[2];
};
__global__ __launch_bounds__(MG_T) void mg_pre(MgPre a) {
    const int s = blockIdx.z;
    const int64_t i = blockIdx.x * (int64_t)MG_T + threadIdx.x;
    if (i >= a.o.M) return;
    const double wd = a.o.wd[s];
    const double *r = a.r[s];
    for (int64_t j = blockIdx.y; j < a.o.P; j += gridDim.y) {
        const size_t o = fidx(i + 1, j + 1, a.o.ld);
        a.z[s][o] = wd * (2 * r[o] - wd * mg_apply(a.o, s, r, i, j));
    }
}

// t = r - B z
struct MgResid {
    MgOp o;
    const double *r[2], *z[2];
    double *t[2];
};
__global__ __launch_bounds__(MG_T) void mg_resid(MgResid a) {
    const int s = blockIdx.z;
    const int64_t i = blockIdx.x * (int64_t)MG_T + threadIdx.x;
    if (i >= a.o.M) return;
    for (int64_t j = blockIdx.y; j < a.o.P; j += gridDim.y) {
        const size_t o = fidx(i + 1, j + 1, a.o.ld);
        a.t[s][o] = a.r[s][o] - mg_apply(a.o, s, a.z[s], i, j);
    }
}

// coarse rhs = full weighting of the fine residual t (1/4, 1/2, 1/4 per coarsened direction)
struct MgRestrict {
    MgOp f;
    const double *t[2];
    int64_t Mc, Pc, ldc;
    int rx, ry;
    double *rc[2];
};
__global__ __launch_bounds__(MG_T) void mg_restrict(MgRestrict a) {
    const int s = blockIdx.z;
    const int64_t I = blockIdx.x * (int64_t)MG_T + threadIdx.x;
    if (I >= a.Mc) return;
    for (int64_t J = blockIdx.y; J < a.Pc; J += gridDim.y) {
        double acc = 0;
        for (int dj = -1; dj <= 1; ++dj) {
            if (!a.ry && dj) continue;
            const double wy = a.ry ? (dj ? 0.25 : 0.5) : 1.0;
            const int64_t j = a.ry ? 2 * J + dj : J;
            double row = 0;
            for (int di = -1; di <= 1; ++di) {
                if (!a.rx && di) continue;
                const double wx = a.rx ? (di ? 0.25 : 0.5) : 1.0;
                const int64_t i = a.rx ? 2 * I + di : I;
                row += wx * mg_at(a.f, a.t[s], i, j);
            }
            acc += wy * row;
        }
        a.rc[s][fidx(I + 1, J + 1, a.ldc)] = acc;
    }
}

// z += bilinear interpolation of the coarse correction.  (Fused into the first post-smoothing
// sweep instead -- the interpolation formed at all five stencil points -- it ran 0.67 ms per
// 4096^2 cycle against 0.25 + 0.24 for the two passes.)
struct MgProlong {
    MgOp c;
    const double *zc[2];
    int64_t M, P, ld;
    int rx, ry;
    double *z[2];
};
__global__ __launch_bounds__(MG_T) void mg_prolong(MgProlong a) {
    const int s = blockIdx.z;
    const int64_t i = blockIdx.x * (int64_t)MG_T + threadIdx.x;
    if (i >= a.M) return;
    const double *zc = a.zc[s];
    const int64_t I = a.rx ? i >> 1 : i;
    const bool hx = a.rx && (i & 1);
    for (int64_t j = blockIdx.y; j < a.P; j += gridDim.y) {
        const int64_t J = a.ry ? j >> 1 : j;
        const bool hy = a.ry && (j & 1);
        double e = mg_at(a.c, zc, I, J);
        if (hx && hy)
            e = 0.25 * ((e + mg_at(a.c, zc, I + 1, J)) + (mg_at(a.c, zc, I, J + 1) + mg_at(a.c, zc, I + 1, J + 1)));
        else if (hx)
            e = 0.5 * (e + mg_at(a.c, zc, I + 1, J));
        else if (hy)
            e = 0.5 * (e + mg_at(a.c, zc, I, J + 1));
        a.z[s][fidx(i + 1, j + 1, a.ld)] += e;
    }
}

// coarsest (global) grid: `sweeps` damped-Jacobi sweeps from zero in LDS, one workgroup per
// system
struct MgCoarse {
    MgOp o;
    const double *r[2];
    double *z[2];
    int sweeps;
};
__global__ __launch_bounds__(MG_T) void mg_coarse(MgCoarse a) {
    extern __shared__ double sh[];
    const int s = blockIdx.x;
    const int M = (int)a.o.M, P = (int)a.o.P, n = M * P;
    double *za = sh, *zb = sh + n, *rr = sh + 2 * n;
    const double wd = a.o.wd[s];
    for (int k = threadIdx.x; k < n; k += MG_T) {
        const double v = a.r[s][fidx(k % M + 1, k / M + 1, a.o.ld)];
        rr[k] = v;
        za[k] = wd * v;
    }
    __syncthreads();
    auto at = [&](const double *f, int i, int j) -> double {
        if (i < 0) i += M;
        else if (i >= M) i -= M;
        if (j < 0) j += P;  // (the coarsest level is a global one: y wraps)
        else if (j >= P) j -= P;
        return f[i + M * j];
    };
    double *src = za, *dst = zb;
    for (int it = 1; it < a.sweeps; ++it) {
        for (int k = threadIdx.x; k < n; k += MG_T) {
            const int i = k % M, j = k / M;
            const double c = src[k];
            const double lap = a.o.cx * ((at(src, i - 1, j) + at(src, i + 1, j)) - 2 * c) +
                               a.o.cy * ((at(src, i, j - 1) + at(src, i, j + 1)) - 2 * c);
            dst[k] = c + wd * (rr[k] + (lap + a.o.alpha[s] * c));
        }
        __syncthreads();
        double *t = src;
        src = dst;
        dst = t;
    }
    for (int k = threadIdx.x; k < n; k += MG_T) a.z[s][fidx(k % M + 1, k / M + 1, a.o.ld)] = src[k];
}

// ------------------------------------------------------------------------------------
// Levels: slab levels (nranks > 1) halve while their rows can (even, >= 8) and the level has
// more than MG_AGG_POINTS points; then the global grid of the same resolution is gathered, and
// global levels halve down to <= 64 points.  (Below ~4096 points per rank a level's work is a
// few microseconds and its five ghost-row exchanges are the whole cost: those levels are
// cycled redundantly on every rank instead.)
constexpr int64_t MG_AGG_POINTS = 4096;
static int plan_levels(int64_t M, int64_t P, int nranks, MgLevel *lv) {
    lv[0] = MgLevel{};
    lv[0].M = M;
    lv[0].P = P;
    lv[0].slab = nranks > 1;
    int n = 1;
    while (n < MG_MAX_LEVELS) {
        const MgLevel &f = lv[n - 1];
        const int rx = f.M % 2 == 0 && f.M >= 8, ry = f.P % 2 == 0 && f.P >= 8;
        MgLevel c{};
        if (f.slab) {
            if (f.M * f.P > MG_AGG_POINTS && ry) {
                c.M = rx ? f.M / 2 : f.M;
                c.P = f.P / 2;
                c.rx = rx;
                c.ry = 1;
                c.slab = 1;
            } else {
                c.M = f.M;
                c.P = f.P * nranks;
                c.agg = 1;
            }
        } else {
            if (f.M * f.P <= 64 || (!rx && !ry)) break;
            c.M = rx ? f.M / 2 : f.M;
            c.P = ry ? f.P / 2 : f.P;
            c.rx = rx;
            c.ry = ry;
        }
        lv[n++] = c;
    }
    return n;
}

bool MgPrecond::supports(int64_t M, int64_t P, int nranks) {
    if (M < 3 || P < 1 || nranks < 1) return false;
    MgLevel lv[MG_MAX_LEVELS];
    const int n = plan_levels(M, P, nranks, lv);
    return !lv[n - 1].slab && lv[n - 1].M * lv[n - 1].P <= MG_COARSE_MAX;
}

int MgPrecond::init(int64_t M, int64_t P, int rank, int nranks, double dx, const double alpha[2]) {
    if (!(dx > 0) || !(alpha[0] <= 0) || !(alpha[1] <= 0) || rank < 0 || rank >= nranks) return QG_ERR_INVALID_ARG;
    if (!supports(M, P, nranks)) return QG_ERR_UNSUPPORTED;
    nl_ = plan_levels(M, P, nranks, lv_);
    rank_ = rank;
    alpha_[0] = alpha[0];
    alpha_[1] = alpha[1];
    double hx = dx, hy = dx;
    size_t total = 0;
    for (int l = 0; l < nl_; ++l) {
        MgLevel &L = lv_[l];
        if (L.rx) hx *= 2;
        if (L.ry) hy *= 2;
        L.ld = L.M + 2;
        L.cx = 1.0 / (hx * hx);
        L.cy = 1.0 / (hy * hy);
        const size_t F = (size_t)(L.M + 2) * (size_t)(L.P + 2);
        total += (l == 0 ? 2 : 6) * F;
    }
    const MgLevel &C = lv_[nl_ - 1];
    ksw_ = (int)std::min<int64_t>(512, 8 * std::max(C.M, C.P));
    QG_HIP(hipFuncSetAttribute((const void *)mg_coarse, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(double) * 3 * MG_COARSE_MAX)));
    if (hipMalloc(&mem_, sizeof(double) * total) != hipSuccess) {
        mem_ = nullptr;
        return QG_ERR_ALLOC;
    }
    QG_HIP(hipMemset(mem_, 0, sizeof(double) * total));
    double *m = static_cast<double *>(mem_);
    for (int l = 0; l < nl_; ++l) {
        MgLevel &L = lv_[l];
        const size_t F = (size_t)(L.M + 2) * (size_t)(L.P + 2);
        for (int s = 0; s < 2; ++s) {
            L.t[s] = m;
            m += F;
            if (l > 0) {
                L.z[s] = m;
                m += F;
                L.r[s] = m;
                m += F;
            }
        }
    }
    return QG_OK;
}

MgPrecond::~MgPrecond() {
    if (mem_) (void)hipFree(mem_);
}

static MgOp level_op(const MgLevel &L, const double alpha[2]) {
    MgOp o{};
    o.M = L.M;
    o.P = L.P;
    o.ld = L.ld;
    o.cx = L.cx;
    o.cy = L.cy;
    o.slab = L.slab;
    for (int s = 0; s < 2; ++s) {
        o.alpha[s] = alpha[s];
        o.wd[s] = MG_OMEGA / (2 * L.cx + 2 * L.cy - alpha[s]);
    }
    return o;
}

static dim3 level_grid(int64_t M, int64_t P) {
    return dim3((unsigned)((M + MG_T - 1) / MG_T), (unsigned)std::min<int64_t>(P, MG_ROWB), 2);
}

// the ghost rows of a slab level's field pair, from the neighbouring slabs
int MgPrecond::refresh(const MgLevel &L, double *const *f, hipStream_t s) {
    if (!L.slab) return QG_OK;
    if (!halo_) return QG_ERR_INVALID_ARG;
    return halo_(halo_user_, f, 2, L.M, L.P, -1, nullptr, s);
}

int MgPrecond::vcycle(int l, hipStream_t st) {
    const MgLevel &L = lv_[l];
    const MgOp op = level_op(L, alpha_);
    if (l == nl_ - 1) {  // coarsest
        MgCoarse a{};
        a.o = op;
        a.sweeps = ksw_;
        for (int s = 0; s < 2; ++s) {
            a.r[s] = L.r[s];
            a.z[s] = L.z[s];
        }
        mg_coarse<<<2, MG_T, sizeof(double) * 3 * (size_t)(L.M * L.P), st>>>(a);
        QG_LAUNCH_CHECK();
        return QG_OK;
    }
    const MgLevel &C = lv_[l + 1];
    if (C.agg) {  // the global grid: every rank's rows of r, the cycle, this rank's rows of z
        if (!gather_) return QG_ERR_INVALID_ARG;
        for (int s = 0; s < 2; ++s) QG_CHECK(gather_(user_, L.r[s] + L.ld, C.r[s] + C.ld, L.P * L.ld, st));
        QG_CHECK(vcycle(l + 1, st));
        for (int s = 0; s < 2; ++s)
            QG_HIP(hipMemcpyAsync(L.z[s] + L.ld, C.z[s] + C.ld * (1 + (int64_t)rank_ * L.P),
                                  sizeof(double) * (size_t)(L.P * L.ld), hipMemcpyDeviceToDevice, st));
        return QG_OK;
    }
    const dim3 grid = level_grid(L.M, L.P);
    double *const *rr = L.r;
    // down: the two pre-smoothing sweeps, residual, restriction
    QG_CHECK(refresh(L, rr, st));
    {
        MgPre a{};
        a.o = op;
        for (int s = 0; s < 2; ++s) {
            a.r[s] = L.r[s];
            a.z[s] = L.z[s];
        }
        mg_pre<<<grid, MG_T, 0, st>>>(a);
        QG_LAUNCH_CHECK();
    }
    QG_CHECK(refresh(L, L.z, st));
    {
        MgResid a{};
        a.o = op;
        for (int s = 0; s < 2; ++s) {
            a.r[s] = L.r[s];
            a.z[s] = L.z[s];
            a.t[s] = L.t[s];
        }
        mg_resid<<<grid, MG_T, 0, st>>>(a);
        QG_LAUNCH_CHECK();
    }
    QG_CHECK(refresh(L, L.t, st));
    {
        MgRestrict a{};
        a.f = op;
        a.Mc = C.M;
        a.Pc = C.P;
        a.ldc = C.ld;
        a.rx = C.rx;
        a.ry = C.ry;
        for (int s = 0; s < 2; ++s) {
            a.t[s] = L.t[s];
            a.rc[s] = C.r[s];
        }
        mg_restrict<<<level_grid(C.M, C.P), MG_T, 0, st>>>(a);
        QG_LAUNCH_CHECK();
    }
    QG_CHECK(vcycle(l + 1, st));
    // up: correct, post-smooth
    QG_CHECK(refresh(C, C.z, st));
    {
        MgProlong a{};
        a.c = level_op(C, alpha_);
        a.M = L.M;
        a.P = L.P;
        a.ld = L.ld;
        a.rx = C.rx;
        a.ry = C.ry;
        for (int s = 0; s < 2; ++s) {
            a.zc[s] = C.z[s];
            a.z[s] = L.z[s];
        }
        mg_prolong<<<grid, MG_T, 0, st>>>(a);
        QG_LAUNCH_CHECK();
    }
    auto jacobi = [&](double *const *zin, double *const *zout) -> int {
        MgJac a{};
        a.o = op;
        for (int s = 0; s < 2; ++s) {
            a.r[s] = L.r[s];
            a.zin[s] = zin[s];
            a.zout[s] = zout[s];
        }
        mg_jacobi<<<grid, MG_T, 0, st>>>(a);
        QG_LAUNCH_CHECK();
        return QG_OK;
    };
    QG_CHECK(refresh(L, L.z, st));
    QG_CHECK(jacobi(L.z, L.t));
    QG_CHECK(refresh(L, L.t, st));
    return jacobi(L.t, L.z);
}

int MgPrecond::apply(const double *r0, const double *r1, double *z0, double *z1, hipStream_t s, GatherFn gather,
                     void *user, HaloFn halo, void *halo_user) {
    if (!mem_) return QG_ERR_NOT_BOUND;
    MgLevel &F = lv_[0];
    F.r[0] = const_cast<double *>(r0);
    F.r[1] = const_cast<double *>(r1);
    F.z[0] = z0;
    F.z[1] = z1;
    gather_ = gather;
    user_ = user;
    halo_ = halo;
    halo_user_ = halo_user;
    return vcycle(0, s);
}

}  // namespace qg
