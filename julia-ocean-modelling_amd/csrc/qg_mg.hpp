// Geometric multigrid V-cycle: the QG_PRECOND_MULTIGRID preconditioner of the matrix-free PCG
// (qg_pcg.hip) -- SURVEY 7 step 5.  See qg_mg.hip.
#pragma once

#include "qg_common.hpp"

namespace qg {

constexpr int MG_MAX_LEVELS = 40;
constexpr int MG_COARSE_MAX = 4096;  // interior points of the coarsest grid (one workgroup's LDS)

struct MgLevel {
    int64_t M = 0, P = 0, ld = 0;
    double cx = 0, cy = 0;  // 1 / hx^2, 1 / hy^2
    int rx = 0, ry = 0;     // coarsened from the previous level in x / y
    int slab = 0;           // 1: a rank's slab (y neighbours from the ghost rows, refreshed by
                            // the transport); 0: the whole y-periodic domain (y wraps)
    int agg = 0;            // the global grid gathered from the previous (slab) level
    double *z[2] = {}, *t[2] = {}, *r[2] = {};  // level 0: z, r are the caller's
};

class MgPrecond {
public:
    typedef int (*GatherFn)(void *user, const double *send, double *recv, int64_t count, hipStream_t s);
    typedef int (*HaloFn)(void *comm, double *const *fields, int nfields, int64_t M, int64_t P, int depth,
                          double *halo_buf, hipStream_t s);
    // M x P points on each of nranks ranks (y-slabs, P_total = nranks P).  alpha[s]:
    // B_s = -(5-point Laplacian + alpha_s), alpha_s <= 0.
    int init(int64_t M, int64_t P, int rank, int nranks, double dx, const double alpha[2]);
    ~MgPrecond();
    // z_s = V(r_s), s = 0, 1: (M+2, P+2) fields; r's interior is read, z's interior written;
    // the ghost rows of both are scratch (a slab refreshes them from its neighbours).
    // nranks > 1: every rank calls it (ghost-row refreshes and the agglomerated level's two
    // all-gathers are collective).
    int apply(const double *r0, const double *r1, double *z0, double *z1, hipStream_t s, GatherFn gather = nullptr,
              void *user = nullptr, HaloFn halo = nullptr, void *halo_user = nullptr);
    static bool supports(int64_t M, int64_t P, int nranks);

private:
    int vcycle(int l, hipStream_t s);
    int refresh(const MgLevel &L, double *const *f, hipStream_t s);
    MgLevel lv_[MG_MAX_LEVELS];
    int nl_ = 0, ksw_ = 0, rank_ = 0;
    double alpha_[2] = {0, 0};
    void *mem_ = nullptr;
    GatherFn gather_ = nullptr;
    HaloFn halo_ = nullptr;
    void *user_ = nullptr, *halo_user_ = nullptr;
};

}  // namespace qg
