// Matrix-free PCG solver for the evolve_psi! pair of systems (see qg_pcg.hip).
#pragma once

#include "qg_common.hpp"
#include "qg_mg.hpp"
#include "qg_spectral.hpp"

namespace qg {

// device scalar slots (per system s: +s)
enum {
    PCG_BB = 0, PCG_RZ = 2, PCG_ALPHA = 4, PCG_BETA = 6, PCG_RR = 8, PCG_RSUM = 10, PCG_RSUM6 = 12,
    PCG_SUMR = 18, PCG_ZPIN = 19,  // multigrid: sum of the Poisson residual, the pinned value of z
    PCG_NSCAL = 20
};

struct PcgArgs {
    int64_t M, P, ld, P_total, j_offset;
    int rank, nranks;
    double idx2;
    double alpha[2];
    int pinned0;
    double proj_in[4], proj_out[4];
    double pinv_out[4];  // proj_out^-1 (certified preconditioner step)
    int ghost_rows;
    const double *in1, *in2;
    double *out1, *out2;
    double *x[2], *r[2], *p[2], *q[2], *z[2];  // (M+2, P+2) fields
    double *partial;                            // [blocks][2] (fast path: [blocks][6])
    double *scal;                               // PCG_NSCAL doubles
};

class PcgSolver {
public:
    typedef int (*HaloFn)(void *comm, double *const *fields, int nfields, int64_t M, int64_t P, int depth,
                          double *halo_buf, hipStream_t s);
    int init(int64_t M, int64_t P, int64_t P_total, int rank, int nranks, double dx, const double alpha[2],
             int pinned0, const double proj_in[4], const double proj_out[4], int precond, double rtol, int maxit,
             int chunk_rows);
    ~PcgSolver();
    // Synchronises the stream once per iteration (convergence test on the host).
    int solve(const double *in1, const double *in2, double *out1, double *out2, int ghost_rows, hipStream_t s,
              SpectralSolver::GatherFn gather = nullptr, void *user = nullptr, HaloFn halo = nullptr,
              void *halo_user = nullptr);
    int iterations() const { return iters_; }
    double relres(int s) const { return relres_[s]; }

    // ---- deferred certification (default; qg_set_pcg_sync(ctx, 1) restores the host-checked
    // iteration -- the library reads no environment switch for it).  The certified step's residual check runs on the device and
    // its verdict is latched there (no host round trip, graph-capturable): fused into the
    // next tendency when `fuse` (one rank), else as its own pass right after the solve.
    void set_deferred(bool on) { deferred_ = on; }
    bool deferred() const { return deferred_ && cert_ && precond_ == QG_PRECOND_SPECTRAL; }
    void set_fuse(bool on) { fuse_ = on; }
    bool pending() const { return pending_; }
    // the certification fields of the next tendency's arguments
    void fill_cert_args(TendArgsT<double> &t) const;
    // after launch_tendency_cert: fold its nblk partials and latch the verdict
    int latch_fused(int nblk, hipStream_t s);
    // workgroups a certifying tendency may write partials for (launch_tendency_cert's cap)
    int64_t cert_capacity() const { return cert_part_n_; }
    // a pending fused certification with no tendency coming: run the check pass now
    int certify_pending(hipStream_t s, SpectralSolver::GatherFn gather = nullptr, void *user = nullptr);
    // latch record (device, doubles): [0] solves certified, [1] failures, [2] first failing
    // solve (1-based, 0 = none), [3] worst relres, [4] [5] last relres (Poisson, Helmholtz)
    const double *latch() const { return latch_; }
    int reset_latch(hipStream_t s);

private:
    int reduce(int what, hipStream_t s, SpectralSolver::GatherFn gather, void *user);
    int mg_precond(hipStream_t s, SpectralSolver::GatherFn gather, void *user, HaloFn halo, void *halo_user);
    PcgArgs a_{};
    SpectralSolver pre_;
    MgPrecond mg_;
    int precond_ = 0, maxit_ = 500, nblk_ = 0, iters_ = 0;
    bool cert_ = false;  // proj_out invertible: the certified preconditioner step
    double rtol_ = 1e-13, relres_[2] = {-1, -1};
    void *mem_ = nullptr;
    double *gathered_ = nullptr;
    bool deferred_ = true, fuse_ = false, pending_ = false;
    PcgArgs prev_{};               // the last deferred solve's arguments (its pending check)
    double *latch_ = nullptr;      // [8]
    double *cert_part_ = nullptr;  // [workgroups][4] of the certifying tendency
    int64_t cert_part_n_ = 0;      // capacity (workgroups)
};

}  // namespace qg
