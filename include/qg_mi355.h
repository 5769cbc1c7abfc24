/*
 * qg_mi355.h -- C-ABI of the MI355X-native two-layer Phillips (baroclinic QG) hot path.
 *
 * Drop-in boundary for the reference's per-timestep path
 * (JSLeadbetter/julia-ocean-modelling @ 2024-10-08, paths relative to its root):
 *
 *   evolve_zeta!(model, zeta, psi, timestep, f_store)      src/model.jl:155-170
 *   evolve_psi!(model, zeta, psi, poisson_chol, helm_chol) src/model.jl:172-199
 *   get_poisson_cholesky / get_helmholtz_cholesky          src/schemes/laplacian.jl:60-75
 *   run_model_no_output(model)                             src/run_model_no_output.jl:3-16
 *   initialise_model(model)                                src/model.jl:37-62
 *   J, laplace_5p, cd, update_doubly_periodic_bc!          arakawa.jl:58, laplacian.jl:15,
 *                                                          model.jl:68, boundary_conditions.jl:2
 *   sp_solve_modified_helmholtz / sp_solve_poisson         src/schemes/laplacian.jl:78-111
 *
 * Conventions (identical to the reference's arrays):
 *   - every field is IEEE Float64 (or Float32 with params.dtype = QG_F32, model state only),
 *     Julia column-major (M+2) x (P+2) with a one-cell ghost
 *     ring: element (i, j) (0-based, ghosts included) lives at  ptr[i + (M+2)*j];
 *   - the model state zeta, psi, f_store are (M+2, P+2, 2, 3) arrays: layer l (0/1) and
 *     history slot s (0/1/2) of field X start at X + (M+2)*(P+2)*(l + 2*s);
 *   - all pointers are DEVICE pointers owned by the caller (the library never frees them);
 *   - all work is enqueued on the stream given at creation (a hipStream_t passed as void*);
 *     entry points return once the work is enqueued unless documented otherwise;
 *   - every entry point returns 0 on success or a negative qg_status; qg_strerror() names it.
 *     A call that fails leaves the state untouched where it can, and never falls back to a
 *     CPU path.
 *
 * History slots.  The reference shifts slots 3<-2<-1 on every store_new_state! (copies of
 * whole fields).  The library keeps the same three physical slots but rotates a head index
 * instead of copying: after a step the newest field is in slot qg_slot(ctx, which, 1), the
 * previous one in qg_slot(ctx, which, 2), the one before in qg_slot(ctx, which, 3) -- exactly
 * the reference's contents, permuted.  qg_canonicalize() physically restores the reference
 * order (slot 1 first) when a caller needs the arrays back in that order.
 *
 * Multi-GPU: the y-direction (second index) is split into slabs, one rank per GPU; every
 * rank passes its LOCAL P and binds local (M+2, P_local+2, 2, 3) arrays.  Halo rows move
 * with RCCL send/recv; the streamfunction inversion needs one small all-gather per step.
 * The ghost ROWS (memory rows 0 and P+1) of the fields a step writes are refreshed lazily
 * (no kernel reads them; a step's exchange carries only the tendency's halo rows): by
 * qg_synchronize() / qg_canonicalize() / qg_snapshot() / qg_diagnostics(), all slots at once,
 * which a caller invokes before reading the arrays (single GPU: always current).
 */
#ifndef QG_MI355_H
#define QG_MI355_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QG_ABI_VERSION 5

typedef enum {
    QG_OK = 0,
    QG_ERR_INVALID_ARG = -1,  /* bad pointer / size / parameter                         */
    QG_ERR_UNSUPPORTED = -2,  /* configuration the selected solver cannot handle         */
    QG_ERR_HIP = -3,          /* a HIP runtime call failed (launch, alloc, copy)         */
    QG_ERR_NOT_BOUND = -4,    /* state arrays not bound / not initialised               */
    QG_ERR_ALLOC = -5,        /* device allocation failed                                */
    QG_ERR_RCCL = -6,         /* an RCCL call failed or no communicator was set up       */
    QG_ERR_NOT_CONVERGED = -7 /* PCG reached pcg_maxit above pcg_rtol (result is kept)   */
} qg_status;

typedef enum {
    QG_SOLVER_SPECTRAL = 0, /* direct: x-DFT + parallel cyclic tridiagonal solve in y;    *
                             * any M in 3..262144 (M = 2^k <= 8192: FFT passes; odd M     *
                             * above 8192 and M above 16384: Bluestein row transforms),   *
                             * P >= 2 per rank, else UNSUPPORTED.  Both solvers refuse   *
                             * a global P (or M) of 2: the reference's matrix is not the  *
                             * periodic 5-point operator there (laplacian.jl:41-46)       */
    QG_SOLVER_PCG = 1       /* matrix-free PCG on the 5-point operator                     */
} qg_solver_kind;

typedef enum {
    QG_F64 = 0,             /* IEEE Float64 state: the reference's arithmetic              */
    QG_F32 = 1              /* Float32 state (BASELINE config 5); transforms and y-solves  *
                             * still run in F64, the fields and u are stored in F32         */
} qg_dtype;

typedef enum {
    QG_PRECOND_NONE = 0,     /* plain CG                                                   */
    QG_PRECOND_SPECTRAL = 1, /* the spectral direct solve as preconditioner (exact: PCG     *
                              * converges in one iteration and certifies it)               */
    QG_PRECOND_MULTIGRID = 2 /* geometric multigrid V(2,2) cycle (damped Jacobi, full      *
                              * weighting, bilinear prolongation); PCG iterates.  Across   *
                              * slabs: each rank's own V-cycle (block Jacobi).  Needs a    *
                              * coarsest grid <= 4096 points (M, P even down to it).       */
} qg_precond_kind;

/* BaroclinicModel (src/model.jl:12-30) plus build options.  Fill with qg_default_params()
 * first, then set the model fields.  M, P are the interior node counts (P per rank). */
typedef struct qg_params {
    double H_1, H_2, beta, Lx, Ly, dt, T, U;
    int64_t M, P;
    double dx, visc, r, R_d, initial_kick;
    /* back-projection psi_l = P_fwd[2l]*psi~_1 + P_fwd[2l+1]*psi~_2.  Default: the
     * reference's P_matrix(H_1, H_1) = [[1,-1],[1,1]] (src/model.jl:173).           */
    double P_fwd[4];
    int32_t solver;     /* qg_solver_kind (default QG_SOLVER_SPECTRAL)                  */
    int32_t precond;    /* qg_precond_kind for QG_SOLVER_PCG (default SPECTRAL)         */
    double pcg_rtol;    /* relative residual target ||b-Ax||/||b|| (default 1e-12); a   *
                         * run that stagnates at its roundoff floor <= 1e-10 also stops */
    int32_t pcg_maxit;  /* default 500                                                  */
    int32_t chunk_rows; /* y-chunk of the spectral solver; 0 = automatic                */
    int32_t dtype;      /* qg_dtype of the state arrays (default QG_F64; QG_F32 needs   *
                         * QG_SOLVER_SPECTRAL)                                          */
    int32_t reserved0;
    /* Double-gyre wind forcing of the upper layer (an extension: the reference has no wind
     * term; BASELINE config 1 names one).  With wind_tau0 != 0, zeta_f1 gains a last term
     *   + w_j,  w_j = -(2 pi tau0 / (rho0 H_1 Ly)) sin(2 pi (j + 1/2) / P_total)
     * for global interior row j (0-based) and Ly = P_total dx: the curl of the wind stress
     * tau_x = -tau0 cos(2 pi y / Ly) over rho0 H_1.  Default 0 (off: the reference's RHS).  */
    double wind_tau0;   /* N m^-2 (e.g. 0.1)                                            */
    double wind_rho0;   /* kg m^-3 (default 1000)                                       */
} qg_params;

typedef struct qg_ctx qg_ctx;       /* one model instance (one rank) on one device       */
typedef struct qg_solver qg_solver; /* a pair of 5-point periodic solves (the "factors") */

/* per-step solver statistics (host-side copy; reading them synchronises the stream) */
typedef struct qg_stats {
    int32_t iters[2];    /* PCG iterations of the Poisson / Helmholtz solve (0 = direct) */
    double relres[2];    /* ||b - A x|| / ||b|| of the last solve (if measured, else -1) */
    double delta;        /* Poisson compatibility adjustment applied at interior (1,1)   */
    double pin;          /* value subtracted from the Poisson solution (pinning)         */
} qg_stats;

int qg_abi_version(void);
const char *qg_strerror(int status);
void qg_default_params(qg_params *p);

/* ---- model context (replaces the state arrays + the two CHOLMOD factors) ------------ */
/* replaces BaroclinicModel(...) + get_poisson_cholesky / get_helmholtz_cholesky
 * (model.jl:12-34, laplacian.jl:60-75, called at run_model_no_output.jl:5-6)        */
int qg_create(const qg_params *p, int device, void *stream, qg_ctx **out);
int qg_destroy(qg_ctx *ctx);
/* zeta, psi, f_store: device (M+2, P+2, 2, 3) arrays owned by the caller, of the element
 * type params.dtype names (double for QG_F64, float for QG_F32), each 16-byte aligned
 * (the slot moves run on 16-byte vectors; QG_ERR_INVALID_ARG otherwise -- every device
 * allocator's base pointers are, only a sub-allocation at an odd offset is not) */
int qg_bind_state(qg_ctx *ctx, void *zeta, void *psi, void *f_store);
/* initialise_model (model.jl:37-62) on the device, seeded: psi_l interior (i, j) =
 * kick*U*Ly*u01(seed_l, i + M*j_global); zeroes all other slots and f_store; resets the
 * slot rotation. */
int qg_initialise(qg_ctx *ctx, uint64_t seed1, uint64_t seed2);
int qg_evolve_zeta(qg_ctx *ctx, int64_t timestep); /* evolve_zeta! model.jl:155-170; 1-based */
int qg_evolve_psi(qg_ctx *ctx);                    /* evolve_psi! model.jl:172-199        */
int qg_step(qg_ctx *ctx, int64_t timestep);        /* the pair run_model_no_output.jl:11-12 */
int qg_run(qg_ctx *ctx, int64_t first_step, int64_t nsteps); /* loop run_model_no_output.jl:10-13 */
/* which: 0 = zeta, 1 = psi, 2 = f_store; logical 1..3 -> physical 0..2 */
int qg_slot(const qg_ctx *ctx, int which, int logical, int *physical);
int qg_set_slots(qg_ctx *ctx, const int heads[3]); /* restore a saved rotation (resume)  */
int qg_canonicalize(qg_ctx *ctx);                   /* physically reorder to 1,2,3       */
/* store_new_state! semantics (model.jl:102-106) on every call: slot 1 holds the newest
 * values after each qg_evolve_zeta / qg_evolve_psi, as the reference's copies leave them.
 * The history is shifted in place (slot 3 <- 2 <- 1: two slot copies per field, the
 * reference's own data movement) before the new values are written to slot 1, so the heads
 * stay 0 and no qg_canonicalize is needed; on one rank the AB3 tendency moves f_store's
 * history itself as it reads it (each slot rewritten with its periodic ghost images).
 * on = 1 canonicalizes first.  For callers that
 * hand the reference's arrays to every call (evolve_zeta!(model, zeta, psi, t, f_store));
 * qg_run is faster rotating (the default, on = 0).
 * on = QG_KEEP_ORDER_SLOT1 (2): slot 1 of zeta and psi and all three slots of f_store as
 * above after every call, slots 2-3 of zeta and psi NOT maintained -- the reference never
 * reads them (only evolve_zeta_layer! reads f_store's history), so its loop computes the
 * same values: no shifts of zeta and psi; the new zeta is written to slot 2 and copied to
 * slot 1 at the end of qg_evolve_zeta, so slot 1 is the newest after EVERY call.
 * on = QG_KEEP_ORDER_SLOT1_DEFERRED (3): as 2, but the copy of the new zeta into slot 1 is
 * done by the next qg_evolve_psi's first solver pass, which reads it anyway (spectral solver,
 * power-of-two M >= 8, one rank; else the copy of mode 2).  Between qg_evolve_zeta and that
 * qg_evolve_psi, slot 1 of zeta is STALE: qg_slot(ctx, 0, 1, ..) names slot 2 as the newest
 * zeta, and qg_synchronize, qg_canonicalize and every call that moves or rebinds slots
 * complete the move first -- for callers that read zeta only after evolve_psi!, as the
 * reference's loop does (run_model_no_output.jl:10-13).  Switching from either lean mode
 * straight to on = 1 returns QG_ERR_INVALID_ARG (slots 2-3 of zeta and psi hold stale
 * values then).                                                                              */
#define QG_KEEP_ORDER_SLOT1 2
#define QG_KEEP_ORDER_SLOT1_DEFERRED 3
int qg_set_keep_order(qg_ctx *ctx, int on);
int qg_get_stats(qg_ctx *ctx, qg_stats *out);
/* PCG with the spectral preconditioner and an invertible P_fwd (the default) takes the
 * certified step: psi = the spectral solve, accepted when the 5-point residual satisfies
 * ||b - B x|| <= pcg_rtol ||b|| (PCG's first iteration with alpha = 1).  Default: DEFERRED --
 * the residual check runs on the device (on one rank fused into the next step's tendency,
 * which reads exactly that solve's zeta and psi; else as its own pass after the solve) and
 * its verdict is latched there: no host round trip, qg_run can replay PCG steps as HIP graphs.
 * A failed certification is reported (QG_ERR_NOT_CONVERGED, once) by qg_evolve_psi / qg_step
 * within two polling intervals (the latch is copied to the host every QG_PACE_STEPS solves and
 * read one interval later, waiting for that copy if needed: the host stays at most two
 * intervals ahead, so every rank stops at the same step, graph replays included), by the end of qg_run (it settles and reads the
 * latch), by qg_synchronize, and in qg_pcg_certificate's record.  sync = 1: the host reads every
 * residual and runs the general PCG iteration when the certificate fails (the old form).  */
int qg_set_pcg_sync(qg_ctx *ctx, int sync);
/* deferred certificates so far: solves certified, failures, first failing solve (1-based,
 * 0 = none), worst relative residual.  QG_ERR_UNSUPPORTED without the PCG solver.       */
int qg_pcg_certificate(qg_ctx *ctx, int64_t *solves, int64_t *failures, int64_t *first_failure,
                       double *worst_relres);
/* the same, flattened (no struct): PCG iterations and relative residuals of the last solve */
int qg_solver_stats(qg_ctx *ctx, int *it_poisson, int *it_helm, double *relres_p, double *relres_h);
int qg_synchronize(qg_ctx *ctx);

/* ---- snapshot output (run_model.jl:55-95 writes zeta[:,:,:,1], psi[:,:,:,1] every
 * sample_timestep steps) -----------------------------------------------------------------
 * qg_snapshot enqueues, in stream order, a device copy of the newest zeta and psi (both
 * layers, ghost ring included: 2 x (M+2) x (P+2) doubles each, the reference's
 * zeta[:,:,:,1] layout) into a library-owned staging buffer, then returns; a copy stream
 * moves the staging buffer to the caller's HOST buffers (page-locked memory gives an
 * asynchronous copy) while the caller keeps stepping.  A second qg_snapshot first waits for
 * the previous copy.  qg_snapshot_wait blocks until the host buffers are complete.          */
int qg_snapshot(qg_ctx *ctx, void *host_zeta, void *host_psi);  /* elements as params.dtype */
int qg_snapshot_wait(qg_ctx *ctx);

/* ---- diagnostics for monitoring long runs ---------------------------------------------
 * Of the newest zeta / psi, reduced over the whole (multi-GPU: global) domain; interior
 * points only (the ghost ring holds periodic copies).  Synchronous: returns when *out is
 * filled.  Multi-GPU: every rank must call it (one all-gather of a 16-double record through
 * the transport) and all ranks receive the same values.  Accumulated in F64 in a fixed
 * order (reproducible run to run).  Field order = the all-gathered record.               */
typedef struct qg_diag {
    double zeta_max[2], zeta_min[2]; /* update_max / update_min (run_model.jl:41-53) of     *
                                      * zeta[:,:,l,1]                                       */
    double psi_max[2], psi_min[2];   /* the same for psi[:,:,l,1]                           */
    double zeta_sum[2];  /* sum zeta_l dx^2: the circulation, conserved by the scheme       */
    double enstrophy[2]; /* 1/2 sum zeta_l^2 dx^2                                           */
    double energy[2];    /* 1/2 sum |grad psi_l|^2 dx^2, forward differences                */
    double interface;    /* 1/2 sum (psi_1 - psi_2)^2 dx^2 (x S1*H_1/H: potential energy)   */
    double reserved;
} qg_diag;
int qg_diagnostics(qg_ctx *ctx, qg_diag *out);

/* ---- multi-GPU (one rank per GPU, slab decomposition in y) ---------------------------
 * Rank r owns global rows [r*P, (r+1)*P) of a global M x (nranks*P) grid; the y direction is
 * periodic over the ring of ranks.  Per step the library exchanges halo rows with the two
 * ring neighbours and all-gathers one small record per rank (the spectral solver's
 * cross-slab carries); both go through the transport set up here.                       */
int qg_comm_unique_id(char out[128]);               /* ncclGetUniqueId on rank 0          */
/* RCCL.  Collective over the nranks ranks (ncclCommInitRank, then one ring exchange and one
 * all-gather at a small and a large size, so every peer connection the stepping uses exists
 * before the first step: afterwards a peer that stops answering leaves only RCCL kernels
 * waiting on the device, which the bounded waits below abort, never this host thread inside
 * RCCL's lazy connection handshake).                                                     */
int qg_comm_init(qg_ctx *ctx, int nranks, int rank, const char id[128]);
/* Host-provided transport (MPI, tests, ...).  Both callbacks receive DEVICE pointers and the
 * stream the library works on; they must complete the transfer in stream order (e.g.
 * synchronise the stream, copy, exchange, copy back) and return 0 on success.
 * sendrecv: one grouped exchange of ns sends and nr receives (peer = rank index); messages
 * between the same pair of ranks match in posting order.                                 */
typedef int (*qg_allgather_fn)(void *user, const double *send, double *recv, int64_t count, void *stream);
typedef int (*qg_sendrecv_fn)(void *user, int ns, const double *const *send, const int64_t *send_count,
                              const int *send_peer, int nr, double *const *recv, const int64_t *recv_count,
                              const int *recv_peer, void *stream);
int qg_comm_init_host(qg_ctx *ctx, int nranks, int rank, qg_allgather_fn allgather, qg_sendrecv_fn sendrecv,
                      void *user);
/* Failure handling.  With a transport attached, every host wait of the context is bounded:
 * qg_synchronize, qg_diagnostics, qg_get_stats, qg_snapshot_wait, the PCG residual reads, and
 * a pacing wait every QG_PACE_STEPS steps of qg_step / qg_run (which keeps the host at most
 * 2*QG_PACE_STEPS steps ahead, so a hang is seen there rather than in a blocked launch).  The
 * wait polls the stream together with ncclCommGetAsyncError and fails with QG_ERR_RCCL --
 * after ncclCommAbort and one stderr line naming the rank and the call -- on an RCCL error,
 * or when no halo exchange has completed for `seconds` (default 120; the environment variable
 * QG_COMM_TIMEOUT, read when the transport is attached, overrides it).  A failed transport
 * stays failed: every later call that needs it returns QG_ERR_RCCL.  (The reference is one
 * Julia process with no failure handling; this guards the multi-GPU path only.)         */
#define QG_PACE_STEPS 16
int qg_comm_set_timeout(qg_ctx *ctx, double seconds);
/* Halo / interior overlap (north_star: "halo exchange overlapped with interior compute").
 * on = 1: each multi-rank evolve_zeta posts the halo exchange (pack, send/recv, unpack) on a
 * second HIP stream and runs the tendency of the interior rows j in [2, P-2), which need no
 * halo, on the context's stream meanwhile; the four boundary rows follow after an event
 * wait.  Bit-identical to on = 0 (the per-point arithmetic does not depend on the launch
 * geometry).  Default: on (the environment variable QG_OVERLAP=0 at qg_create turns it
 * off): on the 1-rank RCCL ring at 4096^2 it measured 0.5-1.4 % faster than off over three
 * same-process A/B runs (r04) -- the exchange completes inside the interior's tail.
 * No effect on a single GPU (no exchange) or for P < 8 (no interior worth splitting).   */
int qg_set_overlap(qg_ctx *ctx, int on);
/* How the halo rows of a step travel (RCCL transport only; collective: every rank calls it
 * with the same value, after qg_comm_init).
 * QG_HALO_RCCL (default): pack kernel + grouped ncclSend/ncclRecv.
 * QG_HALO_PEER: each rank's receive region (uncached device memory) is opened by its ring
 * neighbours through IPC; the rows are copied by the copy engine (hipMemcpyDeviceToDeviceNoCU)
 * straight from the state into the neighbours' regions, a one-lane kernel raises their
 * arrival flags and a one-lane kernel on the receiving side polls its own (bounded by the
 * comm timeout; a missing peer then fails the transport with QG_ERR_RCCL).  No collective
 * kernel holds compute units, so the exchange proceeds beside the interior tendency.
 * QG_HALO_PUT: the same regions and flags, but the rows are stored by one small kernel
 * (8 workgroups per direction, no LDS, few registers: it fits beside the interior tendency)
 * whose workgroups also wait for the incoming parts -- one launch per exchange, fast in the
 * serial schedule too.
 * QG_ERR_UNSUPPORTED (on every rank, the transport unchanged) when a rank cannot export or
 * open the regions.  The environment variable QG_HALO_PEER=1 (2: QG_HALO_PUT) selects it in
 * qg_comm_init. */
enum { QG_HALO_RCCL = 0, QG_HALO_PEER = 1, QG_HALO_PUT = 2 };
int qg_comm_set_halo_transport(qg_ctx *ctx, int transport);
/* How the direct solver's per-step record all-gather travels (collective, RCCL transport
 * only, spectral solver only: QG_ERR_UNSUPPORTED for PCG).
 * QG_GATHER_RCCL (default): ncclAllGather.
 * QG_GATHER_PEER: one kernel per solve; its workgroups store this rank's record straight into
 * every peer's IPC-mapped receive region (all peers in parallel, each over its own link,
 * instead of a ring of nranks - 1 steps), raise the peer's flag, then wait for the peers'
 * flags and copy their records out (waits bounded by the comm timeout).  The environment
 * variable QG_GATHER_PEER=1 selects it in qg_comm_init. */
enum { QG_GATHER_RCCL = 0, QG_GATHER_PEER = 1 };
int qg_comm_set_gather_transport(qg_ctx *ctx, int transport);
/* Time the two collectives of a multi-GPU step in isolation (HIP events on the context's
 * stream, `reps` back-to-back calls each; every rank calls it): out[0] = ms per halo exchange
 * (pack + grouped send/recv of the depth-2 rows of psi and zeta), out[1] = bytes this rank
 * sends per exchange, out[2] = ms per record all-gather of the direct solve, out[3] = bytes
 * this rank receives per all-gather.  Spectral solver only (QG_ERR_UNSUPPORTED for PCG).    */
int qg_comm_probe(qg_ctx *ctx, int reps, double out[4]);
/* The posting schedule of one halo exchange on `rank` of a ring of `nranks` y-slabs, as the
 * library issues it (RCCL: one ncclGroupStart/End; host transport: one sendrecv call):
 * sends k = 0, 1 go to send_peer[k] from buffer send_buf[k], receives k = 0, 1 come from
 * recv_peer[k] into recv_buf[k]; messages between one pair of ranks match in posting order.
 * Buffers: QG_XBUF_TO_NEXT (the slab's top rows), QG_XBUF_TO_PREV (its bottom rows),
 * QG_XBUF_FROM_PREV (the halo below the slab), QG_XBUF_FROM_NEXT (the halo above it).
 * Pure host function (no device needed): lets a test check the schedule for any ring size. */
enum { QG_XBUF_TO_NEXT = 0, QG_XBUF_TO_PREV = 1, QG_XBUF_FROM_PREV = 2, QG_XBUF_FROM_NEXT = 3 };
int qg_comm_exchange_plan(int rank, int nranks, int send_peer[2], int send_buf[2], int recv_peer[2],
                          int recv_buf[2]);

/* ---- solver handle: the get_*_cholesky analogue --------------------------------------
 * Solves, for s = 0, 1,   A_s x_s = g_s  with A_s = construct_spA(M, P, dx, alpha[s])
 * (the periodic 5-point operator + alpha I, src/schemes/laplacian.jl:54-58) and
 *   g_s = proj_in[2s]*f_1 + proj_in[2s+1]*f_2          (interior of the input fields),
 * pinned[s] != 0 selects the pinned Poisson system of get_poisson_cholesky (alpha must be 0;
 * solution is 0 at interior (1,1)), then writes
 *   out_l = proj_out[2l]*x_1 + proj_out[2l+1]*x_2       with the periodic ghost ring.
 * f_2 / out_2 may be NULL when proj_in / proj_out do not need them.  M or P = 2 (spectral,
 * one rank): the matrices exactly as construct_spA builds them, whose two-point operator is
 * laplacian_1d_periodic(2) = [-2 1; 1 -2] (laplacian.jl:40-45), not the periodic stencil;
 * the PCG kind refuses such domains (QG_ERR_UNSUPPORTED).                                   */
int qg_solver_create(int64_t M, int64_t P, double dx, const double alpha[2], const int pinned[2],
                     const double proj_in[4], const double proj_out[4], int kind, int precond,
                     int device, void *stream, qg_solver **out);
/* the `factor \ b` of sp_solve_* (laplacian.jl:78-111) / model.jl:186,191 */
int qg_solver_solve(qg_solver *s, const double *f_1, const double *f_2, double *out_1, double *out_2);
int qg_solver_destroy(qg_solver *s);

/* ---- kernel-form selection (process-wide) ---------------------------------------------
 * Every kernel's form is chosen by problem size.  qg_set_form forces one form, for the tests
 * that check the alternative forms against each other and for BASELINE config 3's LDS tile
 * sweep; value 0 restores the automatic choice (the default).  Read at every launch
 * (QG_FORM_PCG_NO_CERTIFICATE: when a context's PCG solver is built, i.e. qg_create /
 * qg_comm_init).  qg_get_form returns the current value (or QG_ERR_INVALID_ARG).            */
enum {
    QG_FORM_TENDENCY = 0,           /* QG_TEND_* below                                       */
    QG_FORM_TENDENCY_TILE = 1,      /* (W << 16) | R: the LDS-ring tendency in strips W points  *
                                     * wide (W in 64, 128, 256, 512), about R rows per          *
                                     * workgroup (config 3's tile sweep)                        */
    QG_FORM_ROW_SPLIT = 2,          /* 1: row lengths that are not powers of two take the split *
                                     * pipeline (row transforms and y-recurrences as separate   *
                                     * kernels) at every M, not only above 3200 points          */
    QG_FORM_PCG_NO_CERTIFICATE = 3, /* 1: PCG never takes the one-step certificate; it runs the *
                                     * alpha iteration (z0 = M^-1 b, alpha = (b,z0)/(z0,B z0),  *
                                     * then CG) that non-invertible back-projections need       */
    QG_FORM_COUNT = 4
};
enum { QG_TEND_AUTO = 0, QG_TEND_RING = 1, QG_TEND_DIRECT = 2, QG_TEND_ONE_POINT = 3 };
/* QG_TEND_RING: the LDS-ring kernel at every size; QG_TEND_DIRECT: the cache-resident one-point
 * kernel at every size; QG_TEND_ONE_POINT: Float32 states use the one-point kernels instead of
 * the two-points-per-thread pair kernel (size rule otherwise).  All forms are bit-identical. */
int qg_set_form(int which, int value);
int qg_get_form(int which);

/* ---- stateless kernels on (M+2, P+2) device fields (ghost ring refreshed on output) ---- */
int qg_laplace_5p(const double *u, double *out, int64_t M, int64_t P, double dx, void *stream); /* laplacian.jl:15-27 */
int qg_cd(const double *u, double *out, int64_t M, int64_t P, double dx, void *stream);          /* model.jl:68-80 */
int qg_arakawa_J(const double *zeta, const double *psi, double *out, int64_t M, int64_t P,
                 double dx, void *stream);                             /* J, arakawa.jl:7-62 */
int qg_fill_ghosts(double *b, int64_t M, int64_t P, void *stream); /* boundary_conditions.jl:2-13 */

#ifdef __cplusplus
}
#endif
#endif /* QG_MI355_H */
