// C-ABI implementation (include/qg_mi355.h): model context, slot rotation, solver handles,
// stateless operators.  Everything is enqueued on the caller's stream; nothing in a step
// allocates, synchronises or touches the host.
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>
#include <memory>
#include <new>

#include "qg_common.hpp"
#include "qg_pcg.hpp"
#include "qg_spectral.hpp"

namespace qg {
static std::atomic<int> g_form[QG_FORM_COUNT];  // qg_set_form (zero-initialised: automatic)
int form(int which) { return which >= 0 && which < QG_FORM_COUNT ? g_form[which].load(std::memory_order_relaxed) : 0; }
int comm_destroy(void *comm);
int comm_allgather(void *user, const double *send, double *recv, int64_t count, hipStream_t s);
int comm_halo(void *comm, double *const *fields, int nfields, int64_t M, int64_t P, int depth, double *halo_buf,
              hipStream_t s);
int comm_halo_rows(void *comm, double *const *f2, int n2, int64_t ld, int64_t P, hipStream_t s,
                   const double **rows_out);
int comm_exchange(void *comm, double *const *f2, int n2, double *halo_buf, double *const *f1, int n1, int64_t ld,
                  int64_t P, hipStream_t s, bool ghost_f2);
int comm_init(void **comm, int nranks, int rank, const char id[128]);
int comm_set_peer(void *comm, int on, int64_t ld);
int comm_set_peer_gather(void *comm, int on, int64_t count);
int comm_gather_records(void *user, const double *send, double *recv, int64_t count, hipStream_t s);
int comm_init_host(void **comm, int nranks, int rank, qg_allgather_fn ag, qg_sendrecv_fn sr, void *user);
int comm_unique_id(char out[128]);
int diag_record_len();
size_t diag_scratch_doubles();
int launch_diagnostics(const void *z0, const void *z1, const void *p0, const void *p1, int esize, int64_t M,
                       int64_t P, double dx, double *scratch, double *rec, hipStream_t s);
}  // namespace qg

using namespace qg;

struct qg_solver {
    SpectralSolver spec;
    std::unique_ptr<PcgSolver> pcg;
    hipStream_t stream = nullptr;
    int device = 0;
};

struct qg_ctx {
    qg_params p{};
    Derived d{};
    int device = 0;
    hipStream_t stream = nullptr;
    void *zeta = nullptr, *psi = nullptr, *fst = nullptr;  // element type: p.dtype
    size_t esize = 8;                                     // sizeof(element)
    int heads[3] = {0, 0, 0};  // physical slot of logical slot 1 for zeta, psi, f_store
    bool initialised = false;
    // the (rank, nranks) qg_initialise seeded the state for (-1: the contents came from the
    // caller via qg_bind_state); a transport attached later must match it, or the slabs
    // would hold noise drawn for the wrong global rows
    int seeded_rank = -1, seeded_nranks = -1;
    int rank = 0, nranks = 1;
    bool distributed = false;    // a transport is attached: halo exchange + record gather path
    void *comm = nullptr;        // RCCL communicator wrapper (multi-GPU)
    double *halo = nullptr;      // received halo rows (multi-GPU)
    // multi-GPU: the ghost rows of the fields a step writes are refreshed lazily, grouped
    // with the next step's halo exchange (one RCCL launch) or by qg_synchronize /
    // qg_canonicalize
    bool ghosts_pending = false;
    // snapshots: device staging buffer [zeta 2 layers | psi 2 layers], copy stream + events
    char *snap = nullptr;
    hipStream_t snap_stream = nullptr;
    hipEvent_t snap_ready = nullptr, snap_done = nullptr;
    bool snap_inflight = false;
    // qg_run: three AB3 steps captured as one HIP graph per slot-rotation state (the heads
    // return to their values after three steps), replayed on a private stream
    struct StepGraph {
        hipGraphExec_t exec = nullptr;
        int heads[3] = {0, 0, 0};
    };
    StepGraph graphs[3];
    int ngraphs = 0;
    bool graph_ok = true;  // cleared if capture fails (then qg_run launches step by step)
    hipStream_t gstream = nullptr;
    hipEvent_t gev_in = nullptr, gev_out = nullptr;
    // halo / interior overlap (qg_set_overlap): exchange stream, "fields ready" and "halo in"
    bool overlap = true;  // (qg_set_overlap; default on: measured, r04)
    hipStream_t ov_stream = nullptr;
    hipEvent_t ov_ready = nullptr, ov_halo = nullptr;
    hipEvent_t pace_ev = nullptr;  // multi-GPU pacing (qg_step)
    bool pace_armed = false;
    int64_t pace_count = 0;
    // qg_set_keep_order: every call leaves slot 1 = newest, as store_new_state! does
    // (model.jl:102-106), by shifting the history slots in place before the new values are
    // written; the heads then stay 0.  QG_KEEP_ORDER_SLOT1 (lean): slots 2-3 of zeta and psi,
    // which the reference never reads, are not maintained (no shifts of zeta and psi; the new
    // zeta goes through slot 2, one slot copy at the end of the tendency call);
    // QG_KEEP_ORDER_SLOT1_DEFERRED: the same, the copy deferred as below
    int keep_order = 0;
    // deferred lean mode, single GPU, spectral solver: the new zeta waits in slot 2 (heads[0] =
    // 1) and the next solve's pass A, which reads it anyway, writes it into slot 1
    // (settle_zcopy when anything else comes first)
    bool zcopy_pending = false;
    bool capturing = false;  // a step graph is being captured (no host reads, no polls)
    // deferred PCG: the latch is copied to page-locked memory every QG_PACE_STEPS steps and
    // read one interval later without blocking, so a failed certificate stops qg_step /
    // qg_run within a bounded number of steps
    double *latch_host = nullptr;
    hipEvent_t latch_ev = nullptr;
    bool latch_armed = false;
    int64_t poll_count = 0;
    double *wind = nullptr;  // [P] wind forcing of the local rows (qg_params.wind_tau0 != 0)
    double *diag = nullptr;  // diagnostics scratch: partial records | record | gathered records
    size_t diag_cap = 0;
    std::unique_ptr<SpectralSolver> spec;
    std::unique_ptr<PcgSolver> pcg;
    int last_status = QG_OK;  // of the last solve (PCG: QG_ERR_NOT_CONVERGED is kept here)
    int pcg_sync = -1;        // qg_set_pcg_sync (-1: the environment's / the default)
    int64_t cert_reported = 0;  // deferred PCG certification failures already reported
    size_t F = 0;  // doubles per (M+2, P+2) field

    void *fieldv(void *base, int layer, int slot) const {
        return static_cast<char *>(base) + esize * F * (size_t)(layer + 2 * slot);
    }
    double *field(void *base, int layer, int slot) const { return static_cast<double *>(fieldv(base, layer, slot)); }
    template <class T>
    T *fieldt(void *base, int layer, int slot) const { return static_cast<T *>(fieldv(base, layer, slot)); }
    int64_t row_words() const { return (int64_t)((p.M + 2) * esize / 8); }  // a row, in 8-byte words
};

extern "C" {

int qg_abi_version(void) { return QG_ABI_VERSION; }

int qg_set_form(int which, int value) {
    if (which < 0 || which >= QG_FORM_COUNT || value < 0) return QG_ERR_INVALID_ARG;
    if (which == QG_FORM_TENDENCY && value > QG_TEND_ONE_POINT) return QG_ERR_INVALID_ARG;
    if ((which == QG_FORM_ROW_SPLIT || which == QG_FORM_PCG_NO_CERTIFICATE) && value > 1) return QG_ERR_INVALID_ARG;
    if (which == QG_FORM_TENDENCY_TILE && value != 0) {
        const int w = value >> 16, r = value & 0xffff;
        if ((w != 64 && w != 128 && w != 256 && w != 512) || r < 1) return QG_ERR_INVALID_ARG;
    }
    qg::g_form[which].store(value, std::memory_order_relaxed);
    return QG_OK;
}

int qg_get_form(int which) {
    if (which < 0 || which >= QG_FORM_COUNT) return QG_ERR_INVALID_ARG;
    return qg::form(which);
}

const char *qg_strerror(int s) {
    switch (s) {
        case QG_OK: return "ok";
        case QG_ERR_INVALID_ARG: return "invalid argument";
        case QG_ERR_UNSUPPORTED: return "unsupported configuration";
        case QG_ERR_HIP: return "HIP runtime error";
        case QG_ERR_NOT_BOUND: return "state not bound / not initialised";
        case QG_ERR_ALLOC: return "device allocation failed";
        case QG_ERR_RCCL: return "RCCL error or no communicator";
        case QG_ERR_NOT_CONVERGED: return "PCG did not converge";
        default: return "unknown status";
    }
}

void qg_default_params(qg_params *p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->P_fwd[0] = 1.0;  // P_matrix(H_1, H_1): [[1, -H_1/H_1], [1, 1]]  (model.jl:173)
    p->P_fwd[1] = -1.0;
    p->P_fwd[2] = 1.0;
    p->P_fwd[3] = 1.0;
    p->solver = QG_SOLVER_SPECTRAL;
    p->precond = QG_PRECOND_SPECTRAL;
    p->pcg_rtol = 1e-12;
    p->pcg_maxit = 500;
    p->chunk_rows = 0;
    p->wind_tau0 = 0.0;  // off: the reference's right-hand side
    p->wind_rho0 = 1000.0;
}

static int check_params(const qg_params *p) {
    if (!p) return QG_ERR_INVALID_ARG;
    if (p->M < 2 || p->P < 2 || !(p->dx > 0) || !(p->H_1 > 0) || !(p->H_2 > 0) || !(p->R_d > 0))
        return QG_ERR_INVALID_ARG;
    if (p->solver != QG_SOLVER_SPECTRAL && p->solver != QG_SOLVER_PCG) return QG_ERR_INVALID_ARG;
    if (p->dtype != QG_F64 && p->dtype != QG_F32) return QG_ERR_INVALID_ARG;
    if (p->dtype == QG_F32 && (p->solver != QG_SOLVER_SPECTRAL || (p->M % 2) != 0)) return QG_ERR_UNSUPPORTED;
    if (p->wind_tau0 != 0 && !(p->wind_rho0 > 0)) return QG_ERR_INVALID_ARG;
    return QG_OK;
}

// the wind row table of this rank's slab (built on first use; rebuilt after a comm attach)
static int ensure_wind(qg_ctx *c) {
    const qg_params &p = c->p;
    if (p.wind_tau0 == 0 || c->wind) return QG_OK;
    std::vector<double> w((size_t)p.P);
    const int64_t Pt = p.P * c->nranks, j0 = (int64_t)c->rank * p.P;
    for (int64_t j = 0; j < p.P; ++j) w[j] = wind_row(p.wind_tau0, p.wind_rho0, p.H_1, p.dx, Pt, j0 + j);
    QG_HIP(hipMalloc((void **)&c->wind, sizeof(double) * p.P));
    QG_HIP(hipMemcpy(c->wind, w.data(), sizeof(double) * p.P, hipMemcpyHostToDevice));
    return QG_OK;
}

static void drop_graphs(qg_ctx *c) {
    for (int g = 0; g < c->ngraphs; ++g)
        if (c->graphs[g].exec) (void)hipGraphExecDestroy(c->graphs[g].exec);
    c->ngraphs = 0;
}

static int build_solver(qg_ctx *c) {
    const qg_params &p = c->p;
    const double alpha[2] = {0.0, c->d.Seig};
    QG_HIP(hipSetDevice(c->device));
    drop_graphs(c);
    c->spec.reset();
    c->pcg.reset();
    // the wind table is built here (create / comm attach), never inside a captured step
    QG_CHECK(ensure_wind(c));
    if (p.solver == QG_SOLVER_PCG) {
        auto s = std::make_unique<PcgSolver>();
        QG_CHECK(s->init(p.M, p.P, p.P * c->nranks, c->rank, c->nranks, p.dx, alpha, 1, c->d.Pinv, p.P_fwd,
                         p.precond, p.pcg_rtol, p.pcg_maxit, p.chunk_rows));
        // deferred certification: fused into the next tendency on one rank (no transport)
        s->set_fuse(!c->distributed);
        if (c->pcg_sync >= 0) s->set_deferred(c->pcg_sync == 0);
        QG_CHECK(s->reset_latch(c->stream));
        c->pcg = std::move(s);
        c->cert_reported = 0;
        return QG_OK;
    }
    if (!SpectralSolver::supports(p.M, p.P)) return QG_ERR_UNSUPPORTED;
    auto s = std::make_unique<SpectralSolver>();
    QG_CHECK(s->init(p.M, p.P, p.P * c->nranks, c->rank, c->nranks, p.dx, alpha, 1, c->d.Pinv, p.P_fwd,
                     p.chunk_rows, p.dtype == QG_F32));
    c->spec = std::move(s);
    return QG_OK;
}

int qg_create(const qg_params *p, int device, void *stream, qg_ctx **out) {
    if (!out) return QG_ERR_INVALID_ARG;
    *out = nullptr;
    QG_CHECK(check_params(p));
    qg_ctx *c = new (std::nothrow) qg_ctx();
    if (!c) return QG_ERR_ALLOC;
    c->p = *p;
    c->d = derive(*p);
    c->device = device;
    c->stream = static_cast<hipStream_t>(stream);
    c->F = (size_t)(p->M + 2) * (size_t)(p->P + 2);
    c->esize = p->dtype == QG_F32 ? sizeof(float) : sizeof(double);
    // beta_1 and beta_2 must have opposite signs (model.jl:38)
    if (!((c->d.beta1 > 0 && c->d.beta2 < 0) || (c->d.beta1 < 0 && c->d.beta2 > 0))) {
        delete c;
        return QG_ERR_INVALID_ARG;
    }
    int st = build_solver(c);
    if (st != QG_OK) {
        delete c;
        return st;
    }
    if (const char *e = std::getenv("QG_OVERLAP")) c->overlap = std::atoi(e) != 0;
    *out = c;
    return QG_OK;
}

static int settle_zcopy(qg_ctx *c);

int qg_destroy(qg_ctx *c) {
    if (!c) return QG_OK;
    (void)hipSetDevice(c->device);
    // the caller's arrays outlive the context: a pending lean-mode move completes first (in
    // stream order; the caller synchronises its stream before reading them)
    if (c->zeta) (void)settle_zcopy(c);
    if (c->snap_stream) (void)hipStreamSynchronize(c->snap_stream);
    if (c->snap) (void)hipFree(c->snap);
    if (c->snap_ready) (void)hipEventDestroy(c->snap_ready);
    if (c->snap_done) (void)hipEventDestroy(c->snap_done);
    if (c->snap_stream) (void)hipStreamDestroy(c->snap_stream);
    if (c->ov_stream) (void)hipStreamSynchronize(c->ov_stream);
    if (c->comm) comm_destroy(c->comm);
    if (c->halo) (void)hipFree(c->halo);
    if (c->ov_stream) (void)hipStreamDestroy(c->ov_stream);
    if (c->ov_ready) (void)hipEventDestroy(c->ov_ready);
    if (c->ov_halo) (void)hipEventDestroy(c->ov_halo);
    if (c->diag) (void)hipFree(c->diag);
    if (c->wind) (void)hipFree(c->wind);
    drop_graphs(c);
    if (c->gstream) (void)hipStreamDestroy(c->gstream);
    if (c->gev_in) (void)hipEventDestroy(c->gev_in);
    if (c->gev_out) (void)hipEventDestroy(c->gev_out);
    if (c->pace_ev) (void)hipEventDestroy(c->pace_ev);
    if (c->latch_ev) {
        (void)hipEventSynchronize(c->latch_ev);
        (void)hipEventDestroy(c->latch_ev);
    }
    if (c->latch_host) (void)hipHostFree(c->latch_host);
    delete c;
    return QG_OK;
}

// A deferred PCG certification still waiting for its tendency reads the (zeta, psi) slots of
// its solve; anything that moves, replaces or overwrites those slots runs it first.
static int settle_pcg(qg_ctx *c) {
    if (!c->pcg || !c->pcg->pending()) return QG_OK;
    QG_HIP(hipSetDevice(c->device));
    return c->pcg->certify_pending(c->stream, c->distributed ? comm_allgather : nullptr, c->comm);
}

// Lean keep-order mode: complete a pending move of the new zeta into slot 1 (the solve's pass A
// did not run since the tendency; slots 2-3 of zeta are not maintained in this mode).
static int settle_zcopy(qg_ctx *c) {
    if (!c->zcopy_pending) return QG_OK;
    static const int mv[1][3] = {{1, -1, -1}};
    void *arr[1] = {c->zeta};
    QG_HIP(hipSetDevice(c->device));
    QG_CHECK(launch_slot_move(arr, mv, 1, 2 * c->esize * c->F, c->stream));
    c->heads[0] = 0;
    c->zcopy_pending = false;
    return QG_OK;
}

// (the arrays bound before must still be valid here: a pending certification reads them)
int qg_bind_state(qg_ctx *c, void *zeta, void *psi, void *f_store) {
    if (!c || !zeta || !psi || !f_store) return QG_ERR_INVALID_ARG;
    for (const void *b : {zeta, psi, f_store})  // (launch_slot_move's 16-byte vectors)
        if (reinterpret_cast<uintptr_t>(b) % 16 != 0) return QG_ERR_INVALID_ARG;
    if (c->zeta) QG_CHECK(settle_pcg(c));
    if (c->zeta) QG_CHECK(settle_zcopy(c));
    drop_graphs(c);
    c->zeta = zeta;
    c->psi = psi;
    c->fst = f_store;
    c->heads[0] = c->heads[1] = c->heads[2] = 0;
    c->initialised = true;  // caller-provided contents are taken as the reference layout
    c->seeded_rank = c->seeded_nranks = -1;
    return QG_OK;
}

int qg_initialise(qg_ctx *c, uint64_t seed1, uint64_t seed2) {
    if (!c) return QG_ERR_INVALID_ARG;
    if (!c->zeta) return QG_ERR_NOT_BOUND;
    const qg_params &p = c->p;
    QG_CHECK(settle_pcg(c));
    QG_HIP(hipSetDevice(c->device));
    const double amp = p.initial_kick * p.U * p.Ly;
    QG_CHECK(launch_initialise_global(c->zeta, c->psi, c->fst, (int)c->esize, p.M, p.P, p.P * c->nranks,
                                      (int64_t)c->rank * p.P, amp, c->d.S1, c->d.S2, p.dx, seed1, seed2,
                                      c->stream));
    c->heads[0] = c->heads[1] = c->heads[2] = 0;
    c->zcopy_pending = false;  // (every slot rewritten)
    c->initialised = true;
    c->seeded_rank = c->rank;
    c->seeded_nranks = c->nranks;
    return QG_OK;
}

int qg_slot(const qg_ctx *c, int which, int logical, int *physical) {
    if (!c || !physical || which < 0 || which > 2 || logical < 1 || logical > 3) return QG_ERR_INVALID_ARG;
    *physical = (c->heads[which] + logical - 1) % 3;
    return QG_OK;
}

int qg_set_slots(qg_ctx *c, const int heads[3]) {
    if (!c || !heads) return QG_ERR_INVALID_ARG;
    for (int k = 0; k < 3; ++k)
        if (heads[k] < 0 || heads[k] > 2) return QG_ERR_INVALID_ARG;
    if (c->keep_order && (heads[0] || heads[1] || heads[2])) return QG_ERR_INVALID_ARG;
    QG_CHECK(settle_pcg(c));
    QG_CHECK(settle_zcopy(c));
    for (int k = 0; k < 3; ++k) c->heads[k] = heads[k];
    return QG_OK;
}

extern "C++" {
template <class T>
static void fill_wrap_rows(const qg_ctx *c, const T *base, RowSrcT<T> &rs) {
    // single-GPU: rows -2,-1,P,P+1 are the periodic images P-2,P-1,0,1
    const int64_t P = c->p.P, ld = c->p.M + 2;
    const int64_t rows[4] = {(P - 2 + P) % P, P - 1, 0, 1 % P};
    for (int h = 0; h < 4; ++h) rs.halo[h] = base + fidx(1, rows[h] + 1, ld);
}
}  // extern "C++"

// ---- multi-GPU ghost rows --------------------------------------------------------------
// A step's exchange carries only the tendency's halo rows; the ghost rows (memory rows 0 and
// P+1, the drop-in ghost ring) of every field a step writes are left stale -- no kernel reads
// them -- and refreshed, all slots at once, when a caller needs the arrays (flush_ghosts).
static int all_fields(qg_ctx *c, double *f[18]) {
    int n = 0;
    for (void *base : {c->zeta, c->psi, c->fst})
        for (int slot = 0; slot < 3; ++slot)
            for (int l = 0; l < 2; ++l) f[n++] = c->field(base, l, slot);
    return n;
}

// every host wait of a context: bounded (watchdog) once a transport is attached
static int ctx_wait(qg_ctx *c, const char *what) {
    return comm_wait(c->distributed ? c->comm : nullptr, c->stream, nullptr, what);
}

static int flush_ghosts(qg_ctx *c) {
    if (!c->distributed || !c->ghosts_pending) return QG_OK;
    double *f[18];
    const int n = all_fields(c, f);
    QG_CHECK(comm_exchange(c->comm, nullptr, 0, nullptr, f, n, c->row_words(), c->p.P, c->stream, false));
    c->ghosts_pending = false;
    return QG_OK;
}

extern "C++" {
template <class T>
static int evolve_zeta_t(qg_ctx *c, int64_t timestep) {
    const qg_params &p = c->p;
    // physical slots read (zeta, psi, F(t-1), F(t-2)) and written (zeta, F).  Rotating: the
    // new values go to the oldest slot and the heads move.  keep_order: the history is first
    // shifted in place (slot 3 <- 2 <- 1, as store_new_state! copies), so the inputs are read
    // from slots 2 and 3 and the new values are written to slot 1; the heads stay 0.
    int zh = c->heads[0], fh = c->heads[2], fh2 = (fh + 1) % 3;
    const int ph = c->heads[1];
    int zn = (zh + 2) % 3, fn = (fh + 2) % 3;
    // keep_order, one rank, AB3: f_store's shift rides in the tendency (it reads F(t-1) and
    // F(t-2) at every point anyway and writes them one slot down after reading, fshift1/2), so
    // only zeta is shifted here -- zeta's slot 1 is read with a stencil and cannot be
    // overwritten in place
    const bool fuse_fshift = c->keep_order && !c->distributed && timestep >= 3;
    const bool lean = c->keep_order >= QG_KEEP_ORDER_SLOT1;
    QG_CHECK(settle_zcopy(c));  // (two tendencies in a row: the first one's zeta into slot 1 now)
    if (c->keep_order && !lean) {
        void *arr[2] = {c->zeta, c->fst};
        QG_CHECK(launch_slot_shift(arr, fuse_fshift ? 1 : 2, 2 * c->esize * c->F, c->stream));
        zh = 1;
        fh = fuse_fshift ? 0 : 1;
        fh2 = fuse_fshift ? 1 : 2;
        zn = fn = 0;
    } else if (lean) {  // zeta: read slot 1, new values to slot 2, copied to slot 1 below
        if (!fuse_fshift) {
            void *arr[1] = {c->fst};
            QG_CHECK(launch_slot_shift(arr, 1, 2 * c->esize * c->F, c->stream));
        }
        zh = 0;
        zn = 1;
        fh = fuse_fshift ? 0 : 1;
        fh2 = fuse_fshift ? 1 : 2;
        fn = 0;
    }
    TendArgsT<T> a{};
    a.M = p.M;
    a.P = p.P;
    a.ld = p.M + 2;
    a.dx = p.dx;
    a.visc = p.visc;
    a.dt = p.dt;
    a.U = p.U;
    a.r = p.r;
    a.beta[0] = c->d.beta1;
    a.beta[1] = c->d.beta2;
    a.ab3 = timestep >= 3;
    a.j0 = 0;
    a.j1 = (int)p.P;
    a.write_ghost_rows = !c->distributed;
    QG_CHECK(ensure_wind(c));
    a.wind = c->wind;
    for (int l = 0; l < 2; ++l) {
        a.zeta[l] = c->fieldt<T>(c->zeta, l, zh);
        a.psi[l] = c->fieldt<T>(c->psi, l, ph);
        a.fprev1[l] = c->fieldt<T>(c->fst, l, fh);
        a.fprev2[l] = c->fieldt<T>(c->fst, l, fh2);
        a.zeta_out[l] = c->fieldt<T>(c->zeta, l, zn);
        a.f_out[l] = c->fieldt<T>(c->fst, l, fn);
        if (fuse_fshift) {
            a.fshift1[l] = c->fieldt<T>(c->fst, l, 1);
            a.fshift2[l] = c->fieldt<T>(c->fst, l, 2);
        }
    }
    if (!c->distributed) {
        for (int l = 0; l < 2; ++l) {
            fill_wrap_rows(c, a.zeta[l], a.zeta_rows[l]);
            fill_wrap_rows(c, a.psi[l], a.psi_rows[l]);
        }
        bool done = false;
        if constexpr (std::is_same<T, double>::value) {
            // the previous solve's deferred PCG certification rides in this tendency (it reads
            // exactly that solve's zeta and psi)
            if (c->pcg && c->pcg->pending()) {
                c->pcg->fill_cert_args(a);
                int nblk = 0;
                QG_CHECK(launch_tendency_cert(a, c->pcg->cert_capacity(), &nblk, c->stream));
                QG_CHECK(c->pcg->latch_fused(nblk, c->stream));
                done = true;
            }
        }
        if (!done) QG_CHECK(launch_tendency(a, c->stream));
    } else {
        // halo rows of psi (depth 2; zeta uses the inner two) from the neighbouring slabs, read
        // by the tendency where they are received (comm_halo_rows: no unpack, no ghost rows)
        double *f2[4] = {c->field(c->psi, 0, ph), c->field(c->psi, 1, ph), c->field(c->zeta, 0, zh),
                         c->field(c->zeta, 1, zh)};
        const double *hr[16];
        auto set_halo = [&]() {  // (+1: the interior start of a received row)
            for (int l = 0; l < 2; ++l)
                for (int h = 0; h < 4; ++h) {
                    a.psi_rows[l].halo[h] = reinterpret_cast<const T *>(hr[4 * l + h]) + 1;
                    a.zeta_rows[l].halo[h] = reinterpret_cast<const T *>(hr[4 * (2 + l) + h]) + 1;
                }
        };
        if (c->overlap && p.P >= 8) {
            // exchange on the side stream, ordered after everything already queued on the
            // context's stream (the previous step's pass B, a ghost flush using the staging
            // buffer); the interior rows [2, P-2) read only local rows -- no halo, no ghost
            // row -- and write rows the unpack never touches, so they run meanwhile
            if (!c->ov_stream) {
                QG_HIP(hipStreamCreateWithFlags(&c->ov_stream, hipStreamNonBlocking));
                QG_HIP(hipEventCreateWithFlags(&c->ov_ready, hipEventDisableTiming));
                QG_HIP(hipEventCreateWithFlags(&c->ov_halo, hipEventDisableTiming));
            }
            QG_HIP(hipEventRecord(c->ov_ready, c->stream));
            QG_HIP(hipStreamWaitEvent(c->ov_stream, c->ov_ready, 0));
            QG_CHECK(comm_halo_rows(c->comm, f2, 4, c->row_words(), p.P, c->ov_stream, hr));
            QG_HIP(hipEventRecord(c->ov_halo, c->ov_stream));
            set_halo();
            TendArgsT<T> in = a;
            in.j0 = 2;
            in.j1 = (int)p.P - 2;
            in.j2 = in.j3 = 0;
            QG_CHECK(launch_tendency(in, c->stream));
            QG_HIP(hipStreamWaitEvent(c->stream, c->ov_halo, 0));
            TendArgsT<T> bd = a;  // rows 0, 1 and P-2, P-1: one launch, two row ranges
            bd.j0 = 0;
            bd.j1 = 2;
            bd.j2 = (int)p.P - 2;
            bd.j3 = (int)p.P;
            QG_CHECK(launch_tendency(bd, c->stream));
        } else {
            QG_CHECK(comm_halo_rows(c->comm, f2, 4, c->row_words(), p.P, c->stream, hr));
            set_halo();
            QG_CHECK(launch_tendency(a, c->stream));
        }
        c->ghosts_pending = true;
    }
    if (lean) {
        if (c->keep_order == QG_KEEP_ORDER_SLOT1_DEFERRED && c->spec && !c->distributed &&
            c->spec->fuses_input_copy()) {
            // the next solve's pass A reads the new zeta from slot 2 and writes it into slot 1
            // (stores only; r04n's separate move read and wrote the whole field, ~0.09 ms at
            // 4096^2); meanwhile qg_slot names slot 2 as the newest
            zn = 1;
            c->zcopy_pending = true;
        } else {  // slot 1 <- slot 2 (ghost rows too; multi-rank: refreshed by the lazy flush)
            static const int mv[1][3] = {{1, -1, -1}};
            void *arr[1] = {c->zeta};
            QG_CHECK(launch_slot_move(arr, mv, 1, 2 * c->esize * c->F, c->stream));
            zn = 0;
        }
    }
    c->heads[0] = zn;
    c->heads[2] = fn;
    return QG_OK;
}
}  // extern "C++"

int qg_evolve_zeta(qg_ctx *c, int64_t timestep) {
    if (!c || timestep < 1) return QG_ERR_INVALID_ARG;
    if (!c->initialised || !c->zeta) return QG_ERR_NOT_BOUND;
    QG_HIP(hipSetDevice(c->device));
    return c->esize == sizeof(float) ? evolve_zeta_t<float>(c, timestep) : evolve_zeta_t<double>(c, timestep);
}

// Deferred PCG: report new certification failures the device has latched.  Polling (wait =
// false, `steps` more steps enqueued on stream `on`): every QG_PACE_STEPS steps, read the copy
// of the latch made one interval earlier -- waiting for it if it has not landed (bounded), so
// the host is never more than two intervals ahead of the device and a failure is reported at
// a fixed step count: on one rank whatever the host's lead (graph replays enqueue far faster
// than the device runs them), and with a transport at the same step on every rank (the verdict
// comes from all-gathered sums, identical everywhere; one rank returning while its peers step
// into the next exchange would leave them in a mismatched collective).  Final (wait = true,
// the end of qg_run): settle the pending check and read the latch now.
static int poll_pcg(qg_ctx *c, bool wait, int steps = 1, hipStream_t on = nullptr) {
    if (!c->pcg || !c->pcg->deferred() || c->capturing) return QG_OK;
    if (!on) on = c->stream;
    if (!c->latch_host) {
        QG_HIP(hipHostMalloc((void **)&c->latch_host, sizeof(double) * 8, hipHostMallocDefault));
        QG_HIP(hipEventCreateWithFlags(&c->latch_ev, hipEventDisableTiming));
    }
    auto report = [&]() -> int {
        const int64_t f = (int64_t)c->latch_host[1];
        if (f > c->cert_reported) {
            c->cert_reported = f;
            return QG_ERR_NOT_CONVERGED;
        }
        return QG_OK;
    };
    if (wait) {
        QG_CHECK(settle_pcg(c));
        if (c->latch_armed) QG_CHECK(comm_wait(c->distributed ? c->comm : nullptr, c->stream, c->latch_ev,
                                               "qg_run (PCG latch)"));
        QG_HIP(hipMemcpyAsync(c->latch_host, c->pcg->latch(), sizeof(double) * 8, hipMemcpyDeviceToHost, c->stream));
        QG_HIP(hipEventRecord(c->latch_ev, c->stream));
        QG_CHECK(comm_wait(c->distributed ? c->comm : nullptr, c->stream, c->latch_ev, "qg_run (PCG latch)"));
        c->latch_armed = false;
        return report();
    }
    const int64_t before = c->poll_count;
    c->poll_count += steps;
    if (before / QG_PACE_STEPS == c->poll_count / QG_PACE_STEPS) return QG_OK;
    if (c->latch_armed) {
        QG_CHECK(comm_wait(c->distributed ? c->comm : nullptr, on, c->latch_ev, "qg_evolve_psi (PCG latch)"));
        c->latch_armed = false;
        QG_CHECK(report());
    }
    QG_HIP(hipMemcpyAsync(c->latch_host, c->pcg->latch(), sizeof(double) * 8, hipMemcpyDeviceToHost, on));
    QG_HIP(hipEventRecord(c->latch_ev, on));
    c->latch_armed = true;
    return QG_OK;
}

int qg_evolve_psi(qg_ctx *c) {
    if (!c) return QG_ERR_INVALID_ARG;
    if (!c->initialised || !c->zeta) return QG_ERR_NOT_BOUND;
    if (!c->spec && !c->pcg) return QG_ERR_UNSUPPORTED;
    QG_HIP(hipSetDevice(c->device));
    const int zh = c->heads[0];
    int pn = (c->heads[1] + 2) % 3;
    if (c->keep_order) {  // store_new_state!'s shift of psi (lean: none), then the solve writes slot 1
        if (c->keep_order < QG_KEEP_ORDER_SLOT1) {
            void *arr[1] = {c->psi};
            QG_CHECK(launch_slot_shift(arr, 1, 2 * c->esize * c->F, c->stream));
        }
        pn = 0;
    }
    double *o1 = c->field(c->psi, 0, pn), *o2 = c->field(c->psi, 1, pn);  // (element type p.dtype)
    const double *z1 = c->field(c->zeta, 0, zh), *z2 = c->field(c->zeta, 1, zh);
    if (c->pcg) {
        const int st = c->pcg->solve(z1, z2, o1, o2, !c->distributed, c->stream,
                                     c->distributed ? comm_allgather : nullptr, c->comm,
                                     c->distributed ? comm_halo : nullptr, c->comm);
        c->last_status = st;
        if (st != QG_OK && st != QG_ERR_NOT_CONVERGED) return st;
    } else {
        void *zc1 = nullptr, *zc2 = nullptr;
        if (c->zcopy_pending) {  // pass A also moves the new zeta (slot 2) into slot 1
            zc1 = c->field(c->zeta, 0, 0);
            zc2 = c->field(c->zeta, 1, 0);
        }
        QG_CHECK(c->spec->solve(z1, z2, o1, o2, !c->distributed, c->stream,
                                c->distributed ? comm_gather_records : nullptr, c->comm, nullptr, nullptr, zc1, zc2));
        if (c->zcopy_pending) {
            c->heads[0] = 0;
            c->zcopy_pending = false;
        }
    }
    c->heads[1] = pn;
    if (c->distributed) c->ghosts_pending = true;  // psi's ghost rows: at the next ghost flush
    if (c->pcg) QG_CHECK(poll_pcg(c, false));  // deferred certificates: the bounded-delay report
    return c->pcg ? c->last_status : QG_OK;
}

// Multi-GPU pacing: every QG_PACE_STEPS steps, wait (bounded) for the event recorded
// QG_PACE_STEPS steps earlier, then record a new one.  The host stays 1-2 intervals ahead of
// the device (enough to keep the queue full), and a dead peer surfaces as QG_ERR_RCCL from
// the watchdog instead of a host blocked inside a launch on a full queue.
static int pace(qg_ctx *c) {
    if (!c->distributed || ++c->pace_count % QG_PACE_STEPS != 0) return QG_OK;
    if (!c->pace_ev) QG_HIP(hipEventCreateWithFlags(&c->pace_ev, hipEventDisableTiming));
    if (c->pace_armed) QG_CHECK(comm_wait(c->comm, c->stream, c->pace_ev, "qg_run (pacing wait)"));
    QG_HIP(hipEventRecord(c->pace_ev, c->stream));
    c->pace_armed = true;
    return QG_OK;
}

int qg_step(qg_ctx *c, int64_t timestep) {
    QG_CHECK(qg_evolve_zeta(c, timestep));
    const int st = qg_evolve_psi(c);
    if (st != QG_OK && st != QG_ERR_NOT_CONVERGED) return st;
    QG_CHECK(pace(c));
    return st;
}

// Graph replay of AB3 steps (single GPU, spectral solver: no host round trips in a step),
// opt-in with QG_GRAPH=1: on ROCm 7.2 / MI355X replaying the captured graph measured slower
// than launching the same kernels on the stream (0.87x at 128^2 .. 0.99x at 4096^2,
// tools/graph_bench.py), so stream launches are the default.
static bool graphs_enabled(const qg_ctx *c) {
    const char *e = std::getenv("QG_GRAPH");
    // (PCG: only the deferred form, which never reads the residual on the host)
    return e && std::atoi(e) != 0 && c->graph_ok && !c->distributed && (c->spec || (c->pcg && c->pcg->deferred()));
}

// the graph of three AB3 steps starting from the current slot rotation (captured on first use)
static int step_graph(qg_ctx *c, hipGraphExec_t *out) {
    for (int g = 0; g < c->ngraphs; ++g)
        if (std::memcmp(c->graphs[g].heads, c->heads, sizeof(c->heads)) == 0) {
            *out = c->graphs[g].exec;
            return QG_OK;
        }
    if (c->ngraphs == 3) drop_graphs(c);
    if (!c->gstream) {
        QG_HIP(hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking));
        QG_HIP(hipEventCreateWithFlags(&c->gev_in, hipEventDisableTiming));
        QG_HIP(hipEventCreateWithFlags(&c->gev_out, hipEventDisableTiming));
    }
    int heads0[3];
    std::memcpy(heads0, c->heads, sizeof(heads0));
    hipStream_t saved = c->stream;
    c->stream = c->gstream;
    c->capturing = true;
    hipGraph_t graph = nullptr;
    int st = hipStreamBeginCapture(c->gstream, hipStreamCaptureModeThreadLocal) == hipSuccess ? QG_OK : QG_ERR_HIP;
    if (st == QG_OK) {
        for (int k = 0; k < 3 && st == QG_OK; ++k) st = qg_step(c, 3 + k);  // any t >= 3: AB3
        if (hipStreamEndCapture(c->gstream, &graph) != hipSuccess) st = QG_ERR_HIP;
    }
    c->stream = saved;
    c->capturing = false;
    std::memcpy(c->heads, heads0, sizeof(heads0));  // (three steps: the rotation is back anyway)
    hipGraphExec_t exec = nullptr;
    if (st == QG_OK && hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) st = QG_ERR_HIP;
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipGetLastError();
    if (st != QG_OK) {
        c->graph_ok = false;  // launch step by step from now on
        return st;
    }
    c->graphs[c->ngraphs].exec = exec;
    std::memcpy(c->graphs[c->ngraphs].heads, heads0, sizeof(heads0));
    ++c->ngraphs;
    *out = exec;
    return QG_OK;
}

int qg_run(qg_ctx *c, int64_t first_step, int64_t nsteps) {
    if (!c || first_step < 1 || nsteps < 0) return QG_ERR_INVALID_ARG;
    int64_t t = first_step;
    const int64_t end = first_step + nsteps;
    for (; t < end && t < 3; ++t) QG_CHECK(qg_step(c, t));  // the Euler steps
    // deferred PCG: a captured graph's first tendency certifies the solve before it only if
    // that check was pending at capture; capture and replay only in that steady state (one
    // stream step first when a standalone check has already settled it)
    if (end - t >= 7 && graphs_enabled(c) && c->pcg && !c->pcg->pending()) QG_CHECK(qg_step(c, t++));
    if (end - t >= 6 && graphs_enabled(c) && c->initialised && c->zeta && (!c->pcg || c->pcg->pending())) {
        QG_HIP(hipSetDevice(c->device));
        hipGraphExec_t g = nullptr;
        if (step_graph(c, &g) == QG_OK) {
            const int64_t cycles = (end - t) / 3;
            QG_HIP(hipEventRecord(c->gev_in, c->stream));  // after the caller's earlier work
            QG_HIP(hipStreamWaitEvent(c->gstream, c->gev_in, 0));
            int st = QG_OK;
            int64_t k = 0;
            while (k < cycles && st == QG_OK) {
                QG_HIP(hipGraphLaunch(g, c->gstream));
                ++k;
                // deferred PCG: the bounded-delay latch poll between replays, as qg_step does it
                if (c->pcg) st = poll_pcg(c, false, 3, c->gstream);
            }
            QG_HIP(hipEventRecord(c->gev_out, c->gstream));
            QG_HIP(hipStreamWaitEvent(c->stream, c->gev_out, 0));  // before the caller's later work
            t += 3 * k;
            if (st != QG_OK) return st;
        }
    }
    for (; t < end; ++t) QG_CHECK(qg_step(c, t));
    return poll_pcg(c, true);  // deferred PCG: a failed certificate is reported by the run
}

int qg_canonicalize(qg_ctx *c) {
    if (!c) return QG_ERR_INVALID_ARG;
    if (!c->zeta) return QG_ERR_NOT_BOUND;
    QG_HIP(hipSetDevice(c->device));
    QG_CHECK(flush_ghosts(c));  // pending ghost-ring refreshes
    QG_CHECK(settle_pcg(c));    // (its check reads the slots about to move)
    QG_CHECK(settle_zcopy(c));
    // one launch rotates every field whose newest slot is not physical 0: new slot q <- old
    // slot (head + q) mod 3, each slot read once and written once, in place
    void *arr[3];
    int src[3][3], n = 0;
    void *bases[3] = {c->zeta, c->psi, c->fst};
    for (int w = 0; w < 3; ++w) {
        if (c->heads[w] == 0) continue;
        arr[n] = bases[w];
        for (int q = 0; q < 3; ++q) src[n][q] = (c->heads[w] + q) % 3;
        ++n;
    }
    if (n) QG_CHECK(launch_slot_move(arr, src, n, 2 * c->esize * c->F, c->stream));
    c->heads[0] = c->heads[1] = c->heads[2] = 0;
    return QG_OK;
}

int qg_set_keep_order(qg_ctx *c, int on) {
    if (!c || on < 0 || on > QG_KEEP_ORDER_SLOT1_DEFERRED) return QG_ERR_INVALID_ARG;
    // slots 2-3 of zeta and psi were not maintained in the lean modes: full keep-order could
    // not keep its promise for the next two calls
    if (on == 1 && c->keep_order >= QG_KEEP_ORDER_SLOT1) return QG_ERR_INVALID_ARG;
    QG_CHECK(settle_zcopy(c));
    if (on && !c->keep_order && c->zeta) QG_CHECK(qg_canonicalize(c));
    if (c->keep_order != on) drop_graphs(c);
    c->keep_order = on;
    return QG_OK;
}

int qg_get_stats(qg_ctx *c, qg_stats *out) {
    if (!c || !out) return QG_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    out->relres[0] = out->relres[1] = -1;
    if (c->pcg) {
        out->iters[0] = out->iters[1] = c->pcg->iterations();
        out->relres[0] = c->pcg->relres(0);
        out->relres[1] = c->pcg->relres(1);
        if (c->pcg->deferred()) {  // the last certified solve's residuals, from the latch
            double lt[8];
            QG_HIP(hipSetDevice(c->device));
            QG_CHECK(c->pcg->certify_pending(c->stream, c->distributed ? comm_allgather : nullptr, c->comm));
            QG_HIP(hipMemcpyAsync(lt, c->pcg->latch(), sizeof(lt), hipMemcpyDeviceToHost, c->stream));
            QG_CHECK(ctx_wait(c, "qg_get_stats"));
            out->relres[0] = lt[4];
            out->relres[1] = lt[5];
        }
        return QG_OK;
    }
    if (!c->spec) return QG_OK;
    double sc[2];
    QG_HIP(hipSetDevice(c->device));
    QG_HIP(hipMemcpyAsync(sc, c->spec->args().scal, sizeof(sc), hipMemcpyDeviceToHost, c->stream));
    QG_CHECK(ctx_wait(c, "qg_get_stats"));
    out->delta = sc[0];
    out->pin = sc[1];
    return QG_OK;
}

int qg_solver_stats(qg_ctx *c, int *it_poisson, int *it_helm, double *relres_p, double *relres_h) {
    qg_stats st;
    const int rc = qg_get_stats(c, &st);
    if (rc != QG_OK) return rc;
    if (it_poisson) *it_poisson = st.iters[0];
    if (it_helm) *it_helm = st.iters[1];
    if (relres_p) *relres_p = st.relres[0];
    if (relres_h) *relres_h = st.relres[1];
    return QG_OK;
}

int qg_snapshot(qg_ctx *c, void *host_zeta, void *host_psi) {
    if (!c || !host_zeta || !host_psi) return QG_ERR_INVALID_ARG;
    if (!c->initialised || !c->zeta) return QG_ERR_NOT_BOUND;
    QG_HIP(hipSetDevice(c->device));
    if (!c->snap) {
        QG_HIP(hipMalloc((void **)&c->snap, c->esize * 4 * c->F));
        QG_HIP(hipStreamCreateWithFlags(&c->snap_stream, hipStreamNonBlocking));
        QG_HIP(hipEventCreateWithFlags(&c->snap_ready, hipEventDisableTiming));
        QG_HIP(hipEventCreateWithFlags(&c->snap_done, hipEventDisableTiming));
    }
    QG_CHECK(flush_ghosts(c));  // multi-GPU: the ghost rows of the newest fields
    if (c->snap_inflight) QG_HIP(hipStreamWaitEvent(c->stream, c->snap_done, 0));  // staging free
    const size_t fb = c->esize * c->F;
    for (int l = 0; l < 2; ++l) {
        QG_HIP(hipMemcpyAsync(c->snap + l * fb, c->fieldv(c->zeta, l, c->heads[0]), fb, hipMemcpyDeviceToDevice,
                              c->stream));
        QG_HIP(hipMemcpyAsync(c->snap + (2 + l) * fb, c->fieldv(c->psi, l, c->heads[1]), fb,
                              hipMemcpyDeviceToDevice, c->stream));
    }
    QG_HIP(hipEventRecord(c->snap_ready, c->stream));
    QG_HIP(hipStreamWaitEvent(c->snap_stream, c->snap_ready, 0));
    QG_HIP(hipMemcpyAsync(host_zeta, c->snap, 2 * fb, hipMemcpyDeviceToHost, c->snap_stream));
    QG_HIP(hipMemcpyAsync(host_psi, c->snap + 2 * fb, 2 * fb, hipMemcpyDeviceToHost, c->snap_stream));
    QG_HIP(hipEventRecord(c->snap_done, c->snap_stream));
    c->snap_inflight = true;
    return QG_OK;
}

int qg_snapshot_wait(qg_ctx *c) {
    if (!c) return QG_ERR_INVALID_ARG;
    if (!c->snap_inflight) return QG_OK;
    QG_HIP(hipSetDevice(c->device));
    QG_CHECK(comm_wait(c->distributed ? c->comm : nullptr, c->snap_stream, c->snap_done, "qg_snapshot_wait"));
    c->snap_inflight = false;
    return QG_OK;
}

int qg_diagnostics(qg_ctx *c, qg_diag *out) {
    if (!c || !out) return QG_ERR_INVALID_ARG;
    if (!c->initialised || !c->zeta) return QG_ERR_NOT_BOUND;
    constexpr int NREC = (int)(sizeof(qg_diag) / sizeof(double));
    static_assert(NREC == 16, "qg_diag is the 16-double diagnostics record");
    if (diag_record_len() != NREC) return QG_ERR_UNSUPPORTED;
    QG_HIP(hipSetDevice(c->device));
    const size_t scratch = diag_scratch_doubles();
    // sized for the largest world a context can join (a ctx re-attached to a bigger ring reallocates)
    const size_t need = scratch + (size_t)NREC * c->nranks;
    if (c->diag && c->diag_cap < need) {
        QG_CHECK(ctx_wait(c, "qg_diagnostics"));
        QG_HIP(hipFree(c->diag));
        c->diag = nullptr;
    }
    if (!c->diag) {
        QG_HIP(hipMalloc((void **)&c->diag, sizeof(double) * need));
        c->diag_cap = need;
    }
    QG_CHECK(flush_ghosts(c));  // the forward differences read psi's ghost row P+1
    const int zh = c->heads[0], ph = c->heads[1];
    double *rec = c->diag + scratch - NREC, *all = c->diag + scratch;
    QG_CHECK(launch_diagnostics(c->fieldv(c->zeta, 0, zh), c->fieldv(c->zeta, 1, zh), c->fieldv(c->psi, 0, ph),
                                c->fieldv(c->psi, 1, ph), (int)c->esize, c->p.M, c->p.P, c->p.dx, c->diag, rec,
                                c->stream));
    const double *src = rec;
    if (c->distributed) {
        QG_CHECK(comm_allgather(c->comm, rec, all, NREC, c->stream));
        src = all;
    }
    const int n = c->distributed ? c->nranks : 1;
    std::unique_ptr<double[]> h(new (std::nothrow) double[(size_t)NREC * n]);
    if (!h) return QG_ERR_ALLOC;
    QG_HIP(hipMemcpyAsync(h.get(), src, sizeof(double) * NREC * n, hipMemcpyDeviceToHost, c->stream));
    QG_CHECK(ctx_wait(c, "qg_diagnostics"));
    double v[NREC];
    std::memcpy(v, h.get(), sizeof(v));
    for (int r = 1; r < n; ++r) {  // rank order: the same sums on every rank
        const double *q = h.get() + (size_t)NREC * r;
        for (int l = 0; l < 2; ++l) {
            // NaN-propagating, like Julia's maximum / minimum (qg_diag.hip)
            auto nmax = [](double a, double b) { return (a != a || b != b) ? a + b : std::fmax(a, b); };
            auto nmin = [](double a, double b) { return (a != a || b != b) ? a + b : std::fmin(a, b); };
            v[0 + l] = nmax(v[0 + l], q[0 + l]);
            v[2 + l] = nmin(v[2 + l], q[2 + l]);
            v[4 + l] = nmax(v[4 + l], q[4 + l]);
            v[6 + l] = nmin(v[6 + l], q[6 + l]);
        }
        for (int k = 8; k < NREC; ++k) v[k] += q[k];
    }
    v[NREC - 1] = 0.0;
    std::memcpy(out, v, sizeof(v));
    return QG_OK;
}

int qg_synchronize(qg_ctx *c) {
    if (!c) return QG_ERR_INVALID_ARG;
    QG_HIP(hipSetDevice(c->device));
    QG_CHECK(flush_ghosts(c));
    QG_CHECK(settle_zcopy(c));
    if (c->pcg && c->pcg->deferred()) {  // deferred PCG: new certification failures?
        QG_CHECK(c->pcg->certify_pending(c->stream, c->distributed ? comm_allgather : nullptr, c->comm));
        double lt[8];
        QG_HIP(hipMemcpyAsync(lt, c->pcg->latch(), sizeof(lt), hipMemcpyDeviceToHost, c->stream));
        QG_CHECK(ctx_wait(c, "qg_synchronize"));
        if ((int64_t)lt[1] > c->cert_reported) {
            c->cert_reported = (int64_t)lt[1];
            return QG_ERR_NOT_CONVERGED;
        }
        return QG_OK;
    }
    return ctx_wait(c, "qg_synchronize");
}

int qg_set_pcg_sync(qg_ctx *c, int sync) {
    if (!c) return QG_ERR_INVALID_ARG;
    c->pcg_sync = sync != 0 ? 1 : 0;
    if (c->pcg) {
        QG_HIP(hipSetDevice(c->device));
        QG_CHECK(c->pcg->certify_pending(c->stream, c->distributed ? comm_allgather : nullptr, c->comm));
        c->pcg->set_deferred(sync == 0);
    }
    return QG_OK;
}

int qg_pcg_certificate(qg_ctx *c, int64_t *solves, int64_t *failures, int64_t *first_failure, double *worst_relres) {
    if (!c) return QG_ERR_INVALID_ARG;
    if (!c->pcg) return QG_ERR_UNSUPPORTED;
    QG_HIP(hipSetDevice(c->device));
    QG_CHECK(c->pcg->certify_pending(c->stream, c->distributed ? comm_allgather : nullptr, c->comm));
    double lt[8];
    QG_HIP(hipMemcpyAsync(lt, c->pcg->latch(), sizeof(lt), hipMemcpyDeviceToHost, c->stream));
    QG_CHECK(ctx_wait(c, "qg_pcg_certificate"));
    if (solves) *solves = (int64_t)lt[0];
    if (failures) *failures = (int64_t)lt[1];
    if (first_failure) *first_failure = (int64_t)lt[2];
    if (worst_relres) *worst_relres = lt[3];
    return QG_OK;
}

// ---- multi-GPU -------------------------------------------------------------------------
int qg_set_overlap(qg_ctx *c, int on) {
    if (!c) return QG_ERR_INVALID_ARG;
    c->overlap = on != 0;
    return QG_OK;
}

int qg_comm_set_timeout(qg_ctx *c, double seconds) {
    if (!c || !(seconds > 0)) return QG_ERR_INVALID_ARG;
    if (!c->comm) return QG_ERR_RCCL;
    return comm_set_timeout(c->comm, seconds);
}

int qg_comm_unique_id(char out[128]) {
    if (!out) return QG_ERR_INVALID_ARG;
    return comm_unique_id(out);
}

// a state seeded by qg_initialise for another slab layout holds noise drawn for the wrong
// global rows: refuse instead of stepping it (re-run qg_initialise after attaching).  Checked
// before a communicator is created, so a refused attach leaves the context as it was.
static bool seeded_for_other_slab(const qg_ctx *c, int nranks, int rank) {
    return c->initialised && c->seeded_nranks > 0 && (c->seeded_nranks != nranks || c->seeded_rank != rank);
}

static int comm_attach(qg_ctx *c, int nranks, int rank) {
    c->rank = rank;
    c->nranks = nranks;
    if (c->wind) {  // the slab's global rows changed
        (void)hipFree(c->wind);
        c->wind = nullptr;
    }
    c->distributed = true;  // also for nranks == 1: the ring then wraps onto itself
    if (!c->halo) QG_HIP(hipMalloc((void **)&c->halo, sizeof(double) * 16 * (size_t)(c->p.M + 2)));
    return build_solver(c);
}

int qg_comm_init(qg_ctx *c, int nranks, int rank, const char id[128]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return QG_ERR_INVALID_ARG;
    if (seeded_for_other_slab(c, nranks, rank)) return QG_ERR_INVALID_ARG;
    QG_CHECK(settle_pcg(c));  // (the solver is rebuilt)
    if (c->zeta) QG_CHECK(settle_zcopy(c));
    QG_HIP(hipSetDevice(c->device));
    if (c->comm) {
        comm_destroy(c->comm);
        c->comm = nullptr;
    }
    QG_CHECK(comm_init(&c->comm, nranks, rank, id));
    QG_CHECK(comm_attach(c, nranks, rank));
    // environment opt-ins of the peer transports (every rank sees the same environment).  A
    // node whose ranks cannot share the IPC regions (QG_ERR_UNSUPPORTED, the same verdict on
    // every rank) keeps the RCCL transport: the communicator attached above works, so the
    // init succeeds; only the explicit qg_comm_set_*_transport calls report the refusal.
    if (const char *e = std::getenv("QG_HALO_PEER"))
        if (std::atoi(e) != 0) {
            const int st = qg_comm_set_halo_transport(c, std::atoi(e) == 2 ? QG_HALO_PUT : QG_HALO_PEER);
            if (st == QG_ERR_UNSUPPORTED)
                std::fprintf(stderr, "qg_mi355: rank %d: QG_HALO_PEER: peer regions unavailable, the halo stays on RCCL\n", rank);
            else
                QG_CHECK(st);
        }
    if (const char *e = std::getenv("QG_GATHER_PEER"))
        if (std::atoi(e) != 0 && c->spec) {
            const int st = qg_comm_set_gather_transport(c, QG_GATHER_PEER);
            if (st == QG_ERR_UNSUPPORTED)
                std::fprintf(stderr, "qg_mi355: rank %d: QG_GATHER_PEER: peer regions unavailable, the gather stays on RCCL\n", rank);
            else
                QG_CHECK(st);
        }
    return QG_OK;
}

int qg_comm_set_gather_transport(qg_ctx *c, int transport) {
    if (!c || (transport != QG_GATHER_RCCL && transport != QG_GATHER_PEER)) return QG_ERR_INVALID_ARG;
    if (!c->distributed || !c->comm) return QG_ERR_RCCL;
    if (!c->spec) return QG_ERR_UNSUPPORTED;
    QG_HIP(hipSetDevice(c->device));
    return comm_set_peer_gather(c->comm, transport == QG_GATHER_PEER, c->spec->args().rec_stride);
}

int qg_comm_set_halo_transport(qg_ctx *c, int transport) {
    if (!c || (transport != QG_HALO_RCCL && transport != QG_HALO_PEER && transport != QG_HALO_PUT))
        return QG_ERR_INVALID_ARG;
    if (!c->distributed || !c->comm) return QG_ERR_RCCL;
    QG_HIP(hipSetDevice(c->device));
    return comm_set_peer(c->comm, transport == QG_HALO_RCCL ? 0 : transport == QG_HALO_PEER ? 1 : 2, c->row_words());
}

int qg_comm_init_host(qg_ctx *c, int nranks, int rank, qg_allgather_fn allgather, qg_sendrecv_fn sendrecv,
                      void *user) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks || !allgather || !sendrecv) return QG_ERR_INVALID_ARG;
    if (seeded_for_other_slab(c, nranks, rank)) return QG_ERR_INVALID_ARG;
    QG_CHECK(settle_pcg(c));  // (the solver is rebuilt)
    if (c->zeta) QG_CHECK(settle_zcopy(c));
    QG_HIP(hipSetDevice(c->device));
    if (c->comm) {
        comm_destroy(c->comm);
        c->comm = nullptr;
    }
    QG_CHECK(comm_init_host(&c->comm, nranks, rank, allgather, sendrecv, user));
    return comm_attach(c, nranks, rank);
}

// Time the step's two collectives in isolation on the context's stream (HIP events around
// `reps` back-to-back calls each): the tendency's halo exchange (pack + grouped send/recv of
// the depth-2 rows of psi and zeta, both layers, exactly as a step posts it) and the solve's
// record all-gather.  out[0] halo ms per exchange, out[1] bytes this rank sends per exchange,
// out[2] all-gather ms, out[3] bytes this rank receives per all-gather.  Every rank must call
// it (collectives).  Harmless to the state: the halo rows it receives are the ones the next
// step receives again, and the gathered records are recomputed by the next solve.
int qg_comm_probe(qg_ctx *c, int reps, double out[4]) {
    if (!c || !out || reps < 1) return QG_ERR_INVALID_ARG;
    if (!c->distributed || !c->comm) return QG_ERR_RCCL;
    if (!c->spec) return QG_ERR_UNSUPPORTED;
    QG_HIP(hipSetDevice(c->device));
    const qg_params &p = c->p;
    const int zh = c->heads[0], ph = c->heads[1];
    double *f2[4] = {c->field(c->psi, 0, ph), c->field(c->psi, 1, ph), c->field(c->zeta, 0, zh),
                     c->field(c->zeta, 1, zh)};
    const double *hr[16];
    const SpecArgs &sa = c->spec->args();
    hipEvent_t ev[3];
    for (auto &e : ev) QG_HIP(hipEventCreate(&e));
    int st = QG_OK;
    auto run = [&]() -> int {
        QG_CHECK(comm_halo_rows(c->comm, f2, 4, c->row_words(), p.P, c->stream, hr));  // (warm)
        QG_CHECK(comm_gather_records(c->comm, sa.rec, c->spec->gather_buf(), sa.rec_stride, c->stream));
        QG_HIP(hipEventRecord(ev[0], c->stream));
        for (int k = 0; k < reps; ++k) QG_CHECK(comm_halo_rows(c->comm, f2, 4, c->row_words(), p.P, c->stream, hr));
        QG_HIP(hipEventRecord(ev[1], c->stream));
        for (int k = 0; k < reps; ++k)
            QG_CHECK(comm_gather_records(c->comm, sa.rec, c->spec->gather_buf(), sa.rec_stride, c->stream));
        QG_HIP(hipEventRecord(ev[2], c->stream));
        QG_CHECK(comm_wait(c->comm, c->stream, ev[2], "qg_comm_probe"));
        float a = 0, b = 0;
        QG_HIP(hipEventElapsedTime(&a, ev[0], ev[1]));
        QG_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
        out[0] = a / reps;
        out[1] = 2.0 * 8 * (double)c->row_words() * 8;  // two messages of 8 rows (2 x 4 fields)
        out[2] = b / reps;
        out[3] = (double)sa.rec_stride * 8 * (c->nranks - 1);
        return QG_OK;
    };
    st = run();
    for (auto &e : ev) (void)hipEventDestroy(e);
    return st;
}

// ---- solver handles ---------------------------------------------------------------------
int qg_solver_create(int64_t M, int64_t P, double dx, const double alpha[2], const int pinned[2],
                     const double proj_in[4], const double proj_out[4], int kind, int precond, int device,
                     void *stream, qg_solver **out) {
    if (!out || !alpha || !pinned || !proj_in || !proj_out) return QG_ERR_INVALID_ARG;
    *out = nullptr;
    if (kind != QG_SOLVER_SPECTRAL && kind != QG_SOLVER_PCG) return QG_ERR_INVALID_ARG;
    if (pinned[1]) return QG_ERR_UNSUPPORTED;           // only system 0 may be the pinned Poisson
    if (pinned[0] && alpha[0] != 0.0) return QG_ERR_INVALID_ARG;
    qg_solver *s = new (std::nothrow) qg_solver();
    if (!s) return QG_ERR_ALLOC;
    s->device = device;
    s->stream = static_cast<hipStream_t>(stream);
    if (hipSetDevice(device) != hipSuccess) {
        delete s;
        return QG_ERR_HIP;
    }
    int st;
    if (kind == QG_SOLVER_PCG) {
        // CG on -A with b = -(proj_in f): the same x as A x = proj_in f
        s->pcg = std::make_unique<PcgSolver>();
        st = s->pcg->init(M, P, P, 0, 1, dx, alpha, pinned[0], proj_in, proj_out, precond, 1e-13, 4000, 0);
        s->pcg->set_deferred(false);  // a factor handle's solve returns its own verdict
    } else {
        st = s->spec.init(M, P, P, 0, 1, dx, alpha, pinned[0], proj_in, proj_out, 0);
    }
    if (st != QG_OK) {
        delete s;
        return st;
    }
    *out = s;
    return QG_OK;
}

int qg_solver_solve(qg_solver *s, const double *f_1, const double *f_2, double *out_1, double *out_2) {
    if (!s || !f_1 || !out_1) return QG_ERR_INVALID_ARG;
    QG_HIP(hipSetDevice(s->device));
    if (s->pcg) return s->pcg->solve(f_1, f_2, out_1, out_2, 1, s->stream);
    return s->spec.solve(f_1, f_2, out_1, out_2, 1, s->stream);
}

int qg_solver_destroy(qg_solver *s) {
    if (s) {
        (void)hipSetDevice(s->device);
        delete s;
    }
    return QG_OK;
}

// ---- stateless operators ----------------------------------------------------------------
int qg_laplace_5p(const double *u, double *out, int64_t M, int64_t P, double dx, void *stream) {
    if (!u || !out || M < 1 || P < 1 || !(dx > 0)) return QG_ERR_INVALID_ARG;
    return launch_laplace(u, out, M, P, dx, static_cast<hipStream_t>(stream));
}

int qg_cd(const double *u, double *out, int64_t M, int64_t P, double dx, void *stream) {
    if (!u || !out || M < 1 || P < 1 || !(dx > 0)) return QG_ERR_INVALID_ARG;
    return launch_cd(u, out, M, P, dx, static_cast<hipStream_t>(stream));
}

int qg_arakawa_J(const double *zeta, const double *psi, double *out, int64_t M, int64_t P, double dx,
                 void *stream) {
    if (!zeta || !psi || !out || M < 1 || P < 1 || !(dx > 0)) return QG_ERR_INVALID_ARG;
    return launch_arakawa(zeta, psi, out, M, P, dx, static_cast<hipStream_t>(stream));
}

int qg_fill_ghosts(double *b, int64_t M, int64_t P, void *stream) {
    if (!b || M < 1 || P < 1) return QG_ERR_INVALID_ARG;
    return launch_fill_ghosts(b, M, P, static_cast<hipStream_t>(stream));
}

}  // extern "C"
