// RCCL plumbing for the y-slab decomposition (one rank per GPU, ring of ranks in y).
//   - halo rows for the tendency stencil: ncclSend/ncclRecv of whole contiguous rows to the
//     two ring neighbours inside one group (each row already carries its x-ghosts, so the
//     diagonal corners the Arakawa Jacobian reads arrive with it);
//   - ghost-row refresh of the fields written by the previous step (drop-in ghost ring),
//     grouped with the next step's halo exchange;
//   - the spectral solver's per-step all-gather of the rank records (a few hundred KB);
//   - optionally (comm_set_peer / comm_set_peer_gather) the halo rows by copy engine and the
//     records by one kernel, both into IPC-mapped peer buffers.
#include <rccl/rccl.h>
#include <sched.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "qg_common.hpp"

namespace qg {

struct Comm {
    ncclComm_t nccl = nullptr;  // RCCL transport, or
    qg_allgather_fn ag = nullptr;  // host-provided transport (tests, MPI, ...)
    qg_sendrecv_fn sr = nullptr;
    void *user = nullptr;
    int nranks = 1, rank = 0;
    double *stage = nullptr;  // exchange staging: [to_next | to_prev | from_prev | from_next]
    size_t stage_n = 0;
    // watchdog: the unpack kernel of every exchange stores its sequence number into this
    // host-mapped word, so a host wait can tell "slow" from "stuck" (no exchange completing)
    int64_t *progress_h = nullptr, *progress_d = nullptr;
    int64_t seq = 0;
    double timeout_s = 120.0;
    bool failed = false;
    // Peer transports (RCCL communicator only).  Each uses an IpcRegion: uncached device memory
    // of this rank (so writes from other agents are never hidden behind a stale L2 line),
    // opened by the ranks that write into it through IPC.
    // - halo (comm_set_peer): the halo rows go by copy engine straight from the state into
    //   the ring neighbours' regions; a one-lane kernel then raises the neighbour's arrival
    //   flag and a one-lane kernel on the receiving side polls its flags before the halo is
    //   read.  No collective kernel, so no compute-unit slots are needed beside the interior
    //   tendency.  Region: [flags: 2 x 64 B | parity 0: from_prev, from_next | parity 1: ...],
    //   each direction PEER_ROWS rows of ld words.
    // - record gather (comm_set_peer_gather): one kernel per solve, (blocks x ranks)
    //   workgroups; workgroup (b, r) stores part b of this rank's record into rank r's region,
    //   raises r's flag (rank, b), waits for r's flag in this rank's region and copies r's
    //   part b out.  One launch, every peer written in parallel over its own link (no ring).
    struct IpcRegion {
        double *local = nullptr;
        std::vector<double *> remote;  // per rank: its region as mapped here (self: local)
        std::vector<char> opened;      // remote[r] is an IPC mapping to close
    };
    IpcRegion halo_rx, gat_rx;
    bool peer = false;
    bool put = false;  // halo by the put kernel (QG_HALO_PUT) instead of the copy engine
    int64_t peer_ld = 0;
    int64_t pseq = 0;  // peer halo exchanges posted (the arrival flags' values)
    bool pgather = false;
    int64_t pg_count = 0;
    int64_t gseq = 0;  // peer record gathers posted
    int64_t *perr_h = nullptr, *perr_d = nullptr;  // a wait timed out: the exchange number
    // the collective set-up steps' own stream and scratch (allocated at comm_init, so that no
    // rank can fail before joining region_create's / comm_barrier's all-gathers)
    hipStream_t coll_s = nullptr;
    double *coll = nullptr;  // coll_words(nranks) doubles
    uint64_t clock_khz = 100000;
};

constexpr int PEER_ROWS = 8;       // rows per direction (4 fields x 2)
constexpr int PUT_BLOCKS = 8;      // halo put kernel: workgroups per direction
// words before the rows: flags (dir, part) at (dir * PUT_BLOCKS + part) * 8 (dir 0 = from_prev,
// 1 = from_next; the copy-engine mode uses part 0)
constexpr int64_t PEER_HDR = 2 * PUT_BLOCKS * 8;
constexpr int PG_BLOCKS = 4;       // record gather: workgroups per peer
constexpr int PG_MAX_RANKS = 64;

#define QG_NCCL(call)                                                                          \
    do {                                                                                       \
        ncclResult_t r_ = (call);                                                              \
        if (r_ != ncclSuccess) {                                                               \
            std::fprintf(stderr, "qg_mi355: %s failed: %s\n", #call, ncclGetErrorString(r_));  \
            return QG_ERR_RCCL;                                                                \
        }                                                                                      \
    } while (0)

int comm_unique_id(char out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    QG_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, 128);
    return QG_OK;
}

static int comm_setup_watchdog(Comm *c) {
    if (const char *e = std::getenv("QG_COMM_TIMEOUT")) {
        const double t = std::atof(e);
        if (t > 0) c->timeout_s = t;
    }
    QG_HIP(hipHostMalloc((void **)&c->progress_h, sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent));
    *c->progress_h = 0;
    QG_HIP(hipHostGetDevicePointer((void **)&c->progress_d, c->progress_h, 0));
    return QG_OK;
}

static int post(Comm *c, double *const xbuf[4], int64_t cnt, hipStream_t s);

// region_create: [own handle + status: 16 | all: 16 G | own open status: 8 | all: 8 G];
// comm_barrier: [1 | G] after those
static size_t coll_words(int G) { return (size_t)24 * (G + 1) + 1 + (size_t)G; }

// RCCL connects peers lazily, inside the host call of the first operation that needs them
// (ncclGroupEnd / ncclAllGather), in a handshake with the peer.  A peer that died before its
// first exchange would then hold this rank's host thread inside RCCL, where no watchdog runs
// (measured over the loopback network transport: rank 0 blocked in its first exchange for as
// long as its peer stayed silent).  So comm_init, which every rank calls together, runs one
// ring exchange and one all-gather at a small and a large message size: every connection the
// stepping uses is made while all ranks are known to be alive, and afterwards a silent peer
// only leaves RCCL kernels waiting on the device, which the bounded waits abort.
// `local` (this rank's set-up status so far) rides in a last all-gather, so every rank returns
// the same verdict: a rank whose own allocations failed still takes part, and its peers learn
// of the failure here instead of blocking later in a collective it never joins.
static int comm_warmup(Comm *c, int local) {
    constexpr int64_t W = 131072;  // doubles: 1 MB, above every protocol's size threshold
    hipStream_t s = nullptr;
    double *buf = nullptr;
    QG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int st = QG_OK;
    if (hipMalloc((void **)&buf, sizeof(double) * (size_t)(4 + c->nranks) * W) != hipSuccess) st = QG_ERR_HIP;
    if (st == QG_OK) (void)hipMemsetAsync(buf, 0, sizeof(double) * (size_t)(4 + c->nranks) * W, s);
    for (int64_t n : {(int64_t)512, W}) {
        if (st != QG_OK) break;
        double *xbuf[4] = {buf, buf + W, buf + 2 * W, buf + 3 * W};
        st = post(c, xbuf, n, s);
        if (st == QG_OK && ncclAllGather(buf, buf + 4 * W, (size_t)n, ncclDouble, c->nccl, s) != ncclSuccess)
            st = QG_ERR_RCCL;
    }
    const double mine = (double)local;  // (lives until the copy has run: comm_wait below)
    if (st == QG_OK) {  // every rank's local status
        if (hipMemcpyAsync(buf, &mine, sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
            ncclAllGather(buf, buf + 4 * W, 1, ncclDouble, c->nccl, s) != ncclSuccess)
            st = QG_ERR_RCCL;
    }
    if (st == QG_OK) st = comm_wait(c, s, nullptr, "qg_comm_init (connection warm-up)");
    if (st == QG_OK) {
        std::vector<double> all((size_t)c->nranks);
        if (hipMemcpy(all.data(), buf + 4 * W, sizeof(double) * (size_t)c->nranks, hipMemcpyDeviceToHost) != hipSuccess)
            st = QG_ERR_HIP;
        for (int r = 0; r < c->nranks && st == QG_OK; ++r)
            if (all[(size_t)r] != 0.0) st = (int)all[(size_t)r];
    }
    if (buf) (void)hipFree(buf);
    (void)hipStreamDestroy(s);
    return st;
}

int comm_init(void **comm, int nranks, int rank, const char id[128]) {
    Comm *c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    if (comm_setup_watchdog(c) != QG_OK) {
        delete c;
        return QG_ERR_HIP;
    }
    {  // nranks == 1 is allowed: the halo ring then sends to itself (exercises the path)
        ncclUniqueId uid;
        std::memcpy(&uid, id, 128);
        const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
        if (r != ncclSuccess) {
            std::fprintf(stderr, "qg_mi355: ncclCommInitRank failed: %s\n", ncclGetErrorString(r));
            delete c;
            return QG_ERR_RCCL;
        }
    }
    // the collective stream and scratch first: their status joins the warm-up's verdict
    int local = QG_OK;
    if (hipStreamCreateWithFlags(&c->coll_s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&c->coll, sizeof(double) * coll_words(nranks)) != hipSuccess) {
        std::fprintf(stderr, "qg_mi355 rank %d/%d: allocating the collective stream / scratch failed\n", rank, nranks);
        local = QG_ERR_ALLOC;
    }
    const int w = comm_warmup(c, local);
    if (w != QG_OK) {
        if (local == QG_OK)
            std::fprintf(stderr, "qg_mi355 rank %d/%d: RCCL connection warm-up failed (%d)\n", rank, nranks, w);
        if (c->nccl) ncclCommAbort(c->nccl);
        c->nccl = nullptr;
        if (c->progress_h) (void)hipHostFree(c->progress_h);
        if (c->coll) (void)hipFree(c->coll);
        if (c->coll_s) (void)hipStreamDestroy(c->coll_s);
        delete c;
        return w;
    }
    *comm = c;
    return QG_OK;
}

int comm_init_host(void **comm, int nranks, int rank, qg_allgather_fn ag, qg_sendrecv_fn sr, void *user) {
    if (!ag || !sr) return QG_ERR_INVALID_ARG;
    Comm *c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    c->ag = ag;
    c->sr = sr;
    c->user = user;
    if (comm_setup_watchdog(c) != QG_OK) {
        delete c;
        return QG_ERR_HIP;
    }
    *comm = c;
    return QG_OK;
}

static void region_release(Comm::IpcRegion &g) {
    for (size_t r = 0; r < g.remote.size(); ++r)
        if (g.opened[r] && g.remote[r]) (void)hipIpcCloseMemHandle(g.remote[r]);
    g.remote.clear();
    g.opened.clear();
    if (g.local) (void)hipFree(g.local);
    g.local = nullptr;
}

static void peer_release_all(Comm *c) {
    if (c->halo_rx.local || c->gat_rx.local) (void)hipDeviceSynchronize();  // (queued writes)
    region_release(c->halo_rx);
    region_release(c->gat_rx);
    c->peer = c->pgather = false;
    c->peer_ld = c->pg_count = 0;
    if (c->perr_h) (void)hipHostFree(c->perr_h);
    c->perr_h = c->perr_d = nullptr;
}

int comm_destroy(void *comm) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c) return QG_OK;
    peer_release_all(c);
    if (c->nccl) ncclCommDestroy(c->nccl);
    if (c->stage) (void)hipFree(c->stage);
    if (c->progress_h) (void)hipHostFree(c->progress_h);
    if (c->coll) (void)hipFree(c->coll);
    if (c->coll_s) (void)hipStreamDestroy(c->coll_s);
    delete c;
    return QG_OK;
}

int comm_allgather(void *user, const double *send, double *recv, int64_t count, hipStream_t s) {
    Comm *c = static_cast<Comm *>(user);
    if (!c || c->failed) return QG_ERR_RCCL;
    if (c->ag) {
        if (c->ag(c->user, send, recv, count, s) == 0) return QG_OK;
        std::fprintf(stderr, "qg_mi355 rank %d/%d: host transport all-gather failed\n", c->rank, c->nranks);
        c->failed = true;
        return QG_ERR_RCCL;
    }
    if (!c->nccl) return QG_ERR_RCCL;
    QG_NCCL(ncclAllGather(send, recv, (size_t)count, ncclDouble, c->nccl, s));
    return QG_OK;
}

// Row copies (pack / unpack of the exchange): pair k copies one row of ld doubles.
constexpr int XMAX = 64;
struct RowCopies {
    const double *src[XMAX];
    double *dst[XMAX];
    int n;
    int64_t ld;
};

// progress != nullptr (the unpack after a receive): one lane publishes seq to the host
__global__ void copy_rows_kernel(RowCopies rc, int64_t *progress, int64_t seq) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    if (k < rc.n && i < rc.ld) rc.dst[k][i] = rc.src[k][i];
    if (progress && i == 0 && k == 0)
        __hip_atomic_store(progress, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static int copy_rows(const RowCopies &rc, hipStream_t s, int64_t *progress = nullptr, int64_t seq = 0) {
    if (rc.n == 0) return QG_OK;
    copy_rows_kernel<<<dim3((unsigned)((rc.ld + 255) / 256), (unsigned)rc.n), 256, 0, s>>>(rc, progress, seq);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// The exchange schedule (qg_comm_exchange_plan): [send -> next, send -> prev],
// [recv <- prev, recv <- next].  With two ranks (prev == next) the two messages per peer
// match in this posting order: the first message from a peer is its to_next (its top rows,
// our halo below), the second its to_prev.
static void exchange_plan(int rank, int G, int speer[2], int sbuf[2], int rpeer[2], int rbuf[2]) {
    const int next = (rank + 1) % G, prev = (rank - 1 + G) % G;
    speer[0] = next; sbuf[0] = QG_XBUF_TO_NEXT;
    speer[1] = prev; sbuf[1] = QG_XBUF_TO_PREV;
    rpeer[0] = prev; rbuf[0] = QG_XBUF_FROM_PREV;
    rpeer[1] = next; rbuf[1] = QG_XBUF_FROM_NEXT;
}

// Bounded host wait (see qg_comm_set_timeout in the header): polls the event (or the whole
// stream) with the RCCL async error; fails after `timeout_s` without a completed exchange.
int comm_wait(void *comm, hipStream_t s, hipEvent_t ev, const char *what) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c) {
        QG_HIP(ev ? hipEventSynchronize(ev) : hipStreamSynchronize(s));
        return QG_OK;
    }
    if (c->failed) return QG_ERR_RCCL;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto t_prog = t0;
    int64_t seen = c->progress_h ? __atomic_load_n(c->progress_h, __ATOMIC_RELAXED) : 0;
    for (long spin = 0;; ++spin) {
        if (c->perr_h && __atomic_load_n(c->perr_h, __ATOMIC_RELAXED) != 0) {
            std::fprintf(stderr,
                         "qg_mi355 rank %d/%d: %s: peer transfer #%lld did not arrive within %.1f s -- a peer "
                         "died or posted a different schedule; aborting the communicator\n",
                         c->rank, c->nranks, what, (long long)__atomic_load_n(c->perr_h, __ATOMIC_RELAXED),
                         c->timeout_s);
            if (c->nccl) ncclCommAbort(c->nccl);
            c->nccl = nullptr;
            c->failed = true;
            return QG_ERR_RCCL;
        }
        const hipError_t q = ev ? hipEventQuery(ev) : hipStreamQuery(s);
        if (q == hipSuccess) return QG_OK;
        if (q != hipErrorNotReady) {
            std::fprintf(stderr, "qg_mi355 rank %d/%d: %s: %s\n", c->rank, c->nranks, what, hipGetErrorString(q));
            return QG_ERR_HIP;
        }
        const auto now = clk::now();
        ncclResult_t ar = ncclSuccess;
        if (c->nccl && ncclCommGetAsyncError(c->nccl, &ar) == ncclSuccess && ar != ncclSuccess &&
            ar != ncclInProgress) {
            std::fprintf(stderr, "qg_mi355 rank %d/%d: %s: RCCL async error: %s; aborting the communicator\n",
                         c->rank, c->nranks, what, ncclGetErrorString(ar));
            ncclCommAbort(c->nccl);
            c->nccl = nullptr;
            c->failed = true;
            return QG_ERR_RCCL;
        }
        const int64_t p = c->progress_h ? __atomic_load_n(c->progress_h, __ATOMIC_RELAXED) : 0;
        if (p != seen) {
            seen = p;
            t_prog = now;
        }
        const double stuck = std::chrono::duration<double>(now - t_prog).count();
        if (stuck > c->timeout_s) {
            std::fprintf(stderr,
                         "qg_mi355 rank %d/%d: %s: no halo exchange completed for %.1f s (last completed: #%lld of "
                         "%lld posted) -- a peer died or posted a different schedule; aborting the communicator\n",
                         c->rank, c->nranks, what, stuck, (long long)p, (long long)c->seq);
            if (c->nccl) ncclCommAbort(c->nccl);
            c->nccl = nullptr;
            c->failed = true;
            return QG_ERR_RCCL;
        }
        if (spin < 2000) sched_yield();  // the common case: done within a few ms
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

int comm_set_timeout(void *comm, double seconds) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || !(seconds > 0)) return QG_ERR_INVALID_ARG;
    c->timeout_s = seconds;
    return QG_OK;
}

// The staging buffer [to_next | to_prev | from_prev | from_next], `rows` rows of ld words
// each.  Allocated once for the largest exchange (XMAX / 2 rows per direction), so a later,
// larger exchange never frees a buffer an earlier one's pending kernels still read.
static int ensure_stage(Comm *c, int rows, int64_t ld, double *xbuf[4]) {
    const size_t need = (size_t)4 * (XMAX / 2) * ld;
    if (rows > XMAX / 2) return QG_ERR_INVALID_ARG;
    if (need > c->stage_n) {
        if (c->stage) {
            QG_HIP(hipDeviceSynchronize());  // (a wider row length: a new context shape)
            (void)hipFree(c->stage);
        }
        c->stage = nullptr;
        c->stage_n = 0;
        QG_HIP(hipMalloc((void **)&c->stage, sizeof(double) * need));
        c->stage_n = need;
    }
    for (int b = 0; b < 4; ++b) xbuf[b] = c->stage + (size_t)b * rows * ld;
    return QG_OK;
}

// the grouped send / receive of one exchange (the plan of exchange_plan), cnt words each
static int post(Comm *c, double *const xbuf[4], int64_t cnt, hipStream_t s) {
    int speer[2], sbuf[2], rpeer[2], rbuf[2];
    exchange_plan(c->rank, c->nranks, speer, sbuf, rpeer, rbuf);
    if (c->sr) {
        const double *sp[2] = {xbuf[sbuf[0]], xbuf[sbuf[1]]};
        double *rp[2] = {xbuf[rbuf[0]], xbuf[rbuf[1]]};
        const int64_t sc[2] = {cnt, cnt}, rcnt[2] = {cnt, cnt};
        if (c->sr(c->user, 2, sp, sc, speer, 2, rp, rcnt, rpeer, s) != 0) {
            std::fprintf(stderr, "qg_mi355 rank %d/%d: host transport sendrecv failed\n", c->rank, c->nranks);
            c->failed = true;
            return QG_ERR_RCCL;
        }
        return QG_OK;
    }
    QG_NCCL(ncclGroupStart());
    for (int k = 0; k < 2; ++k) QG_NCCL(ncclSend(xbuf[sbuf[k]], (size_t)cnt, ncclDouble, speer[k], c->nccl, s));
    for (int k = 0; k < 2; ++k) QG_NCCL(ncclRecv(xbuf[rbuf[k]], (size_t)cnt, ncclDouble, rpeer[k], c->nccl, s));
    QG_NCCL(ncclGroupEnd());
    return QG_OK;
}

// One exchange with the two ring neighbours, as ONE message per direction: the rows are
// packed into a staging buffer per neighbour, sent / received in one group, and unpacked.
//   f2[0..n2): depth-2 halo -> halo_buf[f][4][M+2] = rows -2,-1 (from rank-1), P,P+1 (from
//              rank+1); with ghost_f2 the ghost rows of f2 (rows -1 and P) are filled too
//   f1[0..n1): refresh of the ghost rows (memory rows 0 and P+1) in place
// Messages: [send -> next, send -> prev], [recv <- prev, recv <- next]; with two ranks
// (prev == next) the two messages per peer match in this posting order.
// ld = row length in 8-byte words ((M+2) for F64 fields, (M+2)/2 for F32 fields: the rows
// move as raw words, their element type does not matter here)
int comm_exchange(void *comm, double *const *f2, int n2, double *halo_buf, double *const *f1, int n1, int64_t ld,
                  int64_t P, hipStream_t s, bool ghost_f2) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || c->failed || (!c->nccl && !c->sr)) return QG_ERR_RCCL;
    const int rows = 2 * n2 + n1;  // rows per direction
    if (n2 < 0 || n1 < 0 || 4 * n2 + (ghost_f2 ? 2 * n2 : 0) + 2 * n1 > XMAX) return QG_ERR_INVALID_ARG;
    if (rows == 0) return QG_OK;
    double *xbuf[4];  // indexed by QG_XBUF_*
    QG_CHECK(ensure_stage(c, rows, ld, xbuf));
    double *to_next = xbuf[QG_XBUF_TO_NEXT], *to_prev = xbuf[QG_XBUF_TO_PREV];
    double *from_prev = xbuf[QG_XBUF_FROM_PREV], *from_next = xbuf[QG_XBUF_FROM_NEXT];
    RowCopies pk{}, up{};
    pk.ld = up.ld = ld;
    int r = 0;
    for (int f = 0; f < n2; ++f, r += 2) {
        double *b = f2[f];
        double *lo = halo_buf + (size_t)f * 4 * ld, *hi = lo + 2 * ld;
        for (int q = 0; q < 2; ++q) {
            pk.src[pk.n] = b + fidx(0, P - 1 + q, ld); pk.dst[pk.n++] = to_next + (r + q) * ld;  // rows P-2, P-1
            pk.src[pk.n] = b + fidx(0, 1 + q, ld);     pk.dst[pk.n++] = to_prev + (r + q) * ld;  // rows 0, 1
            up.src[up.n] = from_prev + (r + q) * ld;   up.dst[up.n++] = lo + q * ld;            // rows -2, -1
            up.src[up.n] = from_next + (r + q) * ld;   up.dst[up.n++] = hi + q * ld;            // rows P, P+1
        }
        if (ghost_f2) {
            up.src[up.n] = from_prev + (r + 1) * ld; up.dst[up.n++] = b + fidx(0, 0, ld);
            up.src[up.n] = from_next + r * ld;       up.dst[up.n++] = b + fidx(0, P + 1, ld);
        }
    }
    for (int f = 0; f < n1; ++f, ++r) {
        double *b = f1[f];
        pk.src[pk.n] = b + fidx(0, P, ld);     pk.dst[pk.n++] = to_next + r * ld;
        pk.src[pk.n] = b + fidx(0, 1, ld);     pk.dst[pk.n++] = to_prev + r * ld;
        up.src[up.n] = from_prev + r * ld;     up.dst[up.n++] = b + fidx(0, 0, ld);
        up.src[up.n] = from_next + r * ld;     up.dst[up.n++] = b + fidx(0, P + 1, ld);
    }
    QG_CHECK(copy_rows(pk, s));
    QG_CHECK(post(c, xbuf, (int64_t)rows * ld, s));
    return copy_rows(up, s, c->progress_d, ++c->seq);
}

// The halo rows of the tendency only, left where they are received: no unpack kernel (the
// tendency reads them from the staging buffer) and no ghost rows (refreshed by the next
// ghost flush).  rows_out[4 f + h] = row h of field f (h: -2, -1, P, P+1).  The pack kernel
// publishes the watchdog's progress: every earlier exchange has completed when it runs.
static int peer_halo_rows(Comm *c, double *const *f2, int n2, int64_t ld, int64_t P, hipStream_t s,
                          const double **rows_out);

int comm_halo_rows(void *comm, double *const *f2, int n2, int64_t ld, int64_t P, hipStream_t s,
                   const double **rows_out) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || c->failed || (!c->nccl && !c->sr)) return QG_ERR_RCCL;
    if (c->peer) return peer_halo_rows(c, f2, n2, ld, P, s, rows_out);
    const int rows = 2 * n2;
    if (n2 < 1 || 2 * rows > XMAX) return QG_ERR_INVALID_ARG;
    double *xbuf[4];
    QG_CHECK(ensure_stage(c, rows, ld, xbuf));
    double *to_next = xbuf[QG_XBUF_TO_NEXT], *to_prev = xbuf[QG_XBUF_TO_PREV];
    const double *from_prev = xbuf[QG_XBUF_FROM_PREV], *from_next = xbuf[QG_XBUF_FROM_NEXT];
    RowCopies pk{};
    pk.ld = ld;
    for (int f = 0; f < n2; ++f) {
        double *b = f2[f];
        for (int q = 0; q < 2; ++q) {
            const int r = 2 * f + q;
            pk.src[pk.n] = b + fidx(0, P - 1 + q, ld); pk.dst[pk.n++] = to_next + r * ld;  // rows P-2, P-1
            pk.src[pk.n] = b + fidx(0, 1 + q, ld);     pk.dst[pk.n++] = to_prev + r * ld;  // rows 0, 1
            rows_out[4 * f + q] = from_prev + r * ld;                                      // rows -2, -1
            rows_out[4 * f + 2 + q] = from_next + r * ld;                                  // rows P, P+1
        }
    }
    QG_CHECK(copy_rows(pk, s, c->progress_d, c->seq));
    ++c->seq;
    return post(c, xbuf, (int64_t)rows * ld, s);
}

// ---- peer-copy halo transport ----------------------------------------------------------
// Raise the arrival flags of exchange `seq` in the neighbours' receive regions.  Stream order
// puts this launch after the copy-engine copies into those regions have completed.
__global__ void peer_signal_kernel(uint64_t *flag_next, uint64_t *flag_prev, uint64_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag_next, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 1) __hip_atomic_store(flag_prev, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait (one lane) until both neighbours have raised this rank's flags to >= seq; bounded by
// `limit` wall-clock ticks, after which the exchange number goes to *err (read by comm_wait,
// which then fails the transport) and the kernel ends, so a dead peer never leaves a wave
// spinning.  On arrival the watchdog's progress word advances.
__global__ void peer_wait_kernel(const uint64_t *flags, uint64_t seq, uint64_t limit, int64_t *progress,
                                 int64_t prog, int64_t *err) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    for (;;) {
        const uint64_t a = __hip_atomic_load(flags, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t b = __hip_atomic_load(flags + PUT_BLOCKS * 8, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a >= seq && b >= seq) break;
        // (an earlier wait already timed out: the transport has failed, do not wait again)
        if (wall_clock64() - t0 > limit || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
            int64_t zero = 0;
            __hip_atomic_compare_exchange_strong(err, &zero, (int64_t)seq, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
    if (progress) __hip_atomic_store(progress, prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double *peer_region(double *base, int64_t ld, int par, int dir) {
    return base + PEER_HDR + (size_t)(2 * par + dir) * PEER_ROWS * ld;
}

// all ranks have reached this point (a one-word all-gather, waited on with the watchdog).  The
// stream and buffer exist since comm_init: no rank returns before the collective.
static int comm_barrier(Comm *c, const char *what) {
    double *b = c->coll + 24 * (size_t)(c->nranks + 1);
    if (hipMemsetAsync(b, 0, sizeof(double), c->coll_s) != hipSuccess) return QG_ERR_HIP;  // (local: before any rank's gather)
    if (ncclAllGather(b, b + 1, 1, ncclDouble, c->nccl, c->coll_s) != ncclSuccess) return QG_ERR_RCCL;
    return comm_wait(c, c->coll_s, nullptr, what);
}

// Collective: allocate this rank's region (`bytes`, uncached, zeroed), all-gather the IPC
// handles over RCCL and open the regions of the ranks flagged in `need`.  Every rank ends
// with the same verdict: a rank whose set-up failed makes all of them return
// QG_ERR_UNSUPPORTED (regions released).  Every rank joins both all-gathers whatever failed
// locally (the stream and the scratch were made at comm_init): local failures travel in the
// gathered status words, so no rank waits in a collective another rank skipped.
//   gather 1: each rank's handle and its set-up status; a rank opens peers' handles only when
//             every status is OK (never a handle a failed rank did not fill in);
//   gather 2: each rank's open status.
static int region_create(Comm *c, Comm::IpcRegion &g, size_t bytes, const std::vector<char> &need, const char *what) {
    const int G = c->nranks;
    hipStream_t s = c->coll_s;
    double *hb = c->coll;
    double *own1 = hb, *all1 = hb + 16, *own2 = hb + 16 * (size_t)(G + 1), *all2 = own2 + 8;
    int local = QG_OK;
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
    g.remote.assign((size_t)G, nullptr);
    g.opened.assign((size_t)G, 0);
    if (hipExtMallocWithFlags((void **)&g.local, bytes, hipDeviceMallocUncached) != hipSuccess) g.local = nullptr;
    if (!g.local || hipMemset(g.local, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        local = QG_ERR_ALLOC;
    if (local == QG_OK && !c->perr_h) {
        if (hipHostMalloc((void **)&c->perr_h, sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&c->perr_d, c->perr_h, 0) != hipSuccess)
            local = QG_ERR_ALLOC;
        else
            *c->perr_h = 0;
    }
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess &&
        khz > 0)
        c->clock_khz = (uint64_t)khz;
    double w1[16] = {};
    if (local == QG_OK && hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t *>(w1), g.local) != hipSuccess)
        local = QG_ERR_UNSUPPORTED;
    w1[8] = (double)local;
    // (a failed upload leaves the status word unknown to the peers: the gather still runs, and
    // this rank reports the failure in gather 2)
    const bool up1 = hipMemcpy(own1, w1, sizeof(w1), hipMemcpyHostToDevice) == hipSuccess;
    int st = ncclAllGather(own1, all1, 16, ncclDouble, c->nccl, s) == ncclSuccess ? QG_OK : QG_ERR_RCCL;
    if (st == QG_OK) st = comm_wait(c, s, nullptr, what);
    if (st != QG_OK) {  // the communicator itself failed (the watchdog aborted it): no gather 2
        region_release(g);
        return st;
    }
    if (!up1 && local == QG_OK) local = QG_ERR_HIP;
    std::vector<double> a1(16 * (size_t)G);
    if (local == QG_OK && hipMemcpy(a1.data(), all1, sizeof(double) * a1.size(), hipMemcpyDeviceToHost) != hipSuccess)
        local = QG_ERR_HIP;
    bool all_ok = local == QG_OK;
    for (int r = 0; all_ok && r < G; ++r) all_ok = a1[16 * (size_t)r + 8] == 0.0;
    for (int r = 0; all_ok && local == QG_OK && r < G; ++r) {
        if (r == c->rank) {
            g.remote[(size_t)r] = g.local;
        } else if (need[(size_t)r]) {
            hipIpcMemHandle_t h;
            std::memcpy(&h, &a1[16 * (size_t)r], sizeof(h));
            if (hipIpcOpenMemHandle((void **)&g.remote[(size_t)r], h, hipIpcMemLazyEnablePeerAccess) == hipSuccess)
                g.opened[(size_t)r] = 1;
            else {
                g.remote[(size_t)r] = nullptr;
                local = QG_ERR_UNSUPPORTED;
            }
        }
    }
    // gather 2: agree -- the transport switches only if every rank's set-up and opens succeeded
    double w2[8] = {(double)(local != QG_OK ? local : (all_ok ? QG_OK : QG_ERR_UNSUPPORTED))};
    if (hipMemcpy(own2, w2, sizeof(w2), hipMemcpyHostToDevice) != hipSuccess && local == QG_OK) local = QG_ERR_HIP;
    st = ncclAllGather(own2, all2, 8, ncclDouble, c->nccl, s) == ncclSuccess ? QG_OK : QG_ERR_RCCL;
    if (st == QG_OK) st = comm_wait(c, s, nullptr, what);
    std::vector<double> sts(8 * (size_t)G);
    if (st == QG_OK && hipMemcpy(sts.data(), all2, sizeof(double) * sts.size(), hipMemcpyDeviceToHost) != hipSuccess)
        st = QG_ERR_HIP;
    if (st == QG_OK && local != QG_OK) st = QG_ERR_UNSUPPORTED;
    for (int r = 0; st == QG_OK && r < G; ++r)
        if (sts[8 * (size_t)r] != 0.0) {
            std::fprintf(stderr, "qg_mi355 rank %d/%d: %s: IPC regions unavailable (rank %d: %s)\n", c->rank, G, what, r,
                         qg_strerror((int)sts[8 * (size_t)r]));
            st = QG_ERR_UNSUPPORTED;
        }
    if (st == QG_ERR_UNSUPPORTED && local != QG_OK)
        std::fprintf(stderr, "qg_mi355 rank %d/%d: %s: IPC regions unavailable here (%s)\n", c->rank, G, what,
                     qg_strerror(local));
    if (st != QG_OK) region_release(g);
    return st;
}

// Leave a peer transport: every rank drains its device, then one all-gather, so no
// neighbour's writes can still be landing in a region when it is released.
static int region_leave(Comm *c, Comm::IpcRegion &g, const char *what) {
    QG_HIP(hipDeviceSynchronize());
    const int b = comm_barrier(c, what);
    region_release(g);
    return b;
}

// Halo by kernel (QG_HALO_PUT): workgroup (b, d) stores part b of this rank's outgoing rows of
// direction d (0: top rows -> next's from_prev, 1: bottom rows -> prev's from_next) into the
// neighbour's region, drains its stores, releases at system scope and raises the neighbour's
// flag (d, b); then it waits for this rank's own flag (d, b), raised by the neighbour's
// matching workgroup.  Every workgroup stores before it waits.  A few small workgroups (no
// LDS, few registers) that fit beside the interior tendency; one launch per exchange.
struct PutArgs {
    const double *src[2][4];  // [dir][field]: the field's two outgoing rows (contiguous)
    double *dst[2];           // the neighbours' rows of this exchange's parity
    uint64_t *flag[2];        // the neighbours' flag bases for this direction
    const uint64_t *mine;     // this rank's flags
    int64_t words, seg;       // words per direction; words per field (2 rows)
    uint64_t seq, limit;
    int64_t *err, *progress;
    int64_t prog;
};

__global__ __launch_bounds__(256) void halo_put_kernel(PutArgs a) {
    const int b = blockIdx.x, d = blockIdx.y;
    const int64_t lo = a.words * b / PUT_BLOCKS, hi = a.words * (b + 1) / PUT_BLOCKS;
    // this workgroup's part, field by field; eight loads in flight per thread before their
    // stores (the state and a peer's region never alias) -- one memory latency per eight
    // words instead of one per word (r04: ~10 us per exchange on the 1-rank ring), and no
    // 64-bit division per word
    double *__restrict__ dst = a.dst[d];
    constexpr int U = 8;
    for (int f = 0; f < 4; ++f) {
        const int64_t f0 = (int64_t)f * a.seg, a0 = lo > f0 ? lo : f0, a1 = hi < f0 + a.seg ? hi : f0 + a.seg;
        const double *__restrict__ src = a.src[d][f] - f0;  // (indexed by the direction's word)
        for (int64_t i0 = a0 + threadIdx.x; i0 < a1; i0 += U * (int64_t)blockDim.x) {
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + (int64_t)u * blockDim.x;
                if (i < a1) v[u] = src[i];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + (int64_t)u * blockDim.x;
                if (i < a1) dst[i] = v[u];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(a.flag[d] + (size_t)b * 8, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t *f = a.mine + ((size_t)d * PUT_BLOCKS + b) * 8;
        const uint64_t t0 = wall_clock64();
        bool ok = true;
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
            if (wall_clock64() - t0 > a.limit ||
                __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                int64_t zero = 0;
                __hip_atomic_compare_exchange_strong(a.err, &zero, (int64_t)a.seq, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok && b == 0 && d == 0 && a.progress)
            __hip_atomic_store(a.progress, a.prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Collective (every rank, same arguments): switch the halo rows of comm_halo_rows to the
// peer transport for rows of `ld` words -- on = 1: copy engine, on = 2: put kernel (the same
// regions and flags; a switch between the two keeps them, flag values stay monotonic) -- or
// back to RCCL (on = 0).  RCCL transport only: the regions' IPC handles are all-gathered over it.
int comm_set_peer(void *comm, int on, int64_t ld) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || c->failed) return QG_ERR_RCCL;
    if (!on && !c->peer) return QG_OK;
    if (on && !c->nccl) return QG_ERR_UNSUPPORTED;
    if (on && ld < 1) return QG_ERR_INVALID_ARG;
    if (on && c->peer && c->peer_ld == ld) {  // (same regions; only the mover changes)
        QG_HIP(hipDeviceSynchronize());
        c->put = on == 2;
        return comm_barrier(c, "qg_comm_set_halo_transport (mode)");
    }
    if (c->peer) {
        c->peer = false;
        QG_CHECK(region_leave(c, c->halo_rx, "qg_comm_set_halo_transport (leave)"));
    }
    if (!on) return QG_OK;
    const int G = c->nranks;
    std::vector<char> need((size_t)G, 0);
    need[(size_t)((c->rank + 1) % G)] = need[(size_t)((c->rank - 1 + G) % G)] = 1;
    QG_CHECK(region_create(c, c->halo_rx, sizeof(double) * (size_t)(PEER_HDR + 4 * PEER_ROWS * ld), need,
                           "qg_comm_set_halo_transport"));
    c->peer = true;
    c->put = on == 2;
    c->peer_ld = ld;
    c->pseq = 0;
    return QG_OK;
}

// One halo exchange over the peer-copy transport: per field, this rank's top two rows go to
// next's from_prev rows and its bottom two rows to prev's from_next rows (copy engine, no
// compute units), then the flags; the rows of exchange seq land in parity seq & 1, so the
// next exchange never writes rows a neighbour may still be reading (every step also runs a
// collective between two exchanges).  rows_out as comm_halo_rows.
static int peer_halo_rows(Comm *c, double *const *f2, int n2, int64_t ld, int64_t P, hipStream_t s,
                          const double **rows_out) {
    if (n2 < 1 || 2 * n2 > PEER_ROWS) return QG_ERR_INVALID_ARG;
    if (ld != c->peer_ld) return QG_ERR_INVALID_ARG;
    if (c->perr_h && __atomic_load_n(c->perr_h, __ATOMIC_RELAXED) != 0) return comm_wait(c, s, nullptr, "halo exchange");
    const int64_t seq = ++c->pseq;
    const int par = (int)(seq & 1);
    const int G = c->nranks;
    double *rx_next = c->halo_rx.remote[(size_t)((c->rank + 1) % G)];
    double *rx_prev = c->halo_rx.remote[(size_t)((c->rank - 1 + G) % G)];
    double *to_next = peer_region(rx_next, ld, par, 0), *to_prev = peer_region(rx_prev, ld, par, 1);
    const double *from_prev = peer_region(c->halo_rx.local, ld, par, 0);
    const double *from_next = peer_region(c->halo_rx.local, ld, par, 1);
    const size_t bytes = sizeof(double) * 2 * (size_t)ld;
    if (c->put) {
        PutArgs a{};
        for (int f = 0; f < n2; ++f) {
            a.src[0][f] = f2[f] + fidx(0, P - 1, ld);
            a.src[1][f] = f2[f] + fidx(0, 1, ld);
            for (int q = 0; q < 2; ++q) {
                rows_out[4 * f + q] = from_prev + (2 * f + q) * ld;
                rows_out[4 * f + 2 + q] = from_next + (2 * f + q) * ld;
            }
        }
        a.dst[0] = to_next;
        a.dst[1] = to_prev;
        a.flag[0] = reinterpret_cast<uint64_t *>(rx_next);                        // next's (0, b)
        a.flag[1] = reinterpret_cast<uint64_t *>(rx_prev) + PUT_BLOCKS * 8;       // prev's (1, b)
        a.mine = reinterpret_cast<const uint64_t *>(c->halo_rx.local);
        a.words = 2 * (int64_t)n2 * ld;
        a.seg = 2 * ld;
        a.seq = (uint64_t)seq;
        a.limit = (uint64_t)(c->timeout_s * (double)c->clock_khz * 1000.0);
        a.err = c->perr_d;
        a.progress = c->progress_d;
        a.prog = c->seq + 1;
        halo_put_kernel<<<dim3(PUT_BLOCKS, 2), 256, 0, s>>>(a);
        QG_LAUNCH_CHECK();
        ++c->seq;
        return QG_OK;
    }
    for (int f = 0; f < n2; ++f) {
        const double *b = f2[f];
        QG_HIP(hipMemcpyAsync(to_next + 2 * f * ld, b + fidx(0, P - 1, ld), bytes, hipMemcpyDeviceToDeviceNoCU, s));
        QG_HIP(hipMemcpyAsync(to_prev + 2 * f * ld, b + fidx(0, 1, ld), bytes, hipMemcpyDeviceToDeviceNoCU, s));
        for (int q = 0; q < 2; ++q) {
            rows_out[4 * f + q] = from_prev + (2 * f + q) * ld;      // rows -2, -1
            rows_out[4 * f + 2 + q] = from_next + (2 * f + q) * ld;  // rows P, P+1
        }
    }
    peer_signal_kernel<<<1, 64, 0, s>>>(reinterpret_cast<uint64_t *>(rx_next),
                                        reinterpret_cast<uint64_t *>(rx_prev) + PUT_BLOCKS * 8,
                                        (uint64_t)seq);
    QG_LAUNCH_CHECK();
    const uint64_t limit = (uint64_t)(c->timeout_s * (double)c->clock_khz * 1000.0);
    peer_wait_kernel<<<1, 64, 0, s>>>(reinterpret_cast<const uint64_t *>(c->halo_rx.local), (uint64_t)seq, limit,
                                      c->progress_d, c->seq + 1, c->perr_d);
    QG_LAUNCH_CHECK();
    ++c->seq;
    return QG_OK;
}

// ---- peer record gather ----------------------------------------------------------------
struct PgArgs {
    const double *send;
    double *recv;
    int64_t count;
    double *dst[PG_MAX_RANKS];  // the ranks' regions as mapped here
    const double *mine;         // this rank's region
    int G, rank, par;
    uint64_t seq, limit;
    int64_t *err;
};

// Workgroup (b, r): part b of this rank's record -> rank r's region (slot [par][rank]), r's flag
// (rank, b) raised after every storing wave has drained (the release below writes the L2 back
// at system scope); then wait for r's flag (r, b) here and copy r's part b into recv.  Every
// workgroup stores before it waits, so no rank's kernel waits on a workgroup that is itself
// waiting.  Double-buffered by gather parity: a rank's gather k + 2 starts only after its
// gather k + 1 saw every peer's k + 1 flags, i.e. after every peer's gather k has finished.
// dst[i] = src[i] for i in [lo, hi) by one workgroup, eight loads in flight per thread before
// their stores (the buffers never alias)
__device__ __forceinline__ void copy_batched(double *__restrict__ dst, const double *__restrict__ src, int64_t lo,
                                             int64_t hi) {
    constexpr int U = 8;
    for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += U * (int64_t)blockDim.x) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * blockDim.x;
            if (i < hi) v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * blockDim.x;
            if (i < hi) dst[i] = v[u];
        }
    }
}

__global__ __launch_bounds__(256) void peer_gather_kernel(PgArgs a) {
    const int b = blockIdx.x, r = blockIdx.y;
    const int64_t hdr = (int64_t)a.G * PG_BLOCKS * 8;
    const int64_t lo = a.count * b / PG_BLOCKS, hi = a.count * (b + 1) / PG_BLOCKS;
    double *out = a.recv + (size_t)r * a.count;
    if (r == a.rank) {
        if (out != a.send) copy_batched(out, a.send, lo, hi);
        return;
    }
    double *rem = a.dst[r] + hdr + ((size_t)a.par * a.G + a.rank) * a.count;
    copy_batched(rem, a.send, lo, hi);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int timed_out;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<uint64_t *>(a.dst[r]) + ((size_t)a.rank * PG_BLOCKS + b) * 8, a.seq,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t *f = reinterpret_cast<const uint64_t *>(a.mine) + ((size_t)r * PG_BLOCKS + b) * 8;
        const uint64_t t0 = wall_clock64();
        timed_out = 0;
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
            if (wall_clock64() - t0 > a.limit ||
                __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                int64_t zero = 0;
                __hip_atomic_compare_exchange_strong(a.err, &zero, (int64_t)a.seq, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM);
                timed_out = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    if (timed_out) return;
    copy_batched(out, a.mine + hdr + ((size_t)a.par * a.G + r) * a.count, lo, hi);
}

// Collective (every rank, same arguments): gather records of `count` doubles (the direct
// solver's per-step rank records) by peer_gather_kernel, or by ncclAllGather (on = 0).
int comm_set_peer_gather(void *comm, int on, int64_t count) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || c->failed) return QG_ERR_RCCL;
    if (!on && !c->pgather) return QG_OK;
    if (on && !c->nccl) return QG_ERR_UNSUPPORTED;
    if (on && (count < 1 || c->nranks > PG_MAX_RANKS)) return QG_ERR_INVALID_ARG;
    if (on && c->pgather && c->pg_count == count) return QG_OK;
    if (c->pgather) {
        c->pgather = false;
        QG_CHECK(region_leave(c, c->gat_rx, "qg_comm_set_gather_transport (leave)"));
    }
    if (!on) return QG_OK;
    const int G = c->nranks;
    std::vector<char> need((size_t)G, 1);
    QG_CHECK(region_create(c, c->gat_rx, sizeof(double) * (size_t)(G * PG_BLOCKS * 8 + 2 * (int64_t)G * count), need,
                           "qg_comm_set_gather_transport"));
    c->pgather = true;
    c->pg_count = count;
    c->gseq = 0;
    return QG_OK;
}

// The solver's record all-gather: the peer kernel when selected, else comm_allgather.
int comm_gather_records(void *user, const double *send, double *recv, int64_t count, hipStream_t s) {
    Comm *c = static_cast<Comm *>(user);
    if (!c || c->failed) return QG_ERR_RCCL;
    if (!c->pgather) return comm_allgather(user, send, recv, count, s);
    if (count != c->pg_count) return QG_ERR_INVALID_ARG;
    if (c->perr_h && __atomic_load_n(c->perr_h, __ATOMIC_RELAXED) != 0) return comm_wait(c, s, nullptr, "record gather");
    if (c->nranks == 1) {  // (the one-rank ring's record is its own gather)
        if (recv != send) QG_HIP(hipMemcpyAsync(recv, send, sizeof(double) * (size_t)count, hipMemcpyDeviceToDevice, s));
        return QG_OK;
    }
    PgArgs a{};
    a.send = send;
    a.recv = recv;
    a.count = count;
    for (int r = 0; r < c->nranks; ++r) a.dst[r] = c->gat_rx.remote[(size_t)r];
    a.mine = c->gat_rx.local;
    a.G = c->nranks;
    a.rank = c->rank;
    a.seq = (uint64_t)++c->gseq;
    a.par = (int)(a.seq & 1);
    a.limit = (uint64_t)(c->timeout_s * (double)c->clock_khz * 1000.0);
    a.err = c->perr_d;
    peer_gather_kernel<<<dim3(PG_BLOCKS, (unsigned)c->nranks), 256, 0, s>>>(a);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

// depth == 2: halo rows into halo_buf; depth == -1: ghost-row refresh in place
int comm_halo(void *comm, double *const *fields, int nfields, int64_t M, int64_t P, int depth, double *halo_buf,
              hipStream_t s) {
    if (depth == 2) return comm_exchange(comm, fields, nfields, halo_buf, nullptr, 0, M + 2, P, s, false);
    return comm_exchange(comm, nullptr, 0, nullptr, fields, nfields, M + 2, P, s, false);
}

}  // namespace qg

extern "C" int qg_comm_exchange_plan(int rank, int nranks, int send_peer[2], int send_buf[2], int recv_peer[2],
                                     int recv_buf[2]) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !send_peer || !send_buf || !recv_peer || !recv_buf)
        return QG_ERR_INVALID_ARG;
    qg::exchange_plan(rank, nranks, send_peer, send_buf, recv_peer, recv_buf);
    return QG_OK;
}
