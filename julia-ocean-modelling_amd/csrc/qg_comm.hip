// RCCL plumbing for the y-slab decomposition (one rank per GPU, ring of ranks in y).
//   - halo rows for the tendency stencil: ncclSend/ncclRecv of whole contiguous rows to the
//     two ring neighbours inside one group (each row already carries its x-ghosts, so the
//     diagonal corners the Arakawa Jacobian reads arrive with it);
//   - ghost-row refresh of freshly written fields (drop-in ghost ring);
//   - the spectral solver's per-step all-gather of the rank records (a few hundred KB).
#include <rccl/rccl.h>

#include <cstring>

#include "qg_common.hpp"

namespace qg {

struct Comm {
    ncclComm_t nccl = nullptr;  // RCCL transport, or
    qg_allgather_fn ag = nullptr;  // host-provided transport (tests, MPI, ...)
    qg_sendrecv_fn sr = nullptr;
    void *user = nullptr;
    int nranks = 1, rank = 0;
};

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

int comm_init(void **comm, int nranks, int rank, const char id[128]) {
    Comm *c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
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
    *comm = c;
    return QG_OK;
}

int comm_destroy(void *comm) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c) return QG_OK;
    if (c->nccl) ncclCommDestroy(c->nccl);
    delete c;
    return QG_OK;
}

int comm_allgather(void *user, const double *send, double *recv, int64_t count, hipStream_t s) {
    Comm *c = static_cast<Comm *>(user);
    if (!c) return QG_ERR_RCCL;
    if (c->ag) return c->ag(c->user, send, recv, count, s) == 0 ? QG_OK : QG_ERR_RCCL;
    if (!c->nccl) return QG_ERR_RCCL;
    QG_NCCL(ncclAllGather(send, recv, (size_t)count, ncclDouble, c->nccl, s));
    return QG_OK;
}

// depth == 2: fill halo_buf[f][4][M+2] with rows -2,-1 (from rank-1) and P,P+1 (from rank+1)
// depth == -1: refresh the ghost rows (memory rows 0 and P+1) of each field in place
int comm_halo(void *comm, double *const *fields, int nfields, int64_t M, int64_t P, int depth, double *halo_buf,
              hipStream_t s) {
    Comm *c = static_cast<Comm *>(comm);
    if (!c || (!c->nccl && !c->sr)) return QG_ERR_RCCL;
    const int G = c->nranks;
    const int next = (c->rank + 1) % G, prev = (c->rank - 1 + G) % G;
    const size_t ld = (size_t)(M + 2);
    // one grouped exchange; per field: [send last rows -> next, send first rows -> prev] and
    // [recv low rows <- prev, recv high rows <- next] (this order also matches the two
    // messages per peer correctly when prev == next, i.e. two ranks)
    const int nmax = 4 * 16;
    if (nfields > 16) return QG_ERR_INVALID_ARG;
    const double *sp[nmax];
    double *rp[nmax];
    int64_t sc[nmax], rc[nmax];
    int speer[nmax], rpeer[nmax];
    int ns = 0, nr = 0;
    for (int f = 0; f < nfields; ++f) {
        double *b = fields[f];
        if (depth == 2) {
            double *lo = halo_buf + (size_t)f * 4 * ld, *hi = lo + 2 * ld;
            sp[ns] = b + fidx(0, P - 1, ld); sc[ns] = 2 * ld; speer[ns++] = next;
            sp[ns] = b + fidx(0, 1, ld);     sc[ns] = 2 * ld; speer[ns++] = prev;
            rp[nr] = lo; rc[nr] = 2 * ld; rpeer[nr++] = prev;
            rp[nr] = hi; rc[nr] = 2 * ld; rpeer[nr++] = next;
        } else {
            sp[ns] = b + fidx(0, P, ld); sc[ns] = ld; speer[ns++] = next;
            sp[ns] = b + fidx(0, 1, ld); sc[ns] = ld; speer[ns++] = prev;
            rp[nr] = b + fidx(0, 0, ld);     rc[nr] = ld; rpeer[nr++] = prev;
            rp[nr] = b + fidx(0, P + 1, ld); rc[nr] = ld; rpeer[nr++] = next;
        }
    }
    if (c->sr) return c->sr(c->user, ns, sp, sc, speer, nr, rp, rc, rpeer, s) == 0 ? QG_OK : QG_ERR_RCCL;
    QG_NCCL(ncclGroupStart());
    for (int k = 0; k < ns; ++k) QG_NCCL(ncclSend(sp[k], (size_t)sc[k], ncclDouble, speer[k], c->nccl, s));
    for (int k = 0; k < nr; ++k) QG_NCCL(ncclRecv(rp[k], (size_t)rc[k], ncclDouble, rpeer[k], c->nccl, s));
    QG_NCCL(ncclGroupEnd());
    return QG_OK;
}

}  // namespace qg
