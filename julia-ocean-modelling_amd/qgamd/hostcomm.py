"""Host-provided transport for qg_comm_init_host: moves halo rows and solver records through
torch.distributed (any backend, e.g. gloo) via host memory.

Used to exercise the multi-rank path when several ranks share one GPU (RCCL refuses
duplicate devices) and as a template for an MPI transport.  The production transport is
RCCL inside the library (qg_comm_init).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import AllgatherFn, SendrecvFn

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
        _hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        _hip.hipStreamSynchronize.restype = C.c_int
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemcpyAsync.restype = C.c_int
    return _hip


H2D, D2H = 1, 2


def _d2h(ptr, count):
    a = np.empty(int(count), dtype=np.float64)
    assert hip().hipMemcpy(a.ctypes.data, ptr, a.nbytes, D2H) == 0
    return a


def _h2d(ptr, a, stream=None):
    """Host -> device on the rank's stream, complete on return (a null-stream copy is not
    ordered with the library's non-blocking streams)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    h = hip()
    assert h.hipMemcpyAsync(ptr, a.ctypes.data, a.nbytes, H2D, stream) == 0
    assert h.hipStreamSynchronize(stream) == 0


class TorchDistTransport:
    """Callbacks over an initialised torch.distributed process group."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self._ag = AllgatherFn(self._allgather)
        self._sr = SendrecvFn(self._sendrecv)

    def _allgather(self, user, send, recv, count, stream):
        try:
            import torch

            hip().hipStreamSynchronize(stream)
            mine = torch.from_numpy(_d2h(send, count))
            parts = [torch.empty_like(mine) for _ in range(self.dist.get_world_size(self.group))]
            self.dist.all_gather(parts, mine, group=self.group)
            _h2d(recv, torch.cat(parts).numpy(), stream)
            return 0
        except Exception as e:  # never let an exception cross the C boundary
            print("allgather callback failed:", e, flush=True)
            return 1

    def _sendrecv(self, user, ns, sp, sc, speer, nr, rp, rc, rpeer, stream):
        try:
            import torch

            hip().hipStreamSynchronize(stream)
            # messages between one pair of ranks match in posting order: tag = per-peer index
            reqs, nsent, nrecv = [], {}, {}
            for k in range(ns):
                t = torch.from_numpy(_d2h(sp[k], sc[k]))
                peer = int(speer[k])
                tag = nsent.get(peer, 0)
                nsent[peer] = tag + 1
                reqs.append(self.dist.isend(t, peer, group=self.group, tag=tag))
            bufs = []
            for k in range(nr):
                b = torch.empty(int(rc[k]), dtype=torch.float64)
                peer = int(rpeer[k])
                tag = nrecv.get(peer, 0)
                nrecv[peer] = tag + 1
                reqs.append(self.dist.irecv(b, peer, group=self.group, tag=tag))
                bufs.append(b)
            for r in reqs:
                r.wait()
            for k in range(nr):
                _h2d(rp[k], bufs[k].numpy(), stream)
            return 0
        except Exception as e:
            print("sendrecv callback failed:", e, flush=True)
            return 1

    def attach(self, state, nranks, rank):
        from ._lib import call

        call("qg_comm_init_host", state._ctx, int(nranks), int(rank), self._ag, self._sr, None)
        state.rank, state.nranks = rank, nranks
        state._attached_ranks = nranks
        state._transport = self  # keep the callbacks alive


class ThreadRing:
    """In-process ring of G ranks, one Python thread per rank, over qg_comm_init_host.

    Every rank's State lives in this process (on one GPU or several); a grouped sendrecv or
    an all-gather is a rendezvous of all G threads at a barrier, then device-to-device copies
    straight between the ranks' staging buffers (no host bounce), then a second barrier so no
    sender reuses a buffer before every receiver has copied it.  Messages between one pair of
    ranks match in posting order, as with RCCL.  ctypes releases the GIL around the library
    calls, so the G ranks' kernels overlap on the device.

    Used to run the multi-rank path at workload size on the single GPU of a test box and to
    compare the slabs with a single-GPU run of the same global model on the device, without
    moving the fields through host memory.  A rank that fails (or a barrier not reached within
    `timeout` seconds) breaks the barrier for all, and each callback returns non-zero, so every
    rank's library call returns QG_ERR_RCCL instead of hanging.
    """

    def __init__(self, nranks, timeout=300.0):
        import threading

        self.G = nranks
        self.timeout = timeout
        self.barrier = threading.Barrier(nranks, timeout=timeout)
        self.sends = [None] * nranks
        self.gather = [None] * nranks
        self._cb = []

    def _wait(self):
        self.barrier.wait()

    def attach(self, state, rank):
        from ._lib import call

        h = hip()
        D2D = 3
        # The copies run on the rank's own stream and complete before the second barrier: a
        # device-to-device hipMemcpy may return before its copy has run, and on the null stream
        # it is not ordered with the ranks' (non-blocking) streams -- a receiver's next kernel
        # could read, or a sender's next pack kernel overwrite, a buffer still being copied.

        def ag(user, send, recv, count, stream):
            try:
                if h.hipStreamSynchronize(stream) != 0:
                    return 1
                self.gather[rank] = (int(send), int(count))
                self._wait()
                for q, (ptr, n) in enumerate(self.gather):
                    if n != count or h.hipMemcpyAsync(int(recv) + 8 * q * count, ptr, 8 * count, D2D, stream) != 0:
                        return 1
                if h.hipStreamSynchronize(stream) != 0:
                    return 1
                self._wait()
                return 0
            except Exception as e:  # includes threading.BrokenBarrierError
                self.barrier.abort()
                print(f"ThreadRing rank {rank}: allgather failed: {e!r}", flush=True)
                return 1

        def sr(user, ns, sp, sc, speer, nr, rp, rc, rpeer, stream):
            try:
                if h.hipStreamSynchronize(stream) != 0:
                    return 1
                self.sends[rank] = [(int(speer[k]), int(sp[k]), int(sc[k])) for k in range(ns)]
                self._wait()
                taken = {}
                for k in range(nr):
                    peer = int(rpeer[k])
                    n = taken.get(peer, 0)  # the n-th message this rank takes from `peer`
                    taken[peer] = n + 1
                    mine = [m for m in self.sends[peer] if m[0] == rank]
                    _, ptr, cnt = mine[n]
                    if cnt != rc[k] or h.hipMemcpyAsync(int(rp[k]), ptr, 8 * cnt, D2D, stream) != 0:
                        return 1
                if h.hipStreamSynchronize(stream) != 0:
                    return 1
                self._wait()
                return 0
            except Exception as e:
                self.barrier.abort()
                print(f"ThreadRing rank {rank}: sendrecv failed: {e!r}", flush=True)
                return 1

        agf, srf = AllgatherFn(ag), SendrecvFn(sr)
        self._cb.append((agf, srf))
        call("qg_comm_init_host", state._ctx, int(self.G), int(rank), agf, srf, None)
        state.rank, state.nranks = rank, self.G
        state._attached_ranks = self.G
        state._transport = self

    @staticmethod
    def run_all(fns):
        """Run fns[r]() on G threads; re-raise the first exception."""
        import threading

        errs = [None] * len(fns)

        def body(r):
            try:
                fns[r]()
            except BaseException as e:  # noqa: BLE001 -- reported below
                errs[r] = e

        ts = [threading.Thread(target=body, args=(r,)) for r in range(len(fns))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in errs:
            if e is not None:
                raise e
