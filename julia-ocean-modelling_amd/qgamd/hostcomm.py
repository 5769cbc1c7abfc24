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
    return _hip


H2D, D2H = 1, 2


def _d2h(ptr, count):
    a = np.empty(int(count), dtype=np.float64)
    assert hip().hipMemcpy(a.ctypes.data, ptr, a.nbytes, D2H) == 0
    return a


def _h2d(ptr, a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    assert hip().hipMemcpy(ptr, a.ctypes.data, a.nbytes, H2D) == 0


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
            _h2d(recv, torch.cat(parts).numpy())
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
                _h2d(rp[k], bufs[k].numpy())
            return 0
        except Exception as e:
            print("sendrecv callback failed:", e, flush=True)
            return 1

    def attach(self, state, nranks, rank):
        from ._lib import call

        call("qg_comm_init_host", state._ctx, int(nranks), int(rank), self._ag, self._sr, None)
        state.rank, state.nranks = rank, nranks
        state._transport = self  # keep the callbacks alive
