"""The halo-exchange posting schedule of the multi-GPU path (qg_comm_exchange_plan, the exact
plan comm_exchange issues through RCCL or the host transport), checked on the CPU for ring
sizes 1..8: messages are matched per (sender, receiver) pair in posting order -- RCCL's
send/recv semantics -- and every slab must receive its neighbours' boundary rows in the right
halo buffer.  G = 1 (the self-ring) and G = 2 (both neighbours are the same rank, so the
order of the two messages per peer decides which halo each lands in) are the cases where a
wrong posting order would silently swap halos; larger rings check distinct peers.

Reference: the y-periodic domain of update_doubly_periodic_bc! (boundary_conditions.jl:2-13)
split into slabs; the halo below slab r is slab r-1's top rows, the halo above
it slab r+1's bottom rows, periodically."""
import collections

import pytest

from qgamd import _lib


def _plan(L, rank, G):
    sp, sb, rp, rb = ((_lib.C.c_int * 2)() for _ in range(4))
    assert L.qg_comm_exchange_plan(rank, G, sp, sb, rp, rb) == _lib.QG_OK
    return list(sp), list(sb), list(rp), list(rb)


@pytest.mark.parametrize("G", [1, 2, 3, 4, 5, 8])
def test_exchange_plan_delivers_the_right_halos(G):
    L = _lib.lib()
    queues = collections.defaultdict(collections.deque)  # (src, dst) -> posted send buffers
    plans = [_plan(L, r, G) for r in range(G)]
    for r, (sp, sb, _, _) in enumerate(plans):
        for peer, buf in zip(sp, sb):
            assert 0 <= peer < G
            queues[(r, peer)].append((r, buf))
    for r, (_, _, rp, rb) in enumerate(plans):
        got = {}
        for peer, buf in zip(rp, rb):
            got[buf] = queues[(peer, r)].popleft()  # FIFO per pair of ranks
        prev, nxt = (r - 1) % G, (r + 1) % G
        assert got[_lib.QG_XBUF_FROM_PREV] == (prev, _lib.QG_XBUF_TO_NEXT), (G, r, got)
        assert got[_lib.QG_XBUF_FROM_NEXT] == (nxt, _lib.QG_XBUF_TO_PREV), (G, r, got)
    assert all(len(q) == 0 for q in queues.values())  # every send matched exactly once


def test_exchange_plan_rejects_bad_ranks():
    L = _lib.lib()
    a = [(_lib.C.c_int * 2)() for _ in range(4)]
    assert L.qg_comm_exchange_plan(2, 2, *a) == _lib.QG_ERR_INVALID_ARG
    assert L.qg_comm_exchange_plan(0, 0, *a) == _lib.QG_ERR_INVALID_ARG
    assert L.qg_comm_exchange_plan(-1, 4, *a) == _lib.QG_ERR_INVALID_ARG
