"""RCCL transport on real hardware with the one GPU of the test box: a one-rank RCCL
communicator turns the y ring onto itself, so every halo send/recv, ghost-row refresh and
record all-gather of the multi-GPU path runs through RCCL (send-to-self) and must reproduce
the plain single-GPU path."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("overlap", [False, True])
def test_one_rank_rccl_ring_matches_single_gpu(overlap):
    """overlap: the halo exchange (RCCL send/recv to self) on the second stream while the
    interior rows' tendency runs -- bitwise equal to the default schedule."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    m = qgamd.bench_model(64, P=48)
    ref = qgamd.run_model_no_output(m, nsteps=7)
    st = qgamd.State(m)
    uid = C.create_string_buffer(128)
    qgamd._lib.call("qg_comm_unique_id", uid)
    st.comm_init(1, 0, uid.raw)
    st.set_overlap(overlap)
    st.initialise()
    st.run(1, 7)
    torch.cuda.synchronize()
    for n in ("zeta", "psi", "f_store"):
        a, b = st.to_numpy(n), ref.to_numpy(n)
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 1e-13, n
    if overlap:  # same ring without the overlap (the default is on): bit for bit
        st2 = qgamd.State(m)
        uid2 = C.create_string_buffer(128)
        qgamd._lib.call("qg_comm_unique_id", uid2)
        st2.comm_init(1, 0, uid2.raw)
        st2.set_overlap(False)
        st2.initialise()
        st2.run(1, 7)
        for n in ("zeta", "psi", "f_store"):
            assert np.array_equal(st.to_numpy(n), st2.to_numpy(n)), n


def _ring_state(qgamd, m, transport, overlap, **kw):
    st = qgamd.State(m, **kw)
    uid = C.create_string_buffer(128)
    qgamd._lib.call("qg_comm_unique_id", uid)
    st.comm_init(1, 0, uid.raw)
    st.set_halo_transport(transport)
    st.set_overlap(overlap)
    st.initialise()
    return st


@pytest.mark.parametrize("M,P,f32,overlap,halo", [(64, 48, False, True, "peer"), (64, 48, False, False, "peer"),
                                                  (96, 64, True, True, "peer"), (1024, 256, False, True, "peer"),
                                                  (64, 48, False, True, "put"), (64, 48, False, False, "put"),
                                                  (96, 64, True, True, "put"), (1024, 256, False, True, "put")])
def test_one_rank_peer_halo_bit_identical(M, P, f32, overlap, halo):
    """The peer-copy halo transport (copy engine into the IPC-style receive region, arrival
    flags, one-lane wait kernel) over the one-rank ring: every slot bit for bit equal to the
    RCCL send/recv transport, for both schedules and both precisions."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    m = qgamd.bench_model(M, P=P)
    kw = {"dtype": torch.float32} if f32 else {}
    a = _ring_state(qgamd, m, "rccl", overlap, **kw)
    a.run(1, 9)
    b = _ring_state(qgamd, m, halo, overlap, **kw)
    b.run(1, 9)
    torch.cuda.synchronize()
    for n in ("zeta", "psi", "f_store"):
        assert np.array_equal(a.to_numpy(n), b.to_numpy(n)), n


def test_one_rank_peer_halo_switch_and_probe():
    """Switching the transport between steps (collective re-setup and release), the comm probe's
    back-to-back exchanges in peer mode, and a second switch back: the trajectory stays bit for
    bit the RCCL one."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    m = qgamd.bench_model(128, P=64)
    a = _ring_state(qgamd, m, "rccl", True)
    a.run(1, 12)
    b = _ring_state(qgamd, m, "rccl", True)
    b.run(1, 4)
    b.set_halo_transport("peer")
    pr = b.comm_probe(5)
    assert pr["halo_ms"] > 0
    b.run(5, 4)
    b.set_halo_transport("rccl")
    b.run(9, 2)
    b.set_halo_transport("put")
    b.run(11, 1)
    b.set_halo_transport("peer")
    b.run(12, 1)
    torch.cuda.synchronize()
    for n in ("zeta", "psi", "f_store"):
        assert np.array_equal(a.to_numpy(n), b.to_numpy(n)), n
