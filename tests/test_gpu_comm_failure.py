"""Failure handling of the multi-GPU path (include/qg_mi355.h, qg_comm_set_timeout): a
transport error or a stalled exchange must come back as QG_ERR_RCCL with the rank and the call
named, never as a hung rank.  Exercised on the one GPU of the test box:
  - a host transport whose sendrecv fails -> qg_run returns QG_ERR_RCCL, and the transport
    stays failed;
  - a stream that makes no progress (a spin kernel standing in for a peer that never posts
    its send) -> qg_synchronize returns QG_ERR_RCCL after the watchdog timeout, through the
    host transport and through a one-rank RCCL ring (ncclCommAbort path), instead of
    blocking until the kernel ends.
The reference (one Julia process) has no such path; this guards SURVEY 8(e)."""
import ctypes as C
import re
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    from qgamd import _lib, hostcomm
    return torch, qgamd, _lib, hostcomm


class Loopback:
    """One-rank host transport: every message goes to this rank itself (device copies)."""

    def __init__(self, _lib, hostcomm, fail_sendrecv=False):
        self.fail = fail_sendrecv
        self.calls = 0
        h = hostcomm.hip()
        h.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        h.hipMemcpyAsync.restype = C.c_int
        self.h = h

        def ag(user, send, recv, count, stream):
            return 0 if h.hipMemcpyAsync(recv, send, 8 * count, 3, stream) == 0 else 1

        def sr(user, ns, sp, sc, speer, nr, rp, rc, rpeer, stream):
            self.calls += 1
            if self.fail:
                return 1
            for k in range(nr):  # per-peer FIFO == posting order with a single peer
                if h.hipMemcpyAsync(rp[k], sp[k], 8 * rc[k], 3, stream) != 0:
                    return 1
            return 0

        self._ag, self._sr = _lib.AllgatherFn(ag), _lib.SendrecvFn(sr)

    def attach(self, st, _lib):
        assert _lib.lib().qg_comm_init_host(st._ctx, 1, 0, self._ag, self._sr, None) == _lib.QG_OK
        st._attached_ranks = 1
        st._transport = self


def _spin_cycles(torch, seconds):
    """torch.cuda._sleep cycles for about `seconds` of wall time (calibrated here)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    torch.cuda._sleep(int(5e7))
    b.record()
    torch.cuda.synchronize()
    per_s = 5e7 / max(a.elapsed_time(b) * 1e-3, 1e-6)
    return int(per_s * seconds)


def test_loopback_transport_matches_single_gpu(env):
    torch, qgamd, _lib, hostcomm = env
    m = qgamd.bench_model(64, P=48)
    ref = qgamd.run_model_no_output(m, nsteps=40)
    st = qgamd.State(m)
    Loopback(_lib, hostcomm).attach(st, _lib)
    st.initialise()
    st.run(1, 40)  # > 2 pacing intervals
    for n in ("zeta", "psi", "f_store"):
        a, b = st.to_numpy(n), ref.to_numpy(n)
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 1e-13, n


def test_failed_sendrecv_returns_rccl_error(env, capfd):
    torch, qgamd, _lib, hostcomm = env
    st = qgamd.State(qgamd.bench_model(64, P=48))
    tr = Loopback(_lib, hostcomm, fail_sendrecv=True)
    tr.attach(st, _lib)
    st.initialise()
    with pytest.raises(_lib.QGError) as e:
        st.run(1, 5)
    assert e.value.status == _lib.QG_ERR_RCCL
    assert "rank 0/1" in capfd.readouterr().err
    tr.fail = False  # the transport stays failed even if the peer would answer now
    n = tr.calls
    with pytest.raises(_lib.QGError) as e:
        st.run(2, 1)
    assert e.value.status == _lib.QG_ERR_RCCL and tr.calls == n


@pytest.mark.parametrize("transport", ["host", "rccl"])
def test_stalled_stream_times_out(env, transport, capfd):
    torch, qgamd, _lib, hostcomm = env
    st = qgamd.State(qgamd.bench_model(64, P=48))
    if transport == "host":
        Loopback(_lib, hostcomm).attach(st, _lib)
    else:
        uid = C.create_string_buffer(128)
        _lib.call("qg_comm_unique_id", uid)
        st.comm_init(1, 0, uid.raw)
    st.initialise()
    st.run(1, 6)
    st.synchronize()  # nothing pending: the next wait sees only the spin kernel
    _lib.call("qg_comm_set_timeout", st._ctx, C.c_double(0.3))
    cycles = _spin_cycles(torch, 2.0)
    torch.cuda._sleep(cycles)  # on the stream the library works on
    t0 = time.perf_counter()
    with pytest.raises(_lib.QGError) as e:
        st.synchronize()
    waited = time.perf_counter() - t0
    torch.cuda.synchronize()  # let the spin kernel finish
    assert e.value.status == _lib.QG_ERR_RCCL
    err = capfd.readouterr().err
    assert "rank 0/1" in err and "qg_synchronize" in err, err
    # the watchdog fired at its timeout, not at the end of the kernel ...
    assert re.search(r"no halo exchange completed for 0\.[3-5] s", err), err
    if transport == "host":  # ... and the call returned then (ncclCommAbort, by contrast,
        assert 0.25 < waited < 1.8, waited  # waits for the stream's non-RCCL kernels)
    else:
        assert waited > 0.25, waited
    with pytest.raises(_lib.QGError):
        st.run(7, 1)  # the failed transport is not reused
