"""Multi-rank RCCL on the one GPU of the test box.  RCCL refuses two ranks on one device of one
host ("Duplicate GPU detected"), so each rank process here declares a host of its own
(NCCL_HOSTID) and the ranks talk through RCCL's network transport over loopback
(NCCL_SOCKET_IFNAME=lo).  What runs is the library's real multi-rank RCCL code -- grouped
ncclSend/ncclRecv to two DISTINCT peers for the halo rows, ncclAllGather of the solver records
over 2 and 4 ranks, the PCG dot-product gathers, the watchdog waits -- not the host transport
and not the one-rank ring.  The transport between the ranks is loopback TCP, so nothing here
measures xGMI; the slabs must reproduce the single-GPU run of the same global model exactly as
the host-transport slabs do (tests/test_gpu_multirank.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, M, P, steps, outdir, solver, overlap, halo="rccl", gather="rccl", devices=False,
            kw=None):
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
    from bench import rccl_one_gpu_env

    if not devices:  # every rank on GPU 0 (RCCL over loopback); devices: rank r on GPU r
        os.environ.update(rccl_one_gpu_env(rank))  # (before RCCL initialises)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)  # (uid broadcast, barriers)
    torch.cuda.set_device(rank if devices else 0)
    import ctypes as C

    import qgamd

    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf = C.create_string_buffer(128)
        qgamd._lib.call("qg_comm_unique_id", buf)
        uid.copy_(torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8))
    dist.broadcast(uid, 0)
    m = qgamd.bench_model(M, P=P)
    st = qgamd.State(m, P_local=P // world, solver=solver, **(kw or {}))
    st.comm_init(world, rank, bytes(uid.numpy().tobytes()))
    if halo != "rccl":
        st.set_halo_transport(halo)
    if gather != "rccl":
        st.set_gather_transport(gather)
    st.set_overlap(overlap)
    st.initialise()
    st.run(1, steps)
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **{n: st.to_numpy(n) for n in ("zeta", "psi", "f_store")})
    dist.barrier()
    del st
    dist.destroy_process_group()


def _run(world, M, P, steps, d, solver, overlap, halo="rccl", gather="rccl", devices=False, kw=None):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, P, steps, d, solver, overlap, halo, gather,
                                               devices, kw))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:  # (a rank left waiting in a collective: stop exactly these children)
        if p.exitcode is None:
            p.terminate()
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]


MG = {"precond": 2, "pcg_rtol": 1e-13}  # QG_PRECOND_MULTIGRID
MG_PCG = dict(MG, solver=1)


@pytest.mark.parametrize("world,M,P,steps,solver,overlap,kw",
                         [(2, 64, 64, 6, 0, True, None), (2, 64, 64, 6, 0, False, None), (4, 64, 64, 5, 0, True, None),
                          (2, 64, 64, 5, 1, True, None), (2, 1024, 128, 4, 0, True, None),
                          (2, 128, 128, 4, 1, True, MG), (4, 256, 256, 3, 1, True, MG)])
def test_rccl_slabs_match_single_gpu(world, M, P, steps, solver, overlap, kw):
    """solver 0 = spectral (halo send/recv + record all-gather), 1 = PCG with the spectral
    preconditioner (its dot-product gathers and z halo also cross RCCL) or, kw = MG, the
    multigrid V-cycle (its per-level ghost-row refreshes and the agglomerated coarse grid's
    all-gathers over RCCL too)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    ref = qgamd.run_model_no_output(qgamd.bench_model(M, P=P), nsteps=steps, solver=solver, **(kw or {}))
    torch.cuda.synchronize()
    g = {n: ref.to_numpy(n) for n in ("zeta", "psi", "f_store")}
    with tempfile.TemporaryDirectory() as d:
        loc = _run(world, M, P, steps, d, solver, overlap, kw=kw)
    Pl = P // world
    for r in range(world):
        for n in ("zeta", "psi", "f_store"):
            want = g[n][:, r * Pl: r * Pl + Pl + 2]
            err = np.linalg.norm(loc[r][n] - want) / np.linalg.norm(want)
            assert err < 1e-12, (r, n, err)


def test_rccl_overlap_is_bit_identical():
    """The halo exchange on the second stream while the interior rows run, over real multi-rank
    RCCL: every slot of both slabs bit for bit equal to the serial schedule."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d0, tempfile.TemporaryDirectory() as d1:
        a = _run(2, 64, 64, 6, d0, 0, False)
        b = _run(2, 64, 64, 6, d1, 0, True)
    for r in range(2):
        for n in ("zeta", "psi", "f_store"):
            assert np.array_equal(a[r][n], b[r][n]), (r, n)


@pytest.mark.parametrize("world,overlap,halo,gather", [(2, True, "peer", "rccl"), (4, True, "peer", "rccl"),
                                                     (4, False, "peer", "rccl"), (2, True, "rccl", "peer"),
                                                     (4, True, "peer", "peer"), (3, True, "peer", "peer"),
                                                     (4, True, "put", "peer"), (2, False, "put", "rccl")])
def test_peer_transports_across_processes_bit_identical(world, overlap, halo, gather):
    """The peer transports between rank processes: each rank's receive regions are opened by
    the ranks that write into them through IPC (here all on the one GPU); halo rows arrive by
    copy engine with an arrival flag, the solver's records by the one-kernel gather; every slot
    of every slab bit for bit equal to the RCCL send/recv + ncclAllGather run (2 ranks: both
    ring neighbours are the same peer)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d0, tempfile.TemporaryDirectory() as d1:
        a = _run(world, 64, 48 * world // 2 if world == 3 else 64, 6, d0, 0, overlap)
        b = _run(world, 64, 48 * world // 2 if world == 3 else 64, 6, d1, 0, overlap, halo, gather)
    for r in range(world):
        for n in ("zeta", "psi", "f_store"):
            assert np.array_equal(a[r][n], b[r][n]), (r, n)


@pytest.mark.parametrize("halo,gather,overlap", [("put", "peer", False), ("peer", "peer", True)])
def test_peer_transports_across_devices_bit_identical(halo, gather, overlap):
    """The same check with one rank per GPU (needs >= 2 devices; skipped on a one-GPU box): the
    IPC regions opened across devices, rows and records written over xGMI, system-scope flags
    seen by the other device -- bit for bit equal to RCCL's send/recv + ncclAllGather."""
    import torch

    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs two GPUs")
    world = min(n, 4)
    with tempfile.TemporaryDirectory() as d0, tempfile.TemporaryDirectory() as d1:
        a = _run(world, 256, 64 * world, 6, d0, 0, True, devices=True)
        b = _run(world, 256, 64 * world, 6, d1, 0, overlap, halo, gather, devices=True)
    for r in range(world):
        for nm in ("zeta", "psi", "f_store"):
            assert np.array_equal(a[r][nm], b[r][nm]), (r, nm)


# ---- BASELINE configs 4 and 5 at their workload size over multi-rank RCCL ----------------

def _config_worker(rank, world, port, M, steps, outdir, f32, kw=None):
    """One slab of an M x (world*M) model over RCCL; saves its current zeta and psi slots
    (both layers, ghost rows included) for the parent's comparison with one GPU."""
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
    from bench import rccl_one_gpu_env

    os.environ.update(rccl_one_gpu_env(rank))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import ctypes as C

    import qgamd

    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf = C.create_string_buffer(128)
        qgamd._lib.call("qg_comm_unique_id", buf)
        uid.copy_(torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8))
    dist.broadcast(uid, 0)
    m = qgamd.bench_model(M, P=world * M, dt=60.0)
    st = qgamd.State(m, P_local=M, dtype=torch.float32 if f32 else torch.float64, **(kw or {}))
    st.comm_init(world, rank, bytes(uid.numpy().tobytes()))
    st.initialise()
    st.run(1, steps)
    st.synchronize()  # (collective: the lazily refreshed ghost rows)
    for n in ("zeta", "psi"):
        np.save(os.path.join(outdir, f"{n}{rank}.npy"), getattr(st, n)[st.slot(n, 1)].cpu().numpy())
    dist.barrier()
    del st
    dist.destroy_process_group()


# bars: test_gpu_configs.py's (F32: zeta < 16 eps_32, psi by the mechanism's derived bars of
# tests/f32_model.py -- the white-noise field's rounding amplified by the gravest Poisson modes)
@pytest.mark.parametrize("world,M,steps,f32,tol,kw", [(4, 4096, 4, False, {"zeta": 1e-10, "psi": 1e-10}, None),
                                                      (8, 8192, 3, True, {"zeta": 16 * 2.0 ** -24, "psi": 1.0}, None),
                                                      (4, 4096, 3, False, {"zeta": 1e-10, "psi": 1e-10}, MG_PCG)])
def test_rccl_config_slabs_match_single_gpu(world, M, steps, f32, tol, kw, capsys):
    """config 4: four 4096^2 F64 slabs (global 4096 x 16384); config 5: eight 8192^2 F32 slabs
    (global 8192 x 65536) -- over multi-rank RCCL, against the single-GPU run of the global
    model (the same bars as the host-transport form in test_gpu_configs.py).  kw = MG_PCG:
    config 4 as BASELINE words it ("RCCL halo + PCG all-reduce"), the PCG iterating with the
    multigrid preconditioner on the slabs, against the spectral direct solve on one GPU."""
    import torch
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_config_worker, args=(r, world, port, M, steps, d, f32, kw))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=400)
        for p in procs:
            if p.exitcode is None:
                p.terminate()
                p.join(timeout=30)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        m = qgamd.bench_model(M, P=world * M, dt=60.0)
        glob = qgamd.State(m, dtype=torch.float32 if f32 else torch.float64)
        glob.initialise()
        glob.run(1, steps)
        torch.cuda.synchronize()
        worst = {}
        for r in range(world):
            for n in ("zeta", "psi"):
                g = getattr(glob, n)[glob.slot(n, 1)][:, r * M: r * M + M + 2].double()
                a = torch.from_numpy(np.load(os.path.join(d, f"{n}{r}.npy"))).cuda().double()
                e = float(torch.linalg.vector_norm((a - g).reshape(-1)) / torch.linalg.vector_norm(g.reshape(-1)))
                worst[n] = max(worst.get(n, 0.0), e)
        rec = None
        if f32:
            import f32_model as F32
            asm = {}
            for n in ("zeta", "psi"):
                full = torch.zeros((2, world * M + 2, M + 2), dtype=torch.float32, device="cuda")
                for r in range(world):
                    a = torch.from_numpy(np.load(os.path.join(d, f"{n}{r}.npy"))).cuda()
                    full[:, 1 + r * M: 1 + (r + 1) * M] = a[:, 1:M + 1]
                asm[n] = full
            rec = F32.compare(qgamd, torch, m, [asm["zeta"][0], asm["zeta"][1]], [asm["psi"][0], asm["psi"][1]],
                              [glob.current("zeta", 1), glob.current("zeta", 2)],
                              [glob.current("psi", 1), glob.current("psi", 2)], mc=8)
    with capsys.disabled():
        print(f"\nRCCL {world} x {M}^2 {'F32' if f32 else 'F64'} slabs{' (MG-PCG)' if kw else ''} vs one GPU, "
              f"{steps} steps: {worst}"
              + (f"; {F32.fmt(rec)}; bars {F32.bars(rec)}" if rec else ""))
    assert all(worst[n] < tol[n] for n in worst), worst
    if rec:
        F32.check(rec)


# ---- failure paths over multi-rank RCCL -------------------------------------------------

def _rccl_state(rank, world, port, m, **kw):
    """(torch, dist, qgamd, State over RCCL) in a rank process (see _worker)."""
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
    from bench import rccl_one_gpu_env

    os.environ.update(rccl_one_gpu_env(rank))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import ctypes as C

    import qgamd

    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf = C.create_string_buffer(128)
        qgamd._lib.call("qg_comm_unique_id", buf)
        uid.copy_(torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8))
    dist.broadcast(uid, 0)
    st = qgamd.State(m(qgamd), P_local=kw.pop("P_local"), **kw)
    st.comm_init(world, rank, bytes(uid.numpy().tobytes()))
    return torch, dist, qgamd, st


def _silent_peer_worker(rank, world, port, outdir, halo="rccl"):
    """rank 1 joins the communicator and then never steps; rank 0 must get QG_ERR_RCCL from its
    watchdog (ncclCommAbort), not hang in the halo exchange."""
    import ctypes as C
    import json
    import time

    torch, dist, qgamd, st = _rccl_state(rank, world, port, lambda q: q.bench_model(64, P=64), P_local=32)
    if halo != "rccl":
        qgamd._lib.call("qg_comm_set_timeout", st._ctx, C.c_double(2.0))  # (the wait kernel's bound too)
        st.set_halo_transport(halo)
    st.initialise()
    dist.barrier()
    if rank == 1:
        time.sleep(25)
        os._exit(0)  # (its communicator's peer has aborted: no orderly destroy)
    qgamd._lib.call("qg_comm_set_timeout", st._ctx, C.c_double(2.0))
    t0 = time.perf_counter()
    res = {"status": 0}
    try:
        st.run(1, 64)
        st.synchronize()
    except qgamd.QGError as e:
        res["status"] = e.status
    res["waited"] = time.perf_counter() - t0
    open(os.path.join(outdir, "silent.json"), "w").write(json.dumps(res))
    os._exit(0)


@pytest.mark.parametrize("halo", ["rccl", "peer"])
def test_rccl_silent_peer_returns_rccl_error(halo):
    import json

    import torch
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qgamd import _lib

    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_silent_peer_worker, args=(r, 2, port, d, halo)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=120)
        for p in procs:
            if p.exitcode is None:
                p.terminate()
                p.join(timeout=30)
        res = json.load(open(os.path.join(d, "silent.json")))
    assert res["status"] == _lib.QG_ERR_RCCL, res
    assert res["waited"] < 20, res  # the watchdog's 2 s (plus the abort), not the peer's 25 s


def _cert_fail_rccl_worker(rank, world, port, outdir):
    import json

    torch, dist, qgamd, st = _rccl_state(rank, world, port, lambda q: q.bench_model(64, P=64), P_local=64 // world,
                                         solver=1, pcg_rtol=1e-30)
    st.initialise()
    res = {"stop": -1}
    for t in range(1, 200):  # the reference's loop, one call per step
        st.evolve_zeta_(t)
        try:
            st.evolve_psi_()
        except qgamd.QGError as e:
            res["status"] = e.status
            res["stop"] = t
            break
    res["cert"] = st.pcg_certificate()
    open(os.path.join(outdir, f"cert{rank}.json"), "w").write(json.dumps(res))
    dist.barrier()
    del st
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_failed_certificate_stops_every_rank_at_the_same_step(world):
    """Deferred PCG with an unreachable residual target across RCCL slabs: every rank reports
    QG_ERR_NOT_CONVERGED at the same step (the latch poll is collective), none steps on into an
    exchange its peers never post."""
    import json

    import torch
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_cert_fail_rccl_worker, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        for p in procs:
            if p.exitcode is None:
                p.terminate()
                p.join(timeout=30)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res = [json.load(open(os.path.join(d, f"cert{r}.json"))) for r in range(world)]
    assert all(r.get("status") == -7 for r in res), res
    assert len({r["stop"] for r in res}) == 1 and 16 <= res[0]["stop"] <= 3 * 16 + 1, res
    assert len({json.dumps(r["cert"], sort_keys=True) for r in res}) == 1, res
