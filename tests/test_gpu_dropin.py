"""The reference-signature drop-in path and the slot bookkeeping around it.

- qg_set_keep_order: store_new_state! semantics (model.jl:102-106) on every call -- the
  history shifted in place, slot 1 = newest -- must give exactly the rotating path's logical
  arrays (bitwise), for both solvers and F32, stepping and qg_run.
- qg_canonicalize: the in-place rotation of every slot (one launch, each slot read once and
  written once) restores the reference order bitwise, and stepping on afterwards is unchanged.
- Deferred PCG certification: a check still pending when the slots move
  (canonicalize, set_slots, initialise, bind) is settled first and reports no false failure;
  HIP-graph replay captures and replays only in the pending steady state, so every solve is
  certified exactly once.
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qg():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    return qgamd


def _logical(st):
    return {n: st.logical(n).clone() for n in ("zeta", "psi", "f_store")}


def _physical(st):
    return {"zeta": st.zeta.clone(), "psi": st.psi.clone(), "f_store": st.f_store.clone()}


def _same(a, b):
    import torch
    for k in a:
        assert torch.equal(a[k], b[k]), k


# (1280 x 1024: above the direct kernel's cut-off, so the LDS-ring tendency (F64), its
# certifying two-layer form (PCG) and the pair kernel (F32) run with f_store's shift fused)
@pytest.mark.parametrize("M,P,solver,f32", [(64, 48, 0, False), (128, 128, 1, False), (64, 64, 0, True),
                                            (45, 30, 0, False), (1280, 1024, 0, False), (1280, 1024, 1, False),
                                            (1280, 1024, 0, True)])
def test_keep_order_matches_rotation(qg, M, P, solver, f32):
    import torch
    m = qg.bench_model(M, P=P)
    kw = dict(solver=solver, dtype=torch.float32 if f32 else None)
    a = qg.initialise_model(m, **kw)
    b = qg.initialise_model(m, **kw)
    b.set_keep_order(True)
    for t in range(1, 8):
        a.step(t)
        b.step(t)
        assert b.heads() == [0, 0, 0]
        _same(_physical(b), _logical(a))
    a.run(8, 11)
    b.run(8, 11)
    _same(_physical(b), _logical(a))


def test_keep_order_switch_canonicalizes(qg):
    m = qg.bench_model(64, P=32)
    a = qg.initialise_model(m)
    a.run(1, 5)  # heads rotated
    want = _logical(a)
    assert a.heads() != [0, 0, 0]
    a.set_keep_order(True)
    assert a.heads() == [0, 0, 0]
    _same(_physical(a), want)
    with pytest.raises(qg.QGError):
        a.set_heads([1, 0, 0])  # a rotation cannot be restored while the order is kept


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_canonicalize_in_place(qg, k):
    m = qg.bench_model(64, P=40)
    a = qg.initialise_model(m)
    b = qg.initialise_model(m)
    for t in range(1, k + 1):
        a.step(t)
        b.step(t)
    want = _logical(a)
    a.canonicalize()
    assert a.heads() == [0, 0, 0]
    _same(_physical(a), want)
    for t in range(k + 1, k + 5):
        a.step(t)
        b.step(t)
    _same(_logical(a), _logical(b))


def test_pending_certificate_settled_before_slots_move(qg):
    """a deferred check left pending by the last solve reads that solve's slots;
    canonicalize / set_slots / initialise run it first, so no false failure is reported."""
    m = qg.bench_model(64)
    st = qg.initialise_model(m, solver=1)
    for t in range(1, 5):
        st.step(t)           # the 4th solve's check is pending (it rides in the next tendency)
    st.canonicalize()        # moves psi slot 2 -> slot 0: settled first
    st.synchronize()
    c = st.pcg_certificate()
    assert c["solves"] == 4 and c["failures"] == 0, c
    st.step(5)
    h = st.heads()
    st.set_heads(h)          # settles the 5th solve's check
    st.step(6)
    st.initialise()          # settles the 6th, then overwrites the state
    st.synchronize()
    c = st.pcg_certificate()
    assert c["solves"] == 6 and c["failures"] == 0, c


def test_graph_replay_certifies_each_solve_once(qg, monkeypatch):
    """replays only in the pending steady state.  A run that starts after a
    standalone check settled the pending solve takes one stream step first; a cached graph
    replayed after a settle does not re-check a solve.  Every solve certified exactly once,
    states bitwise equal to stream launches."""
    m = qg.bench_model(128)
    ref = qg.initialise_model(m, solver=1)
    ref.run(1, 30)
    monkeypatch.setenv("QG_GRAPH", "1")
    st = qg.initialise_model(m, solver=1)
    st.run(1, 3)
    assert st.pcg_certificate()["solves"] == 3   # (qg_run settles at its end)
    st.run(4, 12)        # one stream step, then graph replays (captured with the check pending)
    c = st.pcg_certificate()
    assert c["solves"] == 15 and c["failures"] == 0, c
    st.run(16, 15)       # the cached graphs, after a settle
    c = st.pcg_certificate()
    assert c["solves"] == 30 and c["failures"] == 0, c
    _same(_logical(st), _logical(ref))


@pytest.mark.parametrize("M,solver", [(128, 0), (128, 1), (1280, 0)])
def test_keep_order_graph_replay(qg, monkeypatch, M, solver):
    """Keep-order stepping captured in HIP graphs (QG_GRAPH=1): the captured AB3 steps carry
    the in-place shifts (f_store's inside the tendency on one rank) and replay to exactly the
    rotating stream path's logical arrays."""
    m = qg.bench_model(M, P=1024 if M > 1000 else None)
    ref = qg.initialise_model(m, solver=solver)
    ref.run(1, 25)
    monkeypatch.setenv("QG_GRAPH", "1")
    st = qg.initialise_model(m, solver=solver)
    st.set_keep_order(True)
    st.run(1, 25)
    assert st.heads() == [0, 0, 0]
    _same(_physical(st), _logical(ref))


@pytest.mark.parametrize("f32", [False, True])
def test_reference_signatures_keep_order_and_unbind(qg, f32):
    """evolve_zeta!(model, zeta, psi, t, f_store) / evolve_psi!(model, zeta, psi, P, H) on bare
    arrays (an F32 state too): slot 1 newest after every call, equal to the
    rotating State; a different model for the same arrays is refused by evolve_psi_; unbind
    releases the cached context."""
    import torch
    m = qg.bench_model(64, P=48)
    dt = torch.float32 if f32 else None
    ref2 = qg.initialise_model(m, dtype=dt)
    zeta, psi, f_store = ref2.zeta.clone(), ref2.psi.clone(), ref2.f_store.clone()
    pc = qg.get_poisson_cholesky(m.M, m.P, m.dx)
    hc = qg.get_helmholtz_cholesky(m.M, m.P, m.dx, qg.S_eig(m))
    for t in range(1, 6):
        qg.evolve_zeta_(m, zeta, psi, t, f_store)
        qg.evolve_psi_(m, zeta, psi, pc, hc)
        ref2.step(t)
        _same({"zeta": zeta, "psi": psi, "f_store": f_store}, _logical(ref2))
    m2 = qg.bench_model(64, P=48, dt=m.dt / 2)
    with pytest.raises(ValueError):
        qg.evolve_psi_(m2, zeta, psi, pc, hc)
    assert qg.unbind(zeta, psi, f_store) == 1
    assert qg.unbind(zeta, psi, f_store) == 0


def _slot1_equal(b, a):
    """b keeps QG_KEEP_ORDER_SLOT1 order: physical slot 0 of zeta / psi and every slot of
    f_store equal (bitwise) to the rotating state a's logical ones."""
    import torch
    la = _logical(a)
    assert torch.equal(b.zeta[0], la["zeta"][0]) and torch.equal(b.psi[0], la["psi"][0])
    assert torch.equal(b.f_store, la["f_store"])


# slot 1 only (slots 2-3 of zeta / psi unmaintained, never read by the reference): after every
# evolve_zeta! the new zeta is in physical slot 1 (QG_KEEP_ORDER_SLOT1) or in the newest slot
# qg_slot names (QG_KEEP_ORDER_SLOT1_DEFERRED: slot 2 until the solve's pass A moves it), after
# every step zeta, psi and f_store are what the rotating path holds, ghost ring included --
# both solvers, F32, the LDS-ring and certifying tendencies (1280 x 1024), and the pass-A copies
# of the deferred mode at the benchmarked row lengths: the lane-exchange pass A (M = 4096) and
# the wide-row pass A (M = 8192, its hand-written ghost-column wrap), F64 and F32
@pytest.mark.parametrize("deferred", [False, True])
@pytest.mark.parametrize("M,P,solver,f32", [(64, 48, 0, False), (128, 128, 1, False), (64, 64, 0, True),
                                            (1280, 1024, 0, False), (1280, 1024, 1, False), (1280, 1024, 0, True),
                                            (4096, 16, 0, False), (4096, 16, 0, True), (8192, 8, 0, False),
                                            (8192, 8, 0, True)])
def test_keep_order_slot1_matches_rotation(qg, M, P, solver, f32, deferred):
    import torch
    m = qg.bench_model(M, P=P, dt=60.0 if M >= 4096 else 30.0 * 60)
    kw = dict(solver=solver, dtype=torch.float32 if f32 else None)
    a = qg.initialise_model(m, **kw)
    b = qg.initialise_model(m, **kw)
    b.set_keep_order(True, slot1_only=True, deferred=deferred)
    for t in range(1, 8):
        a.evolve_zeta_(t)
        b.evolve_zeta_(t)
        if deferred:  # the newest zeta is where qg_slot says
            assert torch.equal(b.logical("zeta")[0], a.logical("zeta")[0])
        else:  # slot 1 is the newest after every call
            assert b.heads() == [0, 0, 0] and torch.equal(b.zeta[0], a.logical("zeta")[0])
        a.evolve_psi_()
        b.evolve_psi_()
        assert b.heads() == [0, 0, 0]
        _slot1_equal(b, a)
    a.run(8, 11)
    b.run(8, 11)
    _slot1_equal(b, a)


def test_keep_order_slot1_graph_replay(qg, monkeypatch):
    m = qg.bench_model(128)
    ref = qg.initialise_model(m, solver=1)
    ref.run(1, 25)
    monkeypatch.setenv("QG_GRAPH", "1")
    st = qg.initialise_model(m, solver=1)
    st.set_keep_order(True, slot1_only=True)
    st.run(1, 25)
    _slot1_equal(st, ref)


@pytest.mark.parametrize("M,P,mode", [(1280, 1024, "slot1"), (1280, 1024, "slot1_deferred"),
                                     (256, 128, "slot1"), (256, 128, "slot1_deferred")])
def test_reference_signatures_slot1(qg, M, P, mode):
    """set_dropin_slots("slot1" / "slot1_deferred"): the reference-signature loop on bare
    arrays, slot 1 of zeta / psi and all of f_store equal to the rotating State after every
    step; with "slot1" also zeta[:, :, :, 1] right after evolve_zeta! -- the contract a caller
    reading the arrays between the two calls relies on."""
    import torch
    m = qg.bench_model(M, P=P)
    ref = qg.initialise_model(m)
    zeta, psi, f_store = ref.zeta.clone(), ref.psi.clone(), ref.f_store.clone()
    pc = qg.get_poisson_cholesky(m.M, m.P, m.dx)
    hc = qg.get_helmholtz_cholesky(m.M, m.P, m.dx, qg.S_eig(m))
    qg.set_dropin_slots(mode)
    try:
        for t in range(1, 7):
            qg.evolve_zeta_(m, zeta, psi, t, f_store)
            ref.evolve_zeta_(t)
            if mode == "slot1":
                torch.cuda.synchronize()
                assert torch.equal(zeta[0], _logical(ref)["zeta"][0])
            qg.evolve_psi_(m, zeta, psi, pc, hc)
            ref.evolve_psi_()
            la = _logical(ref)
            assert torch.equal(zeta[0], la["zeta"][0]) and torch.equal(psi[0], la["psi"][0])
            assert torch.equal(f_store, la["f_store"])
    finally:
        qg.set_dropin_slots("all")
        qg.unbind(zeta, psi, f_store)


def test_keep_order_slot1_to_full_refused(qg):
    """Lean mode leaves slots 2-3 of zeta / psi stale, so a direct switch to full keep-order
    (which promises store_new_state!'s slots after every call) is refused; via the rotating
    mode (0) it is allowed, and canonicalizes."""
    m = qg.bench_model(64)
    st = qg.initialise_model(m)
    st.set_keep_order(True, slot1_only=True)
    st.run(1, 3)
    with pytest.raises(qg.QGError) as e:
        st.set_keep_order(True)
    assert e.value.status == qg._lib.QG_ERR_INVALID_ARG
    st.set_keep_order(False)
    st.set_keep_order(True)
    st.run(4, 2)
    assert st.heads() == [0, 0, 0]


def test_keep_order_slot1_pending_move_settles(qg):
    """Deferred lean mode, spectral solver: the new zeta waits in slot 2 until the solve; two
    tendencies in a row, qg_synchronize and qg_canonicalize complete the move into slot 1
    first, so every path sees the reference's slot 1."""
    import torch
    m = qg.bench_model(128)
    a = qg.initialise_model(m)
    b = qg.initialise_model(m)
    b.set_keep_order(True, slot1_only=True, deferred=True)
    a.evolve_zeta_(1)
    b.evolve_zeta_(1)
    assert b.heads()[0] == 1  # pending: newest in slot 2
    b.synchronize()
    assert b.heads() == [0, 0, 0] and torch.equal(b.zeta[0], a.logical("zeta")[0])
    a.evolve_psi_()
    b.evolve_psi_()
    a.evolve_zeta_(2)
    b.evolve_zeta_(2)
    a.evolve_zeta_(3)  # two tendencies in a row
    b.evolve_zeta_(3)
    b.canonicalize()
    assert torch.equal(b.zeta[0], a.logical("zeta")[0])
    a.evolve_psi_()
    b.evolve_psi_()
    _slot1_equal(b, a)
