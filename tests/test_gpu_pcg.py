"""Matrix-free PCG on the 5-point operator (QG_SOLVER_PCG): with the spectral preconditioner
(exact inverse of the periodic operator) and as plain CG, on sizes the direct path does not
support (non-power-of-two M), against the sparse direct solve of the same matrices and the
C oracle.  Tolerance: relative residual target 1e-12 -> solution error < 1e-9 relative
(plain CG: error <= cond(A) x residual) and < 1e-12 with the spectral preconditioner.
The residual target is 1e-12, or the roundoff floor (~cond(A) eps) where that is higher."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    from oracle import qg_oracle, qg_ref

    qg_oracle.build()
    return torch, qgamd, qg_ref, qg_oracle


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64).T)).cuda()


@pytest.mark.parametrize("M,P,precond,tol", [(32, 24, 1, 1e-12), (64, 64, 1, 1e-12), (40, 24, 0, 1e-9),
                                              (24, 20, 0, 1e-9)])
def test_pcg_solves_match_direct(env, M, P, precond, tol):
    torch, qg, R, O = env
    dx = 4e6 / M
    f = R.update_doubly_periodic_bc(R.seeded_rand(M, P, 9) - 0.5) * 1e-9
    for solve, ref in ((lambda: qg.sp_solve_poisson(M, P, dx, _dev(torch, f), kind=1, precond=precond),
                        R.sp_solve_poisson(M, P, dx, f)),
                       (lambda: qg.sp_solve_modified_helmholtz(M, P, dx, _dev(torch, f), -6.25e-10, kind=1,
                                                               precond=precond),
                        R.sp_solve_modified_helmholtz(M, P, dx, f, -6.25e-10))):
        got = solve().cpu().numpy().T
        assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < tol


@pytest.mark.parametrize("M,P,precond", [(64, 64, 1), (48, 40, 0)])
def test_pcg_model_run_matches_oracle(env, M, P, precond):
    torch, qg, R, O = env
    steps = 6
    st = qg.initialise_model(qg.bench_model(M, P=P), solver=1, precond=precond)
    for t in range(1, steps + 1):
        st.step(t)
        s = st.stats()
        assert max(s["relres"]) <= 1e-10 and s["iters"][0] >= 1
        if precond == 1:
            assert s["iters"][0] <= 3  # exact preconditioner: converges at once
    ref = O.State(R.bench_model(M, P=P)).run(steps)
    psi = st.to_numpy("psi")
    tol = 1e-10 if precond else 1e-8
    assert np.linalg.norm(psi - ref.psi) / np.linalg.norm(ref.psi) < tol


def test_certified_preconditioner_step(env):
    """Exact spectral preconditioner: the spectral solve writes psi = P_fwd z0 and one pass
    certifies ||b - B z0|| / ||b|| <= rtol -- one iteration per step, residual at roundoff."""
    torch, qg, R, O = env
    st = qg.initialise_model(qg.bench_model(64), solver=1)
    for t in range(1, 9):
        st.step(t)
        s = st.stats()
        assert s["iters"][0] == 1 and max(s["relres"]) < 1e-13, s
    ref = O.State(R.bench_model(64)).run(8)
    assert np.linalg.norm(st.to_numpy("psi") - ref.psi) / np.linalg.norm(ref.psi) < 1e-10


def test_certification_failure_restarts_from_z0(env):
    """A residual target below the roundoff floor: the certification fails, the general loop
    restarts from x0 = z0 and stops at its stagnation floor; the answer is unchanged."""
    torch, qg, R, O = env
    st = qg.initialise_model(qg.bench_model(64, P=48), solver=1, pcg_rtol=1e-30, pcg_maxit=50)
    st.set_pcg_sync(True)  # the host-checked form (the deferred default latches instead)
    for t in range(1, 5):
        st.step(t)
        s = st.stats()
        assert s["iters"][0] >= 2 and max(s["relres"]) <= 1e-10, s
    ref = O.State(R.bench_model(64, P=48)).run(4)
    assert np.linalg.norm(st.to_numpy("psi") - ref.psi) / np.linalg.norm(ref.psi) < 1e-10


def test_alpha_iteration_path(env):
    """qg_set_form(QG_FORM_PCG_NO_CERTIFICATE, 1): the fused alpha iteration (z0, alpha =
    (b,z0)/(z0,Bz0), psi = P(alpha z0)) that serves non-invertible back-projections; same answer."""
    torch, qg, R, O = env
    with qg.forced_form(qg._lib.QG_FORM_PCG_NO_CERTIFICATE, 1):
        st = qg.run_model_no_output(qg.bench_model(64), nsteps=6, solver=1)
    s = st.stats()
    assert s["iters"][0] == 1 and max(s["relres"]) < 1e-13
    ref = O.State(R.bench_model(64)).run(6)
    assert np.linalg.norm(st.to_numpy("psi") - ref.psi) / np.linalg.norm(ref.psi) < 1e-10


@pytest.mark.parametrize("N,steps", [(64, 9), (256, 7), (1024, 5), (1280, 4)])
def test_deferred_certificate_fused_in_tendency(env, N, steps):
    """Default (deferred) certification: no host read per step; on one GPU each solve's
    5-point residual is checked inside the next step's tendency (both layers per workgroup in
    the LDS-ring form, 1280^2; both layers per thread in the cache-resident form below
    1.2 M points) and latched on the device.  psi, zeta, f_store are bit-identical to the host-checked form,
    every solve is certified (the last one by the stand-alone pass at the read), and the
    latched residuals are at roundoff."""
    torch, qg, R, O = env
    m = qg.bench_model(N)
    a = qg.run_model_no_output(m, nsteps=steps, solver=1)          # deferred (default)
    b = qg.initialise_model(m, solver=1)
    b.set_pcg_sync(True)
    b.run(1, steps)
    for n in ("psi", "zeta", "f_store"):
        assert np.array_equal(a.to_numpy(n), b.to_numpy(n)), n
    c = a.pcg_certificate()
    assert c["solves"] == steps and c["failures"] == 0 and c["first_failure"] == 0, c
    assert 0 < c["worst_relres"] < 1e-13, c
    s = a.stats()
    assert s["iters"] == [1, 1] and max(s["relres"]) < 1e-13, s
    # the host-checked form's stand-alone pass: the same residual, at roundoff too
    sb = b.stats()
    assert sb["iters"] == [1, 1] and max(sb["relres"]) < 1e-13, sb
    # and the PCG trajectory itself against the C oracle (BASELINE config 2 at 1024^2: the
    # Arakawa tendency + Helmholtz PCG per step), psi and zeta at the north-star bar
    ref = O.State(R.bench_model(N)).run(steps)
    for n in ("psi", "zeta"):
        want, got = getattr(ref, n)[:, :, :, 0], a.to_numpy(n)[:, :, :, 0]
        e = np.linalg.norm(got - want) / np.linalg.norm(want)
        print(f"deferred PCG {N}^2 x {steps} steps vs C oracle, {n}: {e:.3e}")
        assert e < 1e-10, (n, e)


def test_deferred_certificate_failure_is_reported(env):
    """A target below the roundoff floor: every deferred certificate fails.  Single steps are
    not blocked; the next qg_synchronize reports QG_ERR_NOT_CONVERGED once, and the
    certificate record counts the failures from the first solve on.  qg_run reports it itself
    at its end (it settles and reads the latch), and a long run stops within two polling
    intervals (QG_PACE_STEPS = 16 steps) of the first failure instead of stepping on."""
    torch, qg, R, O = env
    st = qg.initialise_model(qg.bench_model(64), solver=1, pcg_rtol=1e-30)
    for t in range(1, 6):
        st.step(t)
    with pytest.raises(qg.QGError) as e:
        st.synchronize()
    assert e.value.status == -7
    st.synchronize()  # already reported
    c = st.pcg_certificate()
    assert c["solves"] == 5 and c["failures"] == 5 and c["first_failure"] == 1, c
    # qg_run: reported by the run that hit it, once
    st2 = qg.initialise_model(qg.bench_model(64), solver=1, pcg_rtol=1e-30)
    with pytest.raises(qg.QGError) as e:
        st2.run(1, 5)
    assert e.value.status == -7
    st2.synchronize()
    assert st2.pcg_certificate()["failures"] == 5
    # a long run stops early (the latch poll every 16 steps reads the copy of the interval before)
    st3 = qg.initialise_model(qg.bench_model(64), solver=1, pcg_rtol=1e-30)
    with pytest.raises(qg.QGError) as e:
        st3.run(1, 400)
    assert e.value.status == -7
    c3 = st3.pcg_certificate()
    assert 16 <= c3["solves"] <= 3 * 16 + 1 and c3["failures"] == c3["solves"], c3
    # the reference's own loop (evolve_zeta! / evolve_psi! per step): evolve_psi! polls too
    st4 = qg.initialise_model(qg.bench_model(64), solver=1, pcg_rtol=1e-30)
    stopped = None
    for t in range(1, 200):
        st4.evolve_zeta_(t)
        try:
            st4.evolve_psi_()
        except qg.QGError as e:
            assert e.status == -7
            stopped = t
            break
    assert stopped is not None and 16 <= stopped <= 3 * 16 + 1, stopped


def test_deferred_pcg_graph_replay(env, monkeypatch):
    """Deferred PCG steps have no host round trip, so qg_run replays them as HIP graphs:
    bit-identical to launching them on the stream, all solves certified."""
    torch, qg, R, O = env
    m = qg.bench_model(128)
    a = qg.run_model_no_output(m, nsteps=14, solver=1)
    monkeypatch.setenv("QG_GRAPH", "1")
    b = qg.run_model_no_output(m, nsteps=14, solver=1)
    for n in ("psi", "zeta", "f_store"):
        assert np.array_equal(a.to_numpy(n), b.to_numpy(n)), n
    c = b.pcg_certificate()
    assert c["solves"] == 14 and c["failures"] == 0, c


def test_deferred_failure_stops_graph_replay(env, monkeypatch):
    """QG_GRAPH=1: the replayed step graphs are polled between replays like stream steps, so a
    failed certificate stops a long run within a few polling intervals."""
    torch, qg, R, O = env
    monkeypatch.setenv("QG_GRAPH", "1")
    st = qg.initialise_model(qg.bench_model(64), solver=1, pcg_rtol=1e-30)
    with pytest.raises(qg.QGError) as e:
        st.run(1, 600)
    assert e.value.status == -7
    c = st.pcg_certificate()
    assert 16 <= c["solves"] <= 3 * 16 + 4 and c["failures"] == c["solves"], c


def test_plain_cg_256(env):
    """QG_PRECOND_NONE (plain CG) at 256^2, pcg_rtol 1e-13, pcg_maxit 3000: converges and
    matches the oracle at the north-star bar (1e-10).  Measured (r04, tools/cg_floor.py): 965
    iterations, psi 5.4e-12 from the oracle at 1e-13 (8.7e-11 at 1e-12, 1.0e-12 at 1e-14 and
    below: the floor); the iteration count is reported."""
    torch, qg, R, O = env
    m = qg.bench_model(256)
    st = qg.initialise_model(m, solver=1, precond=0, pcg_rtol=1e-13, pcg_maxit=3000)
    for t in range(1, 3):
        st.step(t)
        s = st.stats()
        print(f"plain CG 256^2 step {t}: iterations {s['iters']}, relres {s['relres']}")
        assert 1 < s["iters"][0] < 3000 and max(s["relres"]) <= 1e-10, s
    ref = O.State(R.bench_model(256)).run(2)
    for n in ("psi", "zeta"):
        e = np.linalg.norm(getattr(ref, n) - st.to_numpy(n)) / np.linalg.norm(getattr(ref, n))
        print(f"plain CG 256^2 vs C oracle, {n}: {e:.3e}")
        assert e < 1e-10, (n, e)
