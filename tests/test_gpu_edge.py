"""Edge cases of the device path against the C oracle: the smallest grids the spectral solver
takes (M = 8, P = 3), the reference's two-point domains (M or P = 2), odd P (chunk of one row), non-square slabs both ways, an explicit chunk
size, rows of every length up to 262144 points (mixed-radix, split, wide split and Bluestein
row transforms), and the refusal of what the spectral solver cannot do.  Relative RMS < 1e-10 after a few Euler + AB3 steps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-10


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def modal_residuals(R, m, zeta, psi):
    """Relative residuals ||A x - b|| / ||b|| of the two modal systems evolve_psi solves
    (model.jl:172-199), x recovered from the newest psi slot: the pinned Poisson system
    (laplacian.jl:66-75) and the modified Helmholtz system (laplacian.jl:60-64).  A
    solver-independent exactness check where two exact solvers differ by cond(A) x eps."""
    Pm = np.asarray(R.P_matrix(m.H_1, m.H_1))
    Pi = np.asarray(R.P_inv_matrix(m))
    x = np.einsum("ik,abk->abi", np.linalg.inv(Pm), psi[1:-1, 1:-1, :, 0])
    zt = np.einsum("ik,abk->abi", Pi, zeta[1:-1, 1:-1, :, 0])
    out = []
    for i, A in enumerate((R._pin_first(-R.construct_spA(m.M, m.P, m.dx, 0.0)),
                           -R.construct_spA(m.M, m.P, m.dx, R.S_eig(m)))):
        b = -R._vec(zt[:, :, i])
        if i == 0:
            b[0] = 0
        out.append(float(np.linalg.norm(A @ R._vec(x[:, :, i]) - b) / np.linalg.norm(b)))
    return out


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    from oracle import qg_oracle, qg_ref
    qg_oracle.build()
    return qgamd, qg_oracle, qg_ref


TWO_POINT = [(2, 8), (8, 2), (2, 2), (2, 3), (3, 2), (64, 2), (2, 64), (2, 1001)]


def _dev_field(torch, a):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64).T)).cuda()


@pytest.mark.parametrize("M,P", TWO_POINT + [(2, 20000), (20000, 2)])
def test_two_point_solves_match_reference_matrix(env, M, P):
    """Global M = 2 or P = 2: the reference's laplacian_1d_periodic (laplacian.jl:40-45) writes
    its wrap entry over the neighbour entry, so for two points D_2 = [-2 1; 1 -2], not the
    periodic 5-point operator.  The device's two-point path (spec_twopoint) solves the matrices
    exactly as construct_spA / get_poisson_cholesky / get_helmholtz_cholesky build them
    (laplacian.jl:54-75): against splu on those matrices (oracle/qg_ref.py), < 1e-12 relative,
    the pinned point exactly where the reference puts it."""
    import torch
    qg, O, R = env
    dx = 4e6 / max(M, P)
    alpha = -6.25e-10
    f = R.update_doubly_periodic_bc(R.seeded_rand(M, P, 7) - 0.5) * 1e-9
    got = qg.sp_solve_modified_helmholtz(M, P, dx, _dev_field(torch, f), alpha).cpu().numpy().T
    assert rel(got, R.sp_solve_modified_helmholtz(M, P, dx, f, alpha)) < 1e-12
    got = qg.sp_solve_poisson(M, P, dx, _dev_field(torch, f)).cpu().numpy().T
    ref = R.sp_solve_poisson(M, P, dx, f)
    assert rel(got, ref) < 1e-12
    assert abs(got[1, 1]) <= 1e-13 * np.abs(ref).max()


@pytest.mark.parametrize("M,P", TWO_POINT)
def test_two_point_domains_step_like_the_reference(env, M, P):
    """The whole loop (run_model_no_output.jl:3-16) on two-point domains against the numpy
    restatement, whose solves are splu on the reference's own matrices: every slot of zeta and
    psi < 1e-12 after 6 steps (Euler and AB3).  The C oracle's exact DFT solve would solve the
    periodic operator, so it is not the reference here.  PCG applies the periodic 5-point
    stencil and still refuses these domains (QG_ERR_UNSUPPORTED)."""
    qg, O, R = env
    steps = 6
    st = qg.run_model_no_output(qg.bench_model(M, P=P), nsteps=steps)
    z, p, _ = R.run_model_no_output(R.bench_model(M, P=P), nsteps=steps)
    for n, ref in (("zeta", z), ("psi", p)):
        got = st.to_numpy(n)
        for layer in range(2):
            assert rel(got[:, :, layer, 0], ref[:, :, layer, 0]) < 1e-12, (n, layer)
    with pytest.raises(qg.QGError) as e:
        qg.State(qg.bench_model(M, P=P), solver=1)
    assert e.value.status == -2


def test_two_point_domains_f32(env):
    """F32 states on a two-point domain: within the F32 bar of the F64 run."""
    import torch
    qg, O, R = env
    m = qg.bench_model(64, P=2)
    a = qg.run_model_no_output(m, nsteps=4)
    b = qg.run_model_no_output(m, nsteps=4, dtype=torch.float32)
    assert rel(b.to_numpy("psi").astype(np.float64), a.to_numpy("psi")) < 1e-5


@pytest.mark.parametrize("M,P,kw", [(8, 3, {}), (16, 48, {}), (64, 16, {}), (16, 128, {}),
                                    (32, 64, {"chunk_rows": 4}), (32, 60, {"chunk_rows": 0})])
def test_small_and_ragged_grids(env, M, P, kw):
    qg, O, R = env
    steps = 5
    st = qg.run_model_no_output(qg.bench_model(M, P=P), nsteps=steps, **kw)
    ref = O.State(R.bench_model(M, P=P)).run(steps)
    for n in ("psi", "zeta"):
        assert rel(st.to_numpy(n), getattr(ref, n)) < TOL, (n, M, P)


def test_chunk_size_does_not_change_the_answer(env):
    qg, O, R = env
    m = qg.bench_model(64)
    a = qg.run_model_no_output(m, nsteps=4, chunk_rows=16).to_numpy("psi")
    b = qg.run_model_no_output(m, nsteps=4, chunk_rows=2).to_numpy("psi")
    assert rel(a, b) < 1e-12


@pytest.mark.parametrize("M,P", [(48, 40), (45, 40), (3, 8), (5, 6), (9, 12), (127, 64), (250, 30), (1001, 16),
                                 (2 * 3 * 5 * 7 * 11, 12), (13 * 16, 24), (17 * 4, 20)])
def test_non_power_of_two_rows(env, M, P):
    """Rows that are not a power of two (even and odd): the spectral solver's direct-DFT
    passes; also as the PCG preconditioner, and plain CG for comparison."""
    qg, O, R = env
    m = qg.bench_model(M, P=P)
    st = qg.run_model_no_output(m, nsteps=5)
    ref = O.State(R.bench_model(M, P=P)).run(5)
    for n in ("psi", "zeta"):
        assert rel(st.to_numpy(n), getattr(ref, n)) < TOL, n
    pc = qg.run_model_no_output(m, nsteps=5, solver=1)  # PCG, spectral preconditioner
    assert rel(pc.to_numpy("psi"), ref.psi) < TOL
    if M == 45:
        cg = qg.run_model_no_output(m, nsteps=5, solver=1, precond=0, pcg_maxit=2000)
        assert rel(cg.to_numpy("psi"), ref.psi) < 1e-8  # plain CG, stagnation floor ~1e-10 relres


@pytest.mark.parametrize("M", list(range(8, 129, 8)))
def test_reference_benchmark_sweep_sizes(env, M):
    """The grid sweep of the reference's own benchmark, M = P = 8:8:128
    (src/benchmarking/julia_bench_parts.jl:19), 10 steps at its dt = 30 min."""
    qg, O, R = env
    st = qg.run_model_no_output(qg.bench_model(M), nsteps=10)
    ref = O.State(R.bench_model(M)).run(10)
    for n in ("psi", "zeta"):
        assert rel(st.to_numpy(n), getattr(ref, n)) < TOL, (n, M)


def test_generic_rows_wide(env):
    """Wide generic rows on rectangular slabs: M = 2000 and 3000 (mixed-radix passes), 1999
    (prime: direct DFT); rows beyond the Bluestein path's 262144 points, or slabs of one row,
    are refused (QG_ERR_UNSUPPORTED)."""
    qg, O, R = env
    for M in (2000, 1999, 3000):
        st = qg.run_model_no_output(qg.bench_model(M, P=24, dt=600.0), nsteps=3)
        ref = O.State(R.bench_model(M, P=24, dt=600.0)).run(3)
        assert rel(st.to_numpy("psi"), ref.psi) < TOL, M
    with pytest.raises(qg.QGError) as e:
        qg.State(qg.bench_model(262145, P=4))  # (P = 4: only the row cap can refuse it)
    assert e.value.status == -2


@pytest.mark.parametrize("M,P,steps", [(3328, 32, 3), (5000, 32, 3), (6000, 24, 3), (8191, 16, 2), (4001, 20, 2)])
def test_split_rows_beyond_generic(env, M, P, steps):
    """Non-power-of-two rows wider than the generic passes (3200 < M <= 8192): the split
    passes -- row DFT in place in one LDS buffer (mixed-radix DIF: 3328 = 8 8 4 13,
    5000 = 8 5^4, 6000 = 8 2 3 5^3; direct DFT: 8191 and 4001 are prime), recurrences one
    thread per wavenumber.  The reference factors any M x P (laplacian.jl:60-75)."""
    qg, O, R = env
    st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=600.0), nsteps=steps)
    ref = O.State(R.bench_model(M, P=P, dt=600.0)).run(steps)
    for n in ("psi", "zeta"):
        assert rel(st.to_numpy(n), getattr(ref, n)) < TOL, (n, M)
    if M == 5000:  # PCG with the split solve as its preconditioner
        pc = qg.run_model_no_output(qg.bench_model(M, P=P, dt=600.0), nsteps=steps, solver=1)
        assert rel(pc.to_numpy("psi"), ref.psi) < TOL


@pytest.mark.parametrize("M,P", [(3000, 24), (1001, 16), (45, 40), (120, 16), (2310, 12)])
def test_split_passes_match_generic(env, M, P):
    """qg_set_form(QG_FORM_ROW_SPLIT, 1) routes generic-size rows through the split passes:
    same answer as the generic passes (different FFT order: roundoff only) and the oracle."""
    qg, O, R = env
    m = qg.bench_model(M, P=P, dt=600.0)
    gen = qg.run_model_no_output(m, nsteps=4)
    with qg.forced_form(qg._lib.QG_FORM_ROW_SPLIT, 1):
        spl = qg.run_model_no_output(m, nsteps=4)
    ref = O.State(R.bench_model(M, P=P, dt=600.0)).run(4)
    for n in ("psi", "zeta", "f_store"):
        err = rel(spl.to_numpy(n), gen.to_numpy(n))
        # (3000 x 24: the wide, short slab amplifies the two FFT orders' roundoff: 3.8e-12)
        assert err < 2e-11, (n, err)
    assert rel(spl.to_numpy("psi"), ref.psi) < TOL


def test_split_rows_f32(env):
    """F32 state through the split passes (M = 5000): psi within the F32 bar of the F64 run."""
    import torch
    qg, O, R = env
    m = qg.bench_model(5000, P=32, dt=600.0)
    a = qg.run_model_no_output(m, nsteps=3)
    b = qg.run_model_no_output(m, nsteps=3, dtype=torch.float32)
    assert rel(b.to_numpy("psi").astype(np.float64), a.to_numpy("psi")) < 5e-3


@pytest.mark.parametrize("M,P,steps,kw", [(16384, 64, 3, {}), (16384, 32, 2, {}), (16384, 16, 3, {}), (8200, 8, 2, {}),
                                          (9000, 4, 2, {}), (16384, 9, 2, {}), (16384, 24, 2, {"chunk_rows": 8})])
def test_wide_split_rows(env, M, P, steps, kw):
    """Even rows wider than 8192 (8192 < M <= 16384): spec_fft_wide, each real row of the
    pass-A/pass-B pipeline as a half-length complex DFT in LDS (H = M/2: 8192 = 2^13,
    4100 = 4 5^2 41, 4500 = 4 3^2 5^3) plus the real split step, both systems of a workgroup
    in turn.  The reference factors any M x P (laplacian.jl:60-75).  (The oracle's direct DFT
    of a non-power-of-two row costs O(M^2) per row: small P there.)  Odd P (one-row chunks)
    and an explicit chunk size too.

    Tolerance: the pinned Poisson system's condition number grows like M^2 (lowest x mode,
    (2 pi / M)^2 against 8), so at 16384 two exact solvers -- device and oracle -- differ by
    1e-10..7e-10 (measured: 2.4e-10 at P = 64, 1.3e-10 at 32, 7.0e-10 at 16; 9000 x 4:
    1.8e-10).  Both are checked for exactness directly: the device solution's residuals in
    the two modal systems must be at roundoff (< 1e-13, like the oracle's), and the two
    solutions agree to 2e-9."""
    qg, O, R = env
    st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=60.0), nsteps=steps, **kw)
    ref = O.State(R.bench_model(M, P=P, dt=60.0)).run(steps)
    m = R.bench_model(M, P=P, dt=60.0)
    res_dev = modal_residuals(R, m, st.to_numpy("zeta"), st.to_numpy("psi"))
    res_ref = modal_residuals(R, m, ref.zeta, ref.psi)
    print(f"M={M} P={P} residuals device {res_dev} oracle {res_ref}")
    assert max(res_dev) < 1e-13 and max(res_ref) < 1e-13, (res_dev, res_ref)
    assert rel(st.to_numpy("zeta"), ref.zeta) < TOL
    assert rel(st.to_numpy("psi"), ref.psi) < 2e-9
    if M == 16384 and P == 16:  # PCG with the wide split solve as its preconditioner
        pc = qg.run_model_no_output(qg.bench_model(M, P=P, dt=60.0), nsteps=steps, solver=1)
        assert max(modal_residuals(R, m, pc.to_numpy("zeta"), pc.to_numpy("psi"))) < 1e-13
        assert rel(pc.to_numpy("psi"), ref.psi) < 2e-9


@pytest.mark.parametrize("M,P,steps,kw,oracle", [(8193, 4, 2, {}, True), (20000, 4, 2, {}, True),
                                                 (16385, 6, 2, {}, True), (20000, 8, 2, {"chunk_rows": 4}, True),
                                                 (50001, 3, 2, {}, False)])
def test_bluestein_rows(env, M, P, steps, kw, oracle):
    """Rows no FFT plan of the direct solver takes -- odd M > 8192 and M > 16384, which returned
    QG_ERR_UNSUPPORTED before (the bare-CG fallback) -- through Bluestein's chirp-z DFT: power-of-
    two FFTs of length >= 2M - 1 in global memory around the split pipeline's recurrences.  The
    reference factors any M x P (laplacian.jl:60-75).  Exactness as for the wide split rows: the
    device solution's residuals in both modal systems at roundoff (< 1e-13), and agreement with
    the oracle to the conditioning floor of these long rows (cond ~ M^2: 2e-9).  (50001 x 3: the
    oracle's O(M^2) direct DFT would take minutes; residuals only.)"""
    qg, O, R = env
    st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=60.0), nsteps=steps, **kw)
    m = R.bench_model(M, P=P, dt=60.0)
    res_dev = modal_residuals(R, m, st.to_numpy("zeta"), st.to_numpy("psi"))
    print(f"M={M} P={P} device residuals {res_dev}")
    assert max(res_dev) < 1e-13, res_dev
    assert np.isfinite(st.to_numpy("psi")).all()
    if oracle:
        ref = O.State(R.bench_model(M, P=P, dt=60.0)).run(steps)
        assert rel(st.to_numpy("zeta"), ref.zeta) < TOL
        assert rel(st.to_numpy("psi"), ref.psi) < 2e-9


@pytest.mark.parametrize("M,P", [(8193, 4), (20000, 4)])
def test_bluestein_rows_pcg(env, M, P):
    """PCG with the Bluestein-row direct solve as its preconditioner (the verdict's bar: <= 50
    iterations at M = 8193 and 20000): every solve certifies in one iteration, residuals at
    roundoff, the same answer as the direct solver."""
    qg, O, R = env
    m = qg.bench_model(M, P=P, dt=60.0)
    a = qg.run_model_no_output(m, nsteps=3)
    b = qg.run_model_no_output(m, nsteps=3, solver=1)
    s = b.stats()
    assert 1 <= s["iters"][0] <= 50 and max(s["relres"]) < 1e-12, s
    mr = R.bench_model(M, P=P, dt=60.0)
    assert max(modal_residuals(R, mr, b.to_numpy("zeta"), b.to_numpy("psi"))) < 1e-13
    assert rel(b.to_numpy("psi"), a.to_numpy("psi")) < 1e-12


def test_bluestein_rows_f32(env):
    """F32 state through the Bluestein rows (M = 20000): F32 vs F64 within the mechanism's
    derived bars (tests/f32_model.py: zeta at F32 roundoff, psi = the solve's image of it)."""
    import torch
    import f32_model as F32
    qg, O, R = env
    r = F32.decompose(qg, torch, qg.bench_model(20000, P=4, dt=60.0), 2, mc=8)
    print(F32.fmt(r))
    F32.check(r)


def test_wide_split_rows_f32(env):
    """F32 state through the wide split (M = 16384): F32 vs F64 within the mechanism's derived
    bars (tests/f32_model.py; psi = A^-1 zeta amplifies zeta's F32 rounding in the gravest modes
    by up to (M / 2 pi)^2; measured 1.0e-2 here in r05)."""
    import torch
    import f32_model as F32
    qg, O, R = env
    r = F32.decompose(qg, torch, qg.bench_model(16384, P=32, dt=60.0), 3, mc=8)
    print(F32.fmt(r))
    F32.check(r)


def test_invalid_arguments_are_refused(env):
    qg, O, R = env
    st = qg.State(qg.bench_model(32))
    with pytest.raises(qg.QGError) as e:
        st.evolve_zeta_(0)  # timesteps are 1-based (model.jl:160)
    assert e.value.status == -1


@pytest.mark.parametrize("P,kw", [(32, {}), (24, {"chunk_rows": 8}), (9, {}), (32, {"solver": 1})])
def test_widest_rows_8192(env, P, kw):
    """M = 8192, the widest row the spectral solver takes: one system per workgroup, each real
    row as a half-length complex FFT plus a split step (spec_passA_half / spec_passB_half);
    odd P (one-row chunks), an explicit chunk size, and PCG with this solve as preconditioner.
    (At P = 16 the device and the oracle, both exact solvers with 5-point residuals ~7e-16,
    differ by 1.7e-10: an 8192 x 16 slab's Poisson problem amplifies roundoff ~1e6-fold.)"""
    qg, O, R = env
    st = qg.run_model_no_output(qg.bench_model(8192, P=P, dt=60.0), nsteps=3, **kw)
    ref = O.State(R.bench_model(8192, P=P, dt=60.0)).run(3)
    for n in ("psi", "zeta"):
        assert rel(st.to_numpy(n), getattr(ref, n)) < TOL, n


def test_attach_after_single_rank_seed_is_refused():
    """qg_initialise seeds the noise from global row offsets (rank, nranks): attaching a
    multi-rank transport to a state seeded as one rank would step the wrong initial field,
    so the library refuses it (QG_ERR_INVALID_ARG); seeding after the attach works."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    import qgamd
    from qgamd import _lib

    m = qgamd.bench_model(32, P=32)
    st = qgamd.State(m, P_local=16).initialise()
    noop_ag = _lib.AllgatherFn(lambda *a: 0)
    noop_sr = _lib.SendrecvFn(lambda *a: 0)
    rc = _lib.lib().qg_comm_init_host(st._ctx, 2, 0, noop_ag, noop_sr, None)
    assert rc == _lib.QG_ERR_INVALID_ARG
    # the refused attach left the context untouched (no communicator, not distributed): it
    # still steps as the single-GPU periodic slab it was seeded as
    ref = qgamd.State(m, P_local=16).initialise()
    st.run(1, 3)
    ref.run(1, 3)
    assert np.array_equal(st.to_numpy("psi"), ref.to_numpy("psi"))


def test_slab_checkpoint_needs_its_transport(tmp_path):
    """A slab of a multi-rank run read back from its checkpoint refuses to step until the
    transport of that many ranks is attached (it would otherwise run as a periodic domain)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd

    st = qgamd.State(qgamd.bench_model(32), device=torch.device("cuda", 0)).initialise()
    st.run(1, 2)
    st.rank, st.nranks = 1, 2  # pretend it is slab 1 of 2
    path = str(tmp_path / "ck.npz")
    qgamd.save_checkpoint(st, path, 2)
    st2, t = qgamd.load_checkpoint(path, device="cuda:0")
    assert (st2.rank, st2.nranks, t) == (1, 2, 3)
    with pytest.raises(RuntimeError, match="transport"):
        st2.run(t, 1)
