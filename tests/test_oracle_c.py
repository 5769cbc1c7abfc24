"""Pin the C oracle (oracle/qg_oracle.c) to the scipy restatement (oracle/qg_ref.py).

The stencils must agree bit for bit (same evaluation order, no FMA contraction); the
exact-DFT solve must agree with the sparse direct solve of the same matrices to roundoff.
"""
import numpy as np
import pytest

from oracle import qg_oracle as O
from oracle import qg_ref as R


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _rand(M, P, seed):
    return R.update_doubly_periodic_bc(R.seeded_rand(M, P, seed) - 0.5)


@pytest.mark.parametrize("M,P", [(8, 8), (16, 12), (10, 5), (33, 17)])
def test_stencils_bitwise(M, P):
    dx = 4e6 / M
    z, p = _rand(M, P, 1), _rand(M, P, 2)
    assert np.array_equal(O.laplace_5p(p, dx), R.laplace_5p(p, dx))
    assert np.array_equal(O.cd(p, dx), R.cd(p, dx))
    assert np.array_equal(O.J(dx, z, p), R.J(dx, z, p))


@pytest.mark.parametrize("M,P,alpha,pinned", [(16, 16, 0.0, True), (32, 16, -6.25e-10, False),
                                              (10, 5, -1e-10, False), (12, 20, 0.0, True)])
def test_solve_matches_sparse_direct(M, P, alpha, pinned):
    dx = 4e6 / M
    f = _rand(M, P, 7) * 1e-9
    got = O.solve(M, P, dx, alpha, f, pinned=pinned)
    if pinned:
        ref = R.sp_solve_poisson(M, P, dx, f)
    else:
        ref = R.sp_solve_modified_helmholtz(M, P, dx, f, alpha)
    assert np.max(np.abs(got - ref)) <= 1e-11 * np.max(np.abs(ref))
    if pinned:
        assert abs(got[1, 1]) < 1e-14 * np.max(np.abs(ref))


@pytest.mark.parametrize("N,steps", [(16, 5), (32, 12)])
def test_run_matches_scipy_oracle(N, steps):
    m = R.bench_model(N)
    z_ref, p_ref, f_ref = R.run_model_no_output(m, nsteps=steps)
    st = O.State(m).run(steps)
    # stencil path is bitwise; the solve differs at roundoff and feeds back into zeta
    for a, b in ((st.psi, p_ref), (st.zeta, z_ref), (st.f_store, f_ref)):
        err = np.linalg.norm(a - b) / np.linalg.norm(b)
        assert err < 1e-12, err


def test_run_with_physical_projection_matches_scipy_oracle():
    """The P_fwd = P_matrix(H_1, H_2) option in the C oracle against the
    literal restatement's evolve_psi(..., P_fwd=...)."""
    m = R.bench_model(32)
    Pf = R.P_matrix(m.H_1, m.H_2)
    zeta, psi = R.initialise_model(m)
    pc = R.get_poisson_cholesky(m.M, m.P, m.dx)
    hc = R.get_helmholtz_cholesky(m.M, m.P, m.dx, R.S_eig(m))
    f = np.zeros((m.M + 2, m.P + 2, 2, 3))
    for t in range(1, 11):
        R.evolve_zeta(m, zeta, psi, t, f)
        R.evolve_psi(m, zeta, psi, pc, hc, P_fwd=Pf)
    st = O.State(m, P_fwd=Pf).run(10)
    assert np.linalg.norm(st.psi - psi) / np.linalg.norm(psi) < 1e-12


def test_diagnostics_definitions():
    """oracle diagnostics (qg_diagnostics' checker) on fields with known values."""
    M = P = 16
    dx = 2.0
    z = np.zeros((M + 2, P + 2, 2, 3))
    p = np.zeros_like(z)
    x = np.arange(M) * 2 * np.pi / M
    p[1:-1, 1:-1, 0, 0] = np.sin(x)[:, None]            # psi_1 = sin(2 pi i / M)
    p[:, :, 0, 0] = R.update_doubly_periodic_bc(p[:, :, 0, 0])
    z[1:-1, 1:-1, 1, 0] = 3.0
    z[:, :, 1, 0] = R.update_doubly_periodic_bc(z[:, :, 1, 0])
    d = R.diagnostics(z, p, dx)
    assert d["zeta_max"] == [0.0, 3.0] and d["zeta_min"] == [0.0, 3.0]
    assert d["zeta_sum"][1] == 3.0 * M * P * dx * dx
    assert d["enstrophy"][1] == 0.5 * 9.0 * M * P * dx * dx
    # sum_i (sin(x+h) - sin x)^2 = 2 M sin^2(h/2) ... per row, P rows
    h = 2 * np.pi / M
    assert np.isclose(d["energy"][0], 0.5 * P * M * 4 * np.sin(h / 2) ** 2 / 2, rtol=1e-13)
    assert d["energy"][1] == 0.0
    assert np.isclose(d["interface"], 0.5 * P * (M / 2) * dx * dx, rtol=1e-13)
    assert R.update_max(5.0, p[:, :, 0, 0]) == 5.0 and R.update_max(0.5, p[:, :, 0, 0]) == 1.0
    assert R.update_min(5.0, p[:, :, 0, 0]) == -1.0 and R.update_min(-2.0, p[:, :, 0, 0]) == -2.0


def test_initial_conditions_bitwise():
    m = R.bench_model(24, P=16)
    z, p = R.initialise_model(m)
    st = O.State(m)
    assert np.array_equal(st.zeta, z) and np.array_equal(st.psi, p)


def test_wind_forcing_extension_term():
    """The wind-forcing extension (not in the reference; include/qg_mi355.h qg_params.wind_*):
    after one Euler step the upper layer's tendency differs from the unforced one by
    w_j = -(2 pi tau0 / (rho0 H_1 P dx)) sin(2 pi (j + 1/2) / P) on every interior row j
    (ghost rows: their periodic images), and the lower layer is untouched."""
    M, P, tau0, rho0 = 32, 24, 0.1, 1000.0
    m = R.bench_model(M, P=P)
    a = O.State(m).run(1)
    b = O.State(m, wind=(tau0, rho0)).run(1)
    d = b.f_store[:, :, 0, 0] - a.f_store[:, :, 0, 0]
    j = (np.arange(P + 2) - 1) % P
    w = -(2 * np.pi * tau0 / (rho0 * m.H_1 * (P * m.dx))) * np.sin(2 * np.pi * (j + 0.5) / P)
    scale = np.abs(a.f_store[:, :, 0, 0]).max()
    np.testing.assert_allclose(d, np.broadcast_to(w, d.shape), rtol=0, atol=1e-14 * np.abs(w).max() + 4e-16 * scale)
    assert np.array_equal(b.f_store[:, :, 1, 0], a.f_store[:, :, 1, 0])
    assert np.abs(w).max() > 0


@pytest.mark.parametrize("M,P,alpha,pinned", [(16, 16, 0.0, True), (12, 20, 0.0, True), (32, 16, -6.25e-10, False),
                                              (9, 30, -1e-10, False)])
def test_longdouble_solve_matches_sparse_direct(M, P, alpha, pinned):
    """The extended-precision solve (qg_ref.solve_longdouble) solves the reference's own
    matrices (splu on construct_spA / get_poisson_cholesky): agreement to F64 roundoff."""
    dx = 4e6 / M
    f = _rand(M, P, 9) * 1e-9
    got = np.asarray(R.solve_longdouble(M, P, dx, alpha, f, pinned=pinned), dtype=np.float64)
    ref = R.sp_solve_poisson(M, P, dx, f) if pinned else R.sp_solve_modified_helmholtz(M, P, dx, f, alpha)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-12


@pytest.mark.parametrize("M,P", [(64, 16384), (256, 8192), (512, 512)])
def test_c_oracle_solve_against_longdouble_on_long_grids(M, P):
    """The C oracle's DFT solve against the long-double solve on long domains, where the
    pinned Poisson problem's gravest modes have eigenvalues ~ (2 pi / P)^2: relative error
    < 1e-11 (measured 1.0e-12 at 64 x 16384).  Round 6 replaced its eigenvalue expression
    2 cos(t) + 2 cos(s) - 4 by -4 (sin^2(t/2) + sin^2(s/2)): the old form lost those
    eigenvalues to cancellation (7.5e-10 at 64 x 16384, 2.0e-9 at 256 x 32768), which was the
    larger part of the device-vs-oracle differences on long grids."""
    dx = 4e6 / M
    f = _rand(M, P, 17) * 1e-9
    for alpha, pinned in ((0.0, True), (-6.25e-10, False)):
        x = R.solve_longdouble(M, P, dx, alpha, f, pinned=pinned)
        got = O.solve(M, P, dx, alpha, f, pinned=pinned)
        e = float(np.linalg.norm((got - x)[1:-1, 1:-1]) / np.linalg.norm(x[1:-1, 1:-1]))
        assert e < 1e-11, (M, P, pinned, e)
