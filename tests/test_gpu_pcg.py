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
