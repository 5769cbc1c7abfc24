"""The multigrid preconditioner's design on the CPU (tests/mg_model.py, a numpy restatement of
csrc/qg_mg.hip and its PCG): the V-cycle is symmetric positive definite, PCG's iteration count
does not grow with the grid, the slab form (ghost-row copies, gathered coarse grid) is the
global cycle, and the PCG solution is the direct solve of the reference's matrices.  The GPU
counterpart is tests/test_gpu_mg.py (device vs C oracle; 10 iterations there, 11 here on
random right-hand sides)."""
import numpy as np
import pytest

import mg_model as MG

S_HELM = -6.25e-10  # a modified-Helmholtz alpha of the benchmark's size (model.jl: -S_eig)


def _rhs(N, seed=1):
    return np.random.default_rng(seed).standard_normal((N, N))


@pytest.mark.parametrize("al", [0.0, S_HELM])
def test_vcycle_is_symmetric_positive_definite(al):
    """(u, V w) = (V u, w) and (u, V u) > 0 on random vectors: the cycle is a valid PCG
    preconditioner (R = c P^T, the same smoother before and after)."""
    N, dx = 32, 4e6 / 32
    rng = np.random.default_rng(3)
    for G in (1, 2):
        u, w = rng.standard_normal((N, N)), rng.standard_normal((N, N))
        Vu, Vw = MG.vcycle(u, dx, al, G), MG.vcycle(w, dx, al, G)
        a, b = float((u * Vw).sum()), float((Vu * w).sum())
        assert abs(a - b) <= 1e-12 * max(abs(a), abs(b)), (G, a, b)
        assert float((u * Vu).sum()) > 0


def test_iterations_do_not_grow_with_the_grid():
    """Pinned Poisson and modified Helmholtz at 32^2 ... 256^2 to a 1e-13 residual: at most 12
    iterations, the count settled by 128^2 (10 on the device at 256^2 ... 4096^2,
    tests/test_gpu_mg.py)."""
    its = {}
    for N in (32, 64, 128, 256):
        dx = 4e6 / N
        for al, pinned in ((0.0, True), (S_HELM, False)):
            _, it, hist = MG.pcg(_rhs(N), dx, al, pinned)
            assert hist[-1] <= 1e-13
            its.setdefault((al, pinned), []).append(it)
    for k, v in its.items():  # (Helmholtz: fewer at coarse grids, where alpha dx^2 dominates)
        assert max(v) <= 12 and abs(v[-1] - v[-2]) <= 1, (k, v)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_slab_cycle_is_the_global_cycle(G):
    """The slab form (each rank's rows, ghost rows from the ring neighbours before every
    stencil, the gathered global grid below AGG_POINTS per rank) equals the global cycle to
    roundoff, so the iteration count does not depend on the number of slabs."""
    N, dx = 128, 4e6 / 128
    r = _rhs(N, 5)
    for al in (0.0, S_HELM):
        a, b = MG.vcycle(r, dx, al, 1), MG.vcycle(r, dx, al, G)
        assert np.linalg.norm(a - b) <= 1e-13 * np.linalg.norm(a), (G, al)
    _, it1, _ = MG.pcg(_rhs(N), dx, 0.0, True, 1)
    _, itG, _ = MG.pcg(_rhs(N), dx, 0.0, True, G)
    assert it1 == itG


def test_pin_shift_removes_the_constant_mode():
    """Without T^T V T (the V-cycle applied to r directly) the pinned Poisson PCG needs more
    iterations: the periodic cycle's near-null constant mode; with it, the solution is the
    direct solve of the reference's pinned matrix."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl

    N, dx = 32, 4e6 / 32
    b = _rhs(N, 7)
    x, it, _ = MG.pcg(b, dx, 0.0, True)
    # the reference's pinned periodic 5-point matrix (laplacian.jl:54-75), negated
    n = N * N
    idx = np.arange(n).reshape(N, N)
    rows, cols, vals = [], [], []
    for j in range(N):
        for i in range(N):
            k = idx[j, i]
            if k == 0:
                rows.append(k), cols.append(k), vals.append(1.0)
                continue
            rows.append(k), cols.append(k), vals.append(4.0 / dx ** 2)
            for jj, ii in ((j, i - 1), (j, i + 1), (j - 1, i), (j + 1, i)):
                kk = idx[jj % N, ii % N]
                if kk != 0:
                    rows.append(k), cols.append(kk), vals.append(-1.0 / dx ** 2)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    bb = b.copy()
    bb[0, 0] = 0
    ref = spl.spsolve(A.tocsc(), bb.reshape(-1)).reshape(N, N)
    assert np.linalg.norm(x - ref) <= 1e-10 * np.linalg.norm(ref)
    # the unshifted form, for contrast
    saved = MG.precond

    def plain(r, dx_, al, pinned, G=1):
        return MG.vcycle(r, dx_, al, G)

    MG.precond = plain
    try:
        _, it_plain, _ = MG.pcg(b, dx, 0.0, True)
    finally:
        MG.precond = saved
    assert it_plain > it, (it_plain, it)
