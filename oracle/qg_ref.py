"""CPU ORACLE -- test infrastructure only, never part of the product path.

A literal numpy/scipy restatement of the reference's hot path
(JSLeadbetter/julia-ocean-modelling @ 2024-10-08).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker.

Conventions follow the reference exactly:

* fields are ``(M+2, P+2)`` Float64 arrays indexed ``[i, j]`` (i = x, first index,
  contiguous in Julia's column-major storage) with a one-cell ghost ring;
* state arrays are ``(M+2, P+2, 2 layers, 3 history slots)``; slot 0 is the newest
  (Julia slot 1);
* every stencil allocates its output, fills the interior, then refreshes the ghosts
  (``update_doubly_periodic_bc!``);
* floating-point evaluation order mirrors the Julia expressions term by term, so the
  stencils here are bit-identical to a loop-by-loop transcription.

The only substitution is the linear solver: the reference factorises the Poisson and
Helmholtz matrices with SuiteSparse CHOLMOD (``laplacian.jl:60-75``, solved at
``model.jl:186,191``).  CHOLMOD is not available here, so the *same* sparse matrices
(built exactly as ``construct_spA`` builds them, including the pinned first row/column of
the Poisson system) are factorised by SuperLU (``scipy.sparse.linalg.splu``).  Any exact
factorisation of the same SPD system agrees to roundoff.

Parity pin: ``tests/test_oracle_kat.py`` checks this module against every known answer
the reference itself holds (``src/test.jl`` testsets and the convergence slopes printed
in ``notebooks/jupyter/scheme_validation.ipynb``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

# model.jl:7-10
MINUTES = 60
DAY = 60 * 60 * 24
KM = 1000.0
YEAR = 60 * 60 * 24 * 365


# ---------------------------------------------------------------------------
# Parameters (model.jl:12-34, 109-121)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class BaroclinicModel:
    """Mirror of ``struct BaroclinicModel`` (model.jl:12-30)."""

    H_1: float
    H_2: float
    H: float
    beta: float
    Lx: float
    Ly: float
    dt: float
    T: float
    U: float
    M: int
    P: int
    dx: float
    visc: float
    r: float
    R_d: float
    initial_kick: float


def make_model(H_1, H_2, beta, Lx, Ly, dt, T, U, M, P, dx, visc, r, R_d, initial_kick):
    """Outer constructor (model.jl:33-34): H = H_1 + H_2."""
    return BaroclinicModel(float(H_1), float(H_2), float(H_1) + float(H_2), float(beta),
                           float(Lx), float(Ly), float(dt), float(T), float(U), int(M),
                           int(P), float(dx), float(visc), float(r), float(R_d),
                           float(initial_kick))


def ratio_term(m):  # model.jl:109-111
    return 0.5 * (m.H_1 + m.H_2) / ((m.R_d * m.R_d) * ((1 / m.H_1) + (1 / m.H_2)))


def S1_plus(m):  # model.jl:113
    return (2 * ratio_term(m)) / (m.H_1 * (m.H_1 + m.H_2))


def S2_minus(m):  # model.jl:114
    return (2 * ratio_term(m)) / (m.H_2 * (m.H_1 + m.H_2))


def beta_1(m):  # model.jl:117
    return m.beta + (S1_plus(m) * m.U)


def beta_2(m):  # model.jl:118
    return m.beta - (S2_minus(m) * m.U)


def S_eig(m):  # model.jl:121
    return -1 / (m.R_d * m.R_d)


def P_matrix(H_1, H_2):  # model.jl:83-87
    P = np.ones((2, 2))
    P[0, 1] = -H_2 / H_1
    return P


def P_inv_matrix(m):  # model.jl:90-99
    a = S1_plus(m)
    b = S2_minus(m)
    P = np.array([[b, a], [-b, b]])
    return (1 / (a + b)) * P


# ---------------------------------------------------------------------------
# Ghost ring (boundary_conditions.jl)
# ---------------------------------------------------------------------------
def update_doubly_periodic_bc(b):
    """boundary_conditions.jl:2-13 -- edges exclude corners, corners copied diagonally."""
    b[1:-1, 0] = b[1:-1, -2]
    b[1:-1, -1] = b[1:-1, 1]
    b[0, 1:-1] = b[-2, 1:-1]
    b[-1, 1:-1] = b[1, 1:-1]
    b[0, 0] = b[-2, -2]
    b[0, -1] = b[-2, 1]
    b[-1, -1] = b[1, 1]
    b[-1, 0] = b[1, -2]
    return b


def add_doubly_periodic_boundaries(u):  # boundary_conditions.jl:16-22
    M, P = u.shape
    e = np.zeros((M + 2, P + 2))
    e[1:-1, 1:-1] = u
    return update_doubly_periodic_bc(e)


# ---------------------------------------------------------------------------
# Stencils
# ---------------------------------------------------------------------------
def _dxm2(dx):
    # Julia literal_pow: dx^-2 == inv(dx)*inv(dx)
    i = 1.0 / dx
    return i * i


def laplace_5p(u, dx):
    """laplacian.jl:15-27: (u[i-1,j] + u[i+1,j] - 4u[i,j] + u[i,j-1] + u[i,j+1]) * dx^-2."""
    lap = np.zeros_like(u)
    lap[1:-1, 1:-1] = ((((u[:-2, 1:-1] + u[2:, 1:-1]) - 4 * u[1:-1, 1:-1]) + u[1:-1, :-2])
                       + u[1:-1, 2:]) * _dxm2(dx)
    return update_doubly_periodic_bc(lap)


def cd(u, dx):
    """model.jl:68-80: 0.5dx^-1 * (u[i+1,j] - u[i-1,j])."""
    out = np.zeros_like(u)
    out[1:-1, 1:-1] = (0.5 * (1.0 / dx)) * (u[2:, 1:-1] - u[:-2, 1:-1])
    return update_doubly_periodic_bc(out)


def _sh(a, di, dj):
    """Interior view of a shifted by (di, dj): a[i+di, j+dj] over the interior."""
    M2, P2 = a.shape
    return a[1 + di:M2 - 1 + di, 1 + dj:P2 - 1 + dj]


def j_pp(z, p):  # arakawa.jl:7-20
    return ((_sh(z, 1, 0) - _sh(z, -1, 0)) * (_sh(p, 0, 1) - _sh(p, 0, -1))
            - (_sh(z, 0, 1) - _sh(z, 0, -1)) * (_sh(p, 1, 0) - _sh(p, -1, 0)))


def j_pt(z, p):  # arakawa.jl:22-38
    return (((_sh(z, 1, 0) * (_sh(p, 1, 1) - _sh(p, 1, -1))
              - _sh(z, -1, 0) * (_sh(p, -1, 1) - _sh(p, -1, -1)))
             - _sh(z, 0, 1) * (_sh(p, 1, 1) - _sh(p, -1, 1)))
            + _sh(z, 0, -1) * (_sh(p, 1, -1) - _sh(p, -1, -1)))


def j_tp(z, p):  # arakawa.jl:40-56
    return (((_sh(z, 1, 1) * (_sh(p, 0, 1) - _sh(p, 1, 0))
              - _sh(z, -1, -1) * (_sh(p, -1, 0) - _sh(p, 0, -1)))
             - _sh(z, -1, 1) * (_sh(p, 0, 1) - _sh(p, -1, 0)))
            + _sh(z, 1, -1) * (_sh(p, 1, 0) - _sh(p, 0, -1)))


def J(dx, zeta, psi):
    """arakawa.jl:58-62: (j_pp + j_pt + j_tp) / (3*4*dx^2), then ghost fill.

    The sub-Jacobians are zero on the ghost ring (they are allocated with ``zeros``), so
    the division leaves ghost values at 0 before the refresh -- identical to the loop.
    """
    out = np.zeros_like(zeta)
    out[1:-1, 1:-1] = ((j_pp(zeta, psi) + j_pt(zeta, psi)) + j_tp(zeta, psi)) / (12 * (dx * dx))
    return update_doubly_periodic_bc(out)


# ---------------------------------------------------------------------------
# Sparse operators and solves (laplacian.jl:30-111)
# ---------------------------------------------------------------------------
def laplacian_1d(N):  # laplacian.jl:30-32
    return sp.diags([np.ones(N - 1), -2 * np.ones(N), np.ones(N - 1)], [-1, 0, 1], format="lil")


def laplacian_2d(M, P):  # laplacian.jl:34-38
    return (sp.kron(sp.identity(P), laplacian_1d(M)) + sp.kron(laplacian_1d(P), sp.identity(M))).tocsc()


def laplacian_1d_periodic(N):  # laplacian.jl:40-45
    lap = laplacian_1d(N)
    lap[0, N - 1] = 1
    lap[N - 1, 0] = 1
    return lap.tocsc()


def laplacian_2d_doubly_periodic(M, P):  # laplacian.jl:47-51
    Dx = laplacian_1d_periodic(M)
    Dy = laplacian_1d_periodic(P)
    return (sp.kron(sp.identity(P), Dx) + sp.kron(Dy, sp.identity(M))).tocsc()


def construct_spA(M, P, dx, alpha):  # laplacian.jl:54-58
    A = laplacian_2d_doubly_periodic(M, P)
    A = A + (alpha * (dx * dx)) * sp.identity(M * P)
    return (_dxm2(dx) * A).tocsc()


class _Factor:
    """Stands in for SparseArrays.CHOLMOD.Factor: ``F.solve(b)`` == ``F \\ b``."""

    def __init__(self, A):
        self.A = A.tocsc()
        self._lu = spla.splu(self.A)

    def solve(self, b):
        return self._lu.solve(np.asarray(b, dtype=np.float64))


def _pin_first(A):
    """A[:,1] .= 0; A[1,:] .= 0; A[1,1] = 1  (laplacian.jl:71-73)."""
    A = A.tolil()
    A[:, 0] = 0
    A[0, :] = 0
    A[0, 0] = 1
    return A.tocsc()


def get_helmholtz_cholesky(M, P, dx, alpha):  # laplacian.jl:60-64
    return _Factor(-construct_spA(M, P, dx, alpha))


def get_poisson_cholesky(M, P, dx):  # laplacian.jl:66-75
    return _Factor(_pin_first(-construct_spA(M, P, dx, 0.0)))


def solve_longdouble(M, P, dx, alpha, f, pinned=False, workers=None):
    """Extended-precision reference solve (x86 80-bit long double, eps = 5.4e-20) of the same
    systems: construct_spA(M, P, dx, alpha) x = f over the interior of the (M+2, P+2) field f
    (laplacian.jl:54-58, M, P >= 3), or with ``pinned`` the pinned Poisson system of
    get_poisson_cholesky (laplacian.jl:66-75, b[1] = 0 as model.jl:185): the compatible
    right-hand side f - sum(f) e_1, the mean-free DFT solve, minus its value at point 1 --
    the pinned solution exactly (the pin drops only the first equation).  2-D DFT by
    scipy.fft in long double, eigenvalues -4 dx^-2 (sin^2(pi kx / M) + sin^2(pi ky / P)) +
    alpha in the cancellation-free form.  Not an F64 solver: it measures how far each F64
    solver (the C oracle, the device) is from the exact solution of the F64 input, so that
    the difference between two of them can be attributed."""
    import scipy.fft as sfft
    ld = np.longdouble
    g = np.asarray(f, dtype=np.float64)[1:-1, 1:-1].astype(ld)
    if pinned:
        g[0, 0] -= np.sum(g)  # (pairwise summation in long double)
    G = sfft.fft2(g, workers=workers)
    del g
    pi = ld("3.14159265358979323846264338327950288")
    sx = np.sin(pi * np.arange(M, dtype=ld) / ld(M)) ** 2
    sy = np.sin(pi * np.arange(P, dtype=ld) / ld(P)) ** 2
    lam = (ld(-4) / (ld(dx) * ld(dx))) * (sx[:, None] + sy[None, :]) + ld(alpha)
    if pinned:
        lam[0, 0] = 1
        G[0, 0] = 0
    G /= lam
    del lam
    x = sfft.ifft2(G, workers=workers).real
    del G
    if pinned:
        x -= x[0, 0]
    out = np.zeros((M + 2, P + 2), dtype=ld)
    out[1:-1, 1:-1] = x
    return update_doubly_periodic_bc(out)


def _vec(a):
    """Julia vec: column-major flatten (i fastest)."""
    return np.asarray(a).flatten(order="F")


def _unvec(v, M, P):
    return np.asarray(v).reshape((M, P), order="F")


def sp_solve_modified_helmholtz(M, P, dx, f, alpha):  # laplacian.jl:78-86
    chol = get_helmholtz_cholesky(M, P, dx, alpha)
    b = -_vec(f[1:-1, 1:-1])
    return add_doubly_periodic_boundaries(_unvec(chol.solve(b), M, P))


def sp_solve_modified_helmholtz_fn(M, P, dx, f_rhs, alpha, domain):  # laplacian.jl:89-98
    x1, x2, y1, y2 = domain
    xs = np.linspace(x1 - dx, x2, M + 2)
    ys = np.linspace(y1 - dx, y2, P + 2)
    b = inflate(f_rhs, xs, ys)
    return sp_solve_modified_helmholtz(M, P, dx, b, alpha)


def sp_solve_poisson(M, P, dx, f):  # laplacian.jl:100-111
    chol = get_poisson_cholesky(M, P, dx)
    b = -_vec(f[1:-1, 1:-1])
    b[0] = 0
    return add_doubly_periodic_boundaries(_unvec(chol.solve(b), M, P))


def inflate(f, xs, ys):
    """inflate(f, xs, ys) = [f(x,y) for x in xs, y in ys] (laplacian.jl:94)."""
    X, Y = np.meshgrid(np.asarray(xs, dtype=np.float64), np.asarray(ys, dtype=np.float64),
                       indexing="ij")
    return np.asarray(f(X, Y), dtype=np.float64)


def julia_range(start, stop, length):
    """Julia ``range(start, stop, length=n)`` (a StepRangeLen with TwicePrecision).

    Julia computes element k as ``start + (k-1)*step`` in double-double arithmetic and
    rounds once; ``numpy.linspace`` computes ``start + k*step`` with a rounded step.  The
    two can differ in the last bit; evaluate in long double to get Julia's rounding.
    """
    n = int(length)
    k = np.arange(n, dtype=np.longdouble)
    s = np.longdouble(start)
    e = np.longdouble(stop)
    v = s + k * ((e - s) / np.longdouble(n - 1))
    return v.astype(np.float64)


# ---------------------------------------------------------------------------
# Seeded initial conditions (the reference's rand() is unseeded: model.jl:41-42)
# ---------------------------------------------------------------------------
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
SEED_LAYER1 = 20241008
SEED_LAYER2 = 20241009


def splitmix64_u01(seed, k):
    """Counter-based uniform in [0,1): mix64(seed + (k+1)*golden) >> 11 * 2^-53.

    The identical function is implemented in the HIP library (device-side
    ``qg_initialise``) and in ``qg_oracle.c``.
    """
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + (np.asarray(k, dtype=np.uint64) + np.uint64(1)) * GOLDEN
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def seeded_rand(M, P, seed, j_offset=0, M_total=None):
    """(M+2, P+2) array whose interior (i, j) is u01(seed, i + M*(j + j_offset)).

    Ghosts are left 0; ``initialise_model`` overwrites them (model.jl:44-45).
    """
    Mt = M if M_total is None else M_total
    i = np.arange(M, dtype=np.uint64)[:, None]
    j = np.arange(P, dtype=np.uint64)[None, :] + np.uint64(j_offset)
    out = np.zeros((M + 2, P + 2))
    out[1:-1, 1:-1] = splitmix64_u01(seed, i + np.uint64(Mt) * j)
    return out


def initialise_model(m, seeds=(SEED_LAYER1, SEED_LAYER2), rand_fields=None):
    """model.jl:37-62 with seeded noise in place of rand()."""
    assert np.sign(beta_1(m)) == -np.sign(beta_2(m))  # model.jl:38
    if rand_fields is None:
        rand_fields = (seeded_rand(m.M, m.P, seeds[0]), seeded_rand(m.M, m.P, seeds[1]))
    amp = m.initial_kick * m.U * m.Ly
    psi_1 = amp * rand_fields[0]
    psi_2 = amp * rand_fields[1]
    update_doubly_periodic_bc(psi_1)
    update_doubly_periodic_bc(psi_2)
    zeta_1 = laplace_5p(psi_1, m.dx) + S1_plus(m) * (psi_2 - psi_1)
    zeta_2 = laplace_5p(psi_2, m.dx) + S2_minus(m) * (psi_1 - psi_2)
    update_doubly_periodic_bc(zeta_1)
    update_doubly_periodic_bc(zeta_2)
    zeta = np.zeros((m.M + 2, m.P + 2, 2, 3))
    psi = np.zeros((m.M + 2, m.P + 2, 2, 3))
    psi[:, :, 0, 0] = psi_1
    psi[:, :, 1, 0] = psi_2
    zeta[:, :, 0, 0] = zeta_1
    zeta[:, :, 1, 0] = zeta_2
    return zeta, psi


# ---------------------------------------------------------------------------
# Time stepping (model.jl:101-199)
# ---------------------------------------------------------------------------
def store_new_state(arr, new_state, z):  # model.jl:102-106
    arr[:, :, z, 2] = arr[:, :, z, 1]
    arr[:, :, z, 1] = arr[:, :, z, 0]
    arr[:, :, z, 0] = new_state


def zeta_f1(m, zeta, psi):  # model.jl:139-145
    v_term = m.visc * laplace_5p(laplace_5p(psi, m.dx), m.dx)
    J_term = J(m.dx, zeta, psi)
    beta_term = beta_1(m) * cd(psi, m.dx)
    U_term = m.U * cd(zeta, m.dx)
    return ((v_term - J_term) - beta_term) - U_term


def zeta_f2(m, zeta, psi):  # model.jl:147-153
    v_term = m.visc * laplace_5p(laplace_5p(psi, m.dx), m.dx)
    J_term = J(m.dx, zeta, psi)
    beta_term = beta_2(m) * cd(psi, m.dx)
    r_term = m.r * laplace_5p(psi, m.dx)
    return ((v_term - J_term) - beta_term) - r_term


def eulers_method(m, f, zeta, psi, z, f_store):  # model.jl:123-127
    f1 = f(m, zeta[:, :, z, 0].copy(), psi[:, :, z, 0].copy())
    store_new_state(f_store, f1, z)
    return zeta[:, :, z, 0] + (m.dt * f1)


def AB3(m, f, zeta, psi, z, f_store):  # model.jl:129-136
    f1 = f(m, zeta[:, :, z, 0].copy(), psi[:, :, z, 0].copy())
    store_new_state(f_store, f1, z)
    f2 = f_store[:, :, z, 1]
    f3 = f_store[:, :, z, 2]
    update = m.dt * (((23 / 12) * f1 - (16 / 12) * f2) + (5 / 12) * f3)
    return zeta[:, :, z, 0] + update


def evolve_zeta_layer(m, zeta, psi, timestep, layer, f, f_store):  # model.jl:160-170
    if timestep == 1 or timestep == 2:
        new_zeta = eulers_method(m, f, zeta, psi, layer, f_store)
    else:
        new_zeta = AB3(m, f, zeta, psi, layer, f_store)
    store_new_state(zeta, new_zeta, layer)


def evolve_zeta(m, zeta, psi, timestep, f_store):  # model.jl:155-158
    evolve_zeta_layer(m, zeta, psi, timestep, 0, zeta_f1, f_store)
    evolve_zeta_layer(m, zeta, psi, timestep, 1, zeta_f2, f_store)


def evolve_psi(m, zeta, psi, poisson_chol, helmholtz_chol, P_fwd=None):  # model.jl:172-199
    """``P_fwd`` defaults to the reference's ``P_matrix(H_1, H_1)`` (model.jl:173)."""
    Pm = P_matrix(m.H_1, m.H_1) if P_fwd is None else np.asarray(P_fwd)
    P_inv = P_inv_matrix(m)
    zeta_tilde = np.zeros((m.M + 2, m.P + 2, 2))
    for i in range(2):
        zeta_tilde[:, :, i] = P_inv[i, 0] * zeta[:, :, 0, 0] + P_inv[i, 1] * zeta[:, :, 1, 0]
    b = -_vec(zeta_tilde[1:-1, 1:-1, 0])
    b[0] = 0
    npt1 = add_doubly_periodic_boundaries(_unvec(poisson_chol.solve(b), m.M, m.P))
    b = -_vec(zeta_tilde[1:-1, 1:-1, 1])
    npt2 = add_doubly_periodic_boundaries(_unvec(helmholtz_chol.solve(b), m.M, m.P))
    for i in range(2):
        new_psi = Pm[i, 0] * npt1 + Pm[i, 1] * npt2
        store_new_state(psi, new_psi, i)


def run_model_no_output(m, nsteps=None, seeds=(SEED_LAYER1, SEED_LAYER2), callback=None):
    """run_model_no_output.jl:3-16 (``nsteps`` overrides floor(T/dt) for tests)."""
    zeta, psi = initialise_model(m, seeds)
    pc = get_poisson_cholesky(m.M, m.P, m.dx)
    hc = get_helmholtz_cholesky(m.M, m.P, m.dx, S_eig(m))
    total_steps = int(np.floor(m.T / m.dt)) if nsteps is None else int(nsteps)
    f_store = np.zeros((m.M + 2, m.P + 2, 2, 3))
    for t in range(1, total_steps + 1):
        evolve_zeta(m, zeta, psi, t, f_store)
        evolve_psi(m, zeta, psi, pc, hc)
        if callback is not None:
            callback(t, zeta, psi, f_store)
    return zeta, psi, f_store


def update_max(current_max, matrix):  # run_model.jl:41-46
    return np.max(matrix) if np.max(matrix) > current_max else current_max


def update_min(current_min, matrix):  # run_model.jl:48-53
    return np.min(matrix) if np.min(matrix) < current_min else current_min


def diagnostics(zeta, psi, dx):
    """The monitoring record of qg_diagnostics from (M+2, P+2, 2, 3) arrays, slot 1 (newest):
    update_max / update_min of each layer (run_model.jl:41-53, starting from -Inf / +Inf) and
    the definitional sums (circulation, enstrophy, forward-difference kinetic energy,
    interface term) -- not part of the reference, so parity unpinned beyond the max / min."""
    out = {k: [0.0, 0.0] for k in ("zeta_max", "zeta_min", "psi_max", "psi_min", "zeta_sum",
                                   "enstrophy", "energy")}
    for l in range(2):
        z, p = zeta[:, :, l, 0], psi[:, :, l, 0]
        out["zeta_max"][l] = update_max(-np.inf, z)
        out["zeta_min"][l] = update_min(np.inf, z)
        out["psi_max"][l] = update_max(-np.inf, p)
        out["psi_min"][l] = update_min(np.inf, p)
        zi = z[1:-1, 1:-1]
        out["zeta_sum"][l] = zi.sum() * dx * dx
        out["enstrophy"][l] = 0.5 * (zi * zi).sum() * dx * dx
        px = p[2:, 1:-1] - p[1:-1, 1:-1]
        py = p[1:-1, 2:] - p[1:-1, 1:-1]
        out["energy"][l] = 0.5 * (px * px + py * py).sum()
    d = psi[1:-1, 1:-1, 0, 0] - psi[1:-1, 1:-1, 1, 0]
    out["interface"] = 0.5 * (d * d).sum() * dx * dx
    return out


def bench_model(N, dt=30.0 * MINUTES, T=1.0 * DAY, P=None, Lx=4000.0 * KM, Ly=None):
    """The benchmark parameter set of src/benchmarking/julia_bench_parts.jl:6-18."""
    P = N if P is None else P
    Ly = Lx * P / N if Ly is None else Ly
    return make_model(1.0 * KM, 2.0 * KM, 2e-11, Lx, Ly, dt, T, 0.1, N, P, Lx / N, 100.0,
                      1e-7, 40.0 * KM, 1e-6)
