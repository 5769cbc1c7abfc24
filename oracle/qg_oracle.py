"""ctypes wrapper of oracle/libqg_oracle.so (CPU ORACLE -- test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libqg_oracle.so")


class QgoParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in
                ("H_1", "H_2", "beta", "Lx", "Ly", "dt", "T", "U", "dx", "visc", "r", "R_d",
                 "initial_kick")] + [("M", C.c_long), ("P", C.c_long), ("Pfwd", C.c_double * 4),
                                     ("wind_tau0", C.c_double), ("wind_rho0", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="F_CONTIGUOUS")
        L.qgo_laplace_5p.argtypes = [dp, dp, C.c_long, C.c_long, C.c_double]
        L.qgo_cd.argtypes = [dp, dp, C.c_long, C.c_long, C.c_double]
        L.qgo_J.argtypes = [C.c_double, dp, dp, dp, C.c_long, C.c_long]
        L.qgo_fill_ghosts.argtypes = [dp, C.c_long, C.c_long]
        L.qgo_solve.argtypes = [C.c_long, C.c_long, C.c_double, C.c_double, C.c_int, dp, dp]
        L.qgo_solve.restype = C.c_int
        L.qgo_run.argtypes = [C.POINTER(QgoParams), C.c_uint64, C.c_uint64, C.c_long, C.c_long,
                              dp, dp, dp, C.c_int, C.c_int]
        L.qgo_run.restype = C.c_int
        L.qgo_max_threads.restype = C.c_int
        _lib = L
    return _lib


def params(m, P_fwd=None, wind=None):
    """QgoParams from an oracle.qg_ref.BaroclinicModel; wind = (tau0, rho0) switches on the
    wind-forcing extension (not in the reference)."""
    p = QgoParams()
    for n in ("H_1", "H_2", "beta", "Lx", "Ly", "dt", "T", "U", "dx", "visc", "r", "R_d",
              "initial_kick"):
        setattr(p, n, float(getattr(m, n)))
    p.M, p.P = int(m.M), int(m.P)
    Pf = np.array([[1.0, -1.0], [1.0, 1.0]]) if P_fwd is None else np.asarray(P_fwd, float)
    # default = P_matrix(H_1, H_1) as the reference's evolve_psi! builds it (model.jl:173)
    if P_fwd is None:
        Pf = np.array([[1.0, -m.H_1 / m.H_1], [1.0, 1.0]])
    for k, v in enumerate(Pf.reshape(-1)):
        p.Pfwd[k] = float(v)
    p.wind_tau0, p.wind_rho0 = (0.0, 1000.0) if wind is None else (float(wind[0]), float(wind[1]))
    return p


def _f(a):
    return np.asfortranarray(a, dtype=np.float64)


def laplace_5p(u, dx):
    u = _f(u)
    out = np.zeros_like(u, order="F")
    lib().qgo_laplace_5p(u, out, u.shape[0], u.shape[1], float(dx))
    return out


def cd(u, dx):
    u = _f(u)
    out = np.zeros_like(u, order="F")
    lib().qgo_cd(u, out, u.shape[0], u.shape[1], float(dx))
    return out


def J(dx, z, p):
    z, p = _f(z), _f(p)
    out = np.zeros_like(z, order="F")
    lib().qgo_J(float(dx), z, p, out, z.shape[0], z.shape[1])
    return out


def solve(M, P, dx, alpha, f, pinned=False):
    f = _f(f)
    out = np.zeros_like(f, order="F")
    rc = lib().qgo_solve(M, P, float(dx), float(alpha), int(pinned), f, out)
    assert rc == 0
    return out


class State:
    """(M+2,P+2,2,3) zeta/psi/f_store arrays, Fortran order (Julia layout)."""

    def __init__(self, m, seeds=(20241008, 20241009), P_fwd=None, nthreads=0, wind=None):
        self.m = m
        self.p = params(m, P_fwd, wind)
        self.seeds = seeds
        self.nthreads = nthreads
        shape = (m.M + 2, m.P + 2, 2, 3)
        self.zeta = np.zeros(shape, order="F")
        self.psi = np.zeros(shape, order="F")
        self.f_store = np.zeros(shape, order="F")
        self.t = 0
        lib().qgo_run(C.byref(self.p), seeds[0], seeds[1], 1, 0, self.zeta, self.psi,
                      self.f_store, 1, nthreads)

    def run(self, nsteps):
        lib().qgo_run(C.byref(self.p), self.seeds[0], self.seeds[1], self.t + 1, int(nsteps),
                      self.zeta, self.psi, self.f_store, 0, self.nthreads)
        self.t += int(nsteps)
        return self
