"""ctypes binding of lib/libqgmi355.so (the C-ABI declared in include/qg_mi355.h).

There is no fallback: if the HIP library is missing or fails to load, every entry point
raises.  The parity tests rely on that (a CPU fallback would void them).
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# QGMI355_LIB: alternative build of the same library (tuning experiments); never a fallback
LIB_PATH = os.environ.get("QGMI355_LIB") or os.path.join(PKG_DIR, "lib", "libqgmi355.so")

QG_OK = 0
QG_ERR_INVALID_ARG, QG_ERR_UNSUPPORTED, QG_ERR_HIP, QG_ERR_NOT_BOUND = -1, -2, -3, -4
QG_ERR_ALLOC, QG_ERR_RCCL, QG_ERR_NOT_CONVERGED = -5, -6, -7
QG_XBUF_TO_NEXT, QG_XBUF_TO_PREV, QG_XBUF_FROM_PREV, QG_XBUF_FROM_NEXT = 0, 1, 2, 3
QG_SOLVER_SPECTRAL = 0
QG_F64, QG_F32 = 0, 1
QG_SOLVER_PCG = 1
QG_PRECOND_NONE = 0
QG_PRECOND_SPECTRAL = 1
QG_PRECOND_MULTIGRID = 2
QG_KEEP_ORDER_SLOT1, QG_KEEP_ORDER_SLOT1_DEFERRED = 2, 3
# qg_set_form (kernel-form selection, process-wide; 0 = automatic)
QG_FORM_TENDENCY, QG_FORM_TENDENCY_TILE, QG_FORM_ROW_SPLIT, QG_FORM_PCG_NO_CERTIFICATE = 0, 1, 2, 3
QG_TEND_AUTO, QG_TEND_RING, QG_TEND_DIRECT, QG_TEND_ONE_POINT = 0, 1, 2, 3


class QgParams(C.Structure):
    """Mirror of ``struct qg_params`` (field order and types must match the header)."""

    _fields_ = [
        ("H_1", C.c_double), ("H_2", C.c_double), ("beta", C.c_double), ("Lx", C.c_double),
        ("Ly", C.c_double), ("dt", C.c_double), ("T", C.c_double), ("U", C.c_double),
        ("M", C.c_int64), ("P", C.c_int64),
        ("dx", C.c_double), ("visc", C.c_double), ("r", C.c_double), ("R_d", C.c_double),
        ("initial_kick", C.c_double),
        ("P_fwd", C.c_double * 4),
        ("solver", C.c_int32), ("precond", C.c_int32),
        ("pcg_rtol", C.c_double),
        ("pcg_maxit", C.c_int32), ("chunk_rows", C.c_int32),
        ("dtype", C.c_int32), ("reserved0", C.c_int32),
        ("wind_tau0", C.c_double), ("wind_rho0", C.c_double),
    ]


class QgDiag(C.Structure):
    _fields_ = [("zeta_max", C.c_double * 2), ("zeta_min", C.c_double * 2), ("psi_max", C.c_double * 2),
                ("psi_min", C.c_double * 2), ("zeta_sum", C.c_double * 2), ("enstrophy", C.c_double * 2),
                ("energy", C.c_double * 2), ("interface", C.c_double), ("reserved", C.c_double)]


class QgStats(C.Structure):
    _fields_ = [("iters", C.c_int32 * 2), ("relres", C.c_double * 2), ("delta", C.c_double),
                ("pin", C.c_double)]


# host-transport callbacks (qg_allgather_fn, qg_sendrecv_fn)
AllgatherFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)
SendrecvFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                         C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                         C.POINTER(C.c_int), C.c_void_p)

# (name, restype, argtypes) of every symbol include/qg_mi355.h declares
_vp, _dp, _i64, _i32 = C.c_void_p, C.c_void_p, C.c_int64, C.c_int
SIGNATURES = [
    ("qg_abi_version", C.c_int, []),
    ("qg_strerror", C.c_char_p, [C.c_int]),
    ("qg_default_params", None, [C.POINTER(QgParams)]),
    ("qg_create", C.c_int, [C.POINTER(QgParams), C.c_int, _vp, C.POINTER(_vp)]),
    ("qg_destroy", C.c_int, [_vp]),
    ("qg_bind_state", C.c_int, [_vp, _dp, _dp, _dp]),
    ("qg_initialise", C.c_int, [_vp, C.c_uint64, C.c_uint64]),
    ("qg_evolve_zeta", C.c_int, [_vp, _i64]),
    ("qg_evolve_psi", C.c_int, [_vp]),
    ("qg_step", C.c_int, [_vp, _i64]),
    ("qg_run", C.c_int, [_vp, _i64, _i64]),
    ("qg_slot", C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    ("qg_set_slots", C.c_int, [_vp, C.c_int * 3]),
    ("qg_canonicalize", C.c_int, [_vp]),
    ("qg_set_keep_order", C.c_int, [_vp, C.c_int]),
    ("qg_get_stats", C.c_int, [_vp, C.POINTER(QgStats)]),
    ("qg_solver_stats", C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double)]),
    ("qg_synchronize", C.c_int, [_vp]),
    ("qg_snapshot", C.c_int, [_vp, _vp, _vp]),
    ("qg_snapshot_wait", C.c_int, [_vp]),
    ("qg_diagnostics", C.c_int, [_vp, C.POINTER(QgDiag)]),
    ("qg_comm_unique_id", C.c_int, [C.c_char_p]),
    ("qg_comm_init", C.c_int, [_vp, C.c_int, C.c_int, C.c_char_p]),
    ("qg_comm_init_host", C.c_int, [_vp, C.c_int, C.c_int, AllgatherFn, SendrecvFn, _vp]),
    ("qg_comm_set_timeout", C.c_int, [_vp, C.c_double]),
    ("qg_set_overlap", C.c_int, [_vp, C.c_int]),
    ("qg_comm_set_halo_transport", C.c_int, [_vp, C.c_int]),
    ("qg_comm_set_gather_transport", C.c_int, [_vp, C.c_int]),
    ("qg_comm_probe", C.c_int, [_vp, C.c_int, C.POINTER(C.c_double)]),
    ("qg_set_pcg_sync", C.c_int, [_vp, C.c_int]),
    ("qg_pcg_certificate", C.c_int, [_vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                     C.POINTER(C.c_double)]),
    ("qg_comm_exchange_plan", C.c_int, [C.c_int, C.c_int, C.c_int * 2, C.c_int * 2, C.c_int * 2, C.c_int * 2]),
    ("qg_solver_create", C.c_int, [_i64, _i64, C.c_double, C.c_double * 2, C.c_int * 2,
                                   C.c_double * 4, C.c_double * 4, C.c_int, C.c_int, C.c_int, _vp,
                                   C.POINTER(_vp)]),
    ("qg_solver_solve", C.c_int, [_vp, _dp, _dp, _dp, _dp]),
    ("qg_solver_destroy", C.c_int, [_vp]),
    ("qg_set_form", C.c_int, [C.c_int, C.c_int]),
    ("qg_get_form", C.c_int, [C.c_int]),
    ("qg_laplace_5p", C.c_int, [_dp, _dp, _i64, _i64, C.c_double, _vp]),
    ("qg_cd", C.c_int, [_dp, _dp, _i64, _i64, C.c_double, _vp]),
    ("qg_arakawa_J", C.c_int, [_dp, _dp, _dp, _i64, _i64, C.c_double, _vp]),
    ("qg_fill_ghosts", C.c_int, [_dp, _i64, _i64, _vp]),
]

_lib = None


class QGError(RuntimeError):
    def __init__(self, fn, status):
        msg = _lib.qg_strerror(status).decode() if _lib is not None else str(status)
        super().__init__(f"{fn} failed with status {status}: {msg}")
        self.status = status


def lib():
    """Load the HIP library (raises if it is not built -- there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not found: build it with `make -C julia-ocean-modelling_amd` "
                "(or __graft_entry__.build()); the QG hot path has no CPU fallback")
        # PyTorch first: it ships its own HIP runtime, and the library must bind to that one
        # (loading ours first would bring in /opt/rocm's libamdhip64 as a second runtime)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            # (an older experiment build named by QGMI355_LIB may lack newer entry points)
            if os.environ.get("QGMI355_LIB") and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(fn, status):
    if status != QG_OK:
        raise QGError(fn, status)
    return status


def call(name, *args):
    return check(name, getattr(lib(), name)(*args))
