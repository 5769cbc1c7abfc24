"""Host-side mirror of the reference's operator surface for the hot path, driving the HIP
C-ABI (include/qg_mi355.h) on device arrays.

Reference surface (JSLeadbetter/julia-ocean-modelling, paths relative to its root):
  BaroclinicModel + outer constructor          src/model.jl:12-34
  ratio_term, S1_plus, S2_minus, beta_1/2, S_eig  src/model.jl:109-121
  P_matrix, P_inv_matrix                        src/model.jl:83-99
  initialise_model                              src/model.jl:37-62
  evolve_zeta!, evolve_psi!                     src/model.jl:155-199
  get_poisson_cholesky, get_helmholtz_cholesky  src/schemes/laplacian.jl:60-75
  run_model_no_output                           src/run_model_no_output.jl:3-16
  laplace_5p, cd, J, update_doubly_periodic_bc! laplacian.jl:15, model.jl:68, arakawa.jl:58,
                                                boundary_conditions.jl:2
  sp_solve_modified_helmholtz, sp_solve_poisson laplacian.jl:78-111

Device arrays are torch float64 CUDA tensors used only as memory: a Julia
(M+2, P+2, 2, 3) column-major array is a C-contiguous tensor of shape (3, 2, P+2, M+2)
(``[slot, layer, j, i]``), a Julia (M+2, P+2) matrix a (P+2, M+2) tensor.  Python names
cannot carry ``!``; the mutating functions end in ``_`` instead.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import QgParams, QgStats, call

MINUTES = 60
DAY = 60 * 60 * 24
KM = 1000.0
YEAR = 60 * 60 * 24 * 365

SEED_LAYER1 = 20241008
SEED_LAYER2 = 20241009


# ---------------------------------------------------------------------------------------
# kernel-form selection (qg_set_form: process-wide, 0 = the library's choice by size)
# ---------------------------------------------------------------------------------------
def set_form(which, value):
    """Force one kernel form (``_lib.QG_FORM_*``); value 0 restores the automatic choice."""
    call("qg_set_form", int(which), int(value))


def get_form(which):
    v = _lib.lib().qg_get_form(int(which))
    if v < 0:
        raise _lib.QGError("qg_get_form", v)
    return v


@contextlib.contextmanager
def forced_form(which, value):
    """``with forced_form(QG_FORM_TENDENCY, QG_TEND_RING): ...`` -- the previous value after."""
    old = get_form(which)
    set_form(which, value)
    try:
        yield
    finally:
        set_form(which, old)


# ---------------------------------------------------------------------------------------
# parameters
# ---------------------------------------------------------------------------------------
@dataclass(frozen=True)
class BaroclinicModel:
    """``struct BaroclinicModel`` (src/model.jl:12-30).  Build with :func:`make_model`
    (the outer constructor, model.jl:33-34) or :meth:`create`."""

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

    @staticmethod
    def create(H_1, H_2, beta, Lx, Ly, dt, T, U, M, P, dx, visc, r, R_d, initial_kick):
        return make_model(H_1, H_2, beta, Lx, Ly, dt, T, U, M, P, dx, visc, r, R_d, initial_kick)


def make_model(H_1, H_2, beta, Lx, Ly, dt, T, U, M, P, dx, visc, r, R_d, initial_kick):
    """Outer constructor (model.jl:33-34): H = H_1 + H_2."""
    return BaroclinicModel(float(H_1), float(H_2), float(H_1) + float(H_2), float(beta), float(Lx),
                           float(Ly), float(dt), float(T), float(U), int(M), int(P), float(dx),
                           float(visc), float(r), float(R_d), float(initial_kick))


def bench_model(N, dt=30.0 * MINUTES, T=1.0 * DAY, P=None, Lx=4000.0 * KM):
    """Benchmark parameter set of src/benchmarking/julia_bench_parts.jl:6-18 (square cells)."""
    P = N if P is None else P
    return make_model(1.0 * KM, 2.0 * KM, 2e-11, Lx, Lx * P / N, dt, T, 0.1, N, P, Lx / N, 100.0,
                      1e-7, 40.0 * KM, 1e-6)


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
    a, b = S1_plus(m), S2_minus(m)
    return (1 / (a + b)) * np.array([[b, a], [-b, b]])


def qg_params(m, solver=_lib.QG_SOLVER_SPECTRAL, P_fwd=None, chunk_rows=0, P_local=None,
              precond=_lib.QG_PRECOND_SPECTRAL, pcg_rtol=1e-12, pcg_maxit=500, dtype=_lib.QG_F64,
              wind=None):
    """wind = (tau0 [N m^-2], rho0 [kg m^-3]) switches on the double-gyre wind forcing
    extension of the upper layer (include/qg_mi355.h; not in the reference)."""
    p = QgParams()
    _lib.lib().qg_default_params(C.byref(p))
    for n in ("H_1", "H_2", "beta", "Lx", "Ly", "dt", "T", "U", "dx", "visc", "r", "R_d",
              "initial_kick"):
        setattr(p, n, float(getattr(m, n)))
    p.M = int(m.M)
    p.P = int(m.P if P_local is None else P_local)
    if P_fwd is not None:
        for k, v in enumerate(np.asarray(P_fwd, dtype=np.float64).reshape(-1)):
            p.P_fwd[k] = float(v)
    p.solver = int(solver)
    p.precond = int(precond)
    p.pcg_rtol = float(pcg_rtol)
    p.pcg_maxit = int(pcg_maxit)
    p.chunk_rows = int(chunk_rows)
    p.dtype = int(dtype)
    if wind is not None:
        p.wind_tau0, p.wind_rho0 = float(wind[0]), float(wind[1])
    return p


# ---------------------------------------------------------------------------------------
# device plumbing
# ---------------------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def _stream_ptr():
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr())


def _check_field(t, M, P):
    torch = _torch()
    if not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
        raise ValueError("expected a contiguous float64 CUDA tensor")
    if tuple(t.shape[-2:]) != (P + 2, M + 2):
        raise ValueError(f"field shape {tuple(t.shape)} does not match (P+2, M+2) = {(P + 2, M + 2)}")


def device_zeros(m, P_local=None, device="cuda", dtype=None):
    """zeros(M+2, P+2, 2, 3) in Julia layout -> tensor (3, 2, P+2, M+2)."""
    torch = _torch()
    P = m.P if P_local is None else P_local
    return torch.zeros((3, 2, P + 2, m.M + 2), dtype=torch.float64 if dtype is None else dtype, device=device)


class State:
    """The model state zeta, psi, f_store plus the library context that evolves it.

    Plays the role of the reference's (zeta, psi, f_store) arrays and its two CHOLMOD
    factors.  History slots rotate (no copies): :meth:`slot` maps the reference's slot
    index (1 = newest) to the physical slot, :meth:`logical` returns the reference-ordered
    view, :meth:`canonicalize` physically restores the reference order.
    """

    def __init__(self, m, solver=_lib.QG_SOLVER_SPECTRAL, P_fwd=None, chunk_rows=0,
                 device=None, rank=0, nranks=1, P_local=None, precond=_lib.QG_PRECOND_SPECTRAL,
                 pcg_rtol=1e-12, pcg_maxit=500, dtype=None, wind=None, arrays=None):
        """dtype: torch.float64 (default, the reference's arithmetic) or torch.float32 (the
        F32 state of BASELINE config 5; spectral solver only).  wind: (tau0, rho0) of the
        wind-forcing extension, or None (the reference's right-hand side).  arrays: an
        existing (zeta, psi, f_store) triple of (3, 2, P+2, M+2) device tensors to bind
        instead of allocating new ones (the caller keeps ownership)."""
        _lib.lib()  # the HIP library first: no CPU fallback, fail before touching the device
        torch = _torch()
        self.model = m
        self.P_local = m.P if P_local is None else P_local
        # device: None (current), an ordinal, "cuda:k" or a torch.device -> ordinal k.  The
        # arrays and the stream the library launches on all belong to that device.
        if device is None:
            self.device = torch.cuda.current_device()
        else:
            dev = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
            if dev.type != "cuda":
                raise ValueError(f"State needs a CUDA (HIP) device, got {dev}")
            self.device = dev.index if dev.index is not None else torch.cuda.current_device()
        self.dtype = torch.float64 if dtype is None else dtype
        if self.dtype not in (torch.float64, torch.float32):
            raise ValueError("dtype must be torch.float64 or torch.float32")
        with torch.cuda.device(self.device):
            dev = torch.device("cuda", self.device)
            if arrays is None:
                self.zeta = device_zeros(m, self.P_local, device=dev, dtype=self.dtype)
                self.psi = device_zeros(m, self.P_local, device=dev, dtype=self.dtype)
                self.f_store = device_zeros(m, self.P_local, device=dev, dtype=self.dtype)
            else:
                shape = (3, 2, self.P_local + 2, m.M + 2)
                for t in arrays:
                    if (tuple(t.shape) != shape or t.dtype != self.dtype or t.device != dev
                            or not t.is_contiguous()):
                        raise ValueError(f"bound arrays must be contiguous {self.dtype} tensors of shape "
                                         f"{shape} on {dev}")
                self.zeta, self.psi, self.f_store = arrays
            self.params = qg_params(m, solver, P_fwd, chunk_rows, self.P_local, precond, pcg_rtol, pcg_maxit,
                                    _lib.QG_F32 if self.dtype == torch.float32 else _lib.QG_F64, wind)
            self._ctx = C.c_void_p()
            call("qg_create", C.byref(self.params), int(self.device), _stream_ptr(), C.byref(self._ctx))
            call("qg_bind_state", self._ctx, _ptr(self.zeta), _ptr(self.psi), _ptr(self.f_store))
        # rank / nranks describe the slab this state holds (e.g. read back from a slab
        # checkpoint); stepping a slab of a multi-rank run needs that transport attached first
        self.rank, self.nranks = rank, nranks
        self._attached_ranks = 1

    def close(self):
        """Destroy the library context now (qg_destroy); the arrays stay with the caller."""
        ctx = getattr(self, "_ctx", None)
        if ctx and _lib._lib is not None:
            _lib._lib.qg_destroy(ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    # -- multi-GPU ---------------------------------------------------------------------
    def comm_init(self, nranks, rank, uid: bytes):
        call("qg_comm_init", self._ctx, int(nranks), int(rank), C.c_char_p(uid))
        self.rank, self.nranks = rank, nranks
        self._attached_ranks = nranks

    def set_overlap(self, on=True):
        """qg_set_overlap: post each step's halo exchange on a second stream and run the
        interior rows' tendency meanwhile (multi-rank only; bit-identical results)."""
        call("qg_set_overlap", self._ctx, 1 if on else 0)

    def set_halo_transport(self, transport="rccl"):
        """qg_comm_set_halo_transport (collective, RCCL transport only): "rccl" (pack kernel +
        grouped send/recv), "peer" (copy-engine copies into the neighbours' IPC-mapped
        receive regions + arrival flags; no collective kernel beside the interior tendency) or
        "put" (the same regions, rows stored by one small kernel that also waits)."""
        modes = {"rccl": 0, "peer": 1, "put": 2}
        if transport not in modes:
            raise ValueError(f"halo transport {transport!r}: one of {sorted(modes)}")
        call("qg_comm_set_halo_transport", self._ctx, modes[transport])
        self.halo_transport = transport

    def set_gather_transport(self, transport="rccl"):
        """qg_comm_set_gather_transport (collective, RCCL transport, direct solver): "rccl"
        (ncclAllGather of the rank records) or "peer" (one kernel storing the record into every
        peer's IPC-mapped region in parallel, flags, copy-out)."""
        modes = {"rccl": 0, "peer": 1}
        if transport not in modes:
            raise ValueError(f"gather transport {transport!r}: one of {sorted(modes)}")
        call("qg_comm_set_gather_transport", self._ctx, modes[transport])
        self.gather_transport = transport

    def comm_probe(self, reps=20):
        """qg_comm_probe: event-timed halo exchange and record all-gather of one step, in
        isolation (every rank must call it): ms and bytes per collective."""
        out = (C.c_double * 4)()
        call("qg_comm_probe", self._ctx, int(reps), out)
        return {"halo_ms": out[0], "halo_bytes_sent": int(out[1]), "allgather_ms": out[2],
                "allgather_bytes_received": int(out[3]), "reps": int(reps)}

    def set_pcg_sync(self, sync=True):
        """qg_set_pcg_sync: 1 = the host checks every PCG residual (and iterates when the
        certificate fails); 0 = deferred on-device certification (default)."""
        call("qg_set_pcg_sync", self._ctx, 1 if sync else 0)

    def pcg_certificate(self):
        """qg_pcg_certificate: deferred PCG certificates so far."""
        n, f, first, worst = C.c_int64(), C.c_int64(), C.c_int64(), C.c_double()
        call("qg_pcg_certificate", self._ctx, C.byref(n), C.byref(f), C.byref(first), C.byref(worst))
        return {"solves": n.value, "failures": f.value, "first_failure": first.value, "worst_relres": worst.value}

    def _need_transport(self):
        if self.nranks != self._attached_ranks:
            raise RuntimeError(f"this state is slab {self.rank} of {self.nranks}: attach the {self.nranks}-rank "
                               "transport (comm_init / TorchDistTransport.attach) before stepping it")

    # -- reference operations ----------------------------------------------------------
    def initialise(self, seeds=(SEED_LAYER1, SEED_LAYER2)):
        call("qg_initialise", self._ctx, int(seeds[0]), int(seeds[1]))
        return self

    def evolve_zeta_(self, timestep):
        self._need_transport()
        call("qg_evolve_zeta", self._ctx, int(timestep))

    def evolve_psi_(self):
        self._need_transport()
        call("qg_evolve_psi", self._ctx)

    def step(self, timestep):
        self._need_transport()
        call("qg_step", self._ctx, int(timestep))

    def run(self, first_step, nsteps):
        self._need_transport()
        call("qg_run", self._ctx, int(first_step), int(nsteps))

    def synchronize(self):
        call("qg_synchronize", self._ctx)

    def stats(self):
        s = QgStats()
        call("qg_get_stats", self._ctx, C.byref(s))
        return {"delta": s.delta, "pin": s.pin, "iters": list(s.iters), "relres": list(s.relres)}

    def diagnostics(self):
        """qg_diagnostics: max / min of the newest zeta and psi per layer (the update_max /
        update_min of run_model.jl:41-53), circulation, enstrophy, kinetic energy and the
        interface term, over the global domain (multi-GPU: every rank calls it)."""
        d = _lib.QgDiag()
        call("qg_diagnostics", self._ctx, C.byref(d))
        return {f: (list(getattr(d, f)) if f != "interface" else d.interface)
                for f, _ in _lib.QgDiag._fields_ if f != "reserved"}

    # -- slot rotation -----------------------------------------------------------------
    def slot(self, which, logical):
        w = {"zeta": 0, "psi": 1, "f_store": 2}[which]
        out = C.c_int()
        call("qg_slot", self._ctx, w, int(logical), C.byref(out))
        return out.value

    def heads(self):
        return [self.slot(w, 1) for w in ("zeta", "psi", "f_store")]

    def set_heads(self, heads):
        call("qg_set_slots", self._ctx, (C.c_int * 3)(*[int(h) for h in heads]))

    def logical(self, which):
        """(3, 2, P+2, M+2) tensor in reference slot order (a gathered copy)."""
        torch = _torch()
        t = getattr(self, which)
        order = [self.slot(which, s) for s in (1, 2, 3)]
        return t[torch.tensor(order, device=t.device)]

    def current(self, which, layer):
        """Reference ``X[:, :, layer, 1]`` (layer 1-based) as a (P+2, M+2) view (multi-GPU:
        ghost rows current after synchronize())."""
        return getattr(self, which)[self.slot(which, 1), layer - 1]

    def canonicalize(self):
        call("qg_canonicalize", self._ctx)

    def set_keep_order(self, on=True, slot1_only=False, deferred=False):
        """qg_set_keep_order: every call leaves slot 1 = newest (store_new_state!'s shift, in
        place, before the new values are written), so the arrays are always in the
        reference's slot order; off (default) rotates the slots instead.  slot1_only
        (QG_KEEP_ORDER_SLOT1): slot 1 of zeta / psi and all of f_store kept so after every
        call, slots 2-3 of zeta and psi (never read by the reference) not maintained -- one
        slot copy per step instead of four.  deferred (with slot1_only,
        QG_KEEP_ORDER_SLOT1_DEFERRED): that copy rides in the next evolve_psi!'s first solver
        pass, so slot 1 of zeta is stale between evolve_zeta! and evolve_psi! (qg_slot names
        the newest; synchronize() completes the move)."""
        mode = (_lib.QG_KEEP_ORDER_SLOT1_DEFERRED if deferred else _lib.QG_KEEP_ORDER_SLOT1) if slot1_only else 1
        call("qg_set_keep_order", self._ctx, mode if on else 0)

    def to_numpy(self, which):
        """Reference-ordered numpy array of shape (M+2, P+2, 2, 3) (Julia index order).
        Synchronises first (multi-GPU: completes the lazily refreshed ghost rows)."""
        self.synchronize()
        return self.logical(which).permute(3, 2, 1, 0).contiguous().cpu().numpy()


# ---------------------------------------------------------------------------------------
# the reference's free functions
# ---------------------------------------------------------------------------------------
def initialise_model(m, seeds=(SEED_LAYER1, SEED_LAYER2), **kw):
    """initialise_model (model.jl:37-62) with seeded noise; returns the device State."""
    if not np.sign(beta_1(m)) == -np.sign(beta_2(m)):  # model.jl:38
        raise AssertionError("sign(beta_1) must equal -sign(beta_2)")
    return State(m, **kw).initialise(seeds)


_BOUND = {}
_DROPIN_SLOTS = ["all"]


def set_dropin_slots(mode):
    """Slots the reference-signature calls below maintain on arrays bound from now on:
    "all" (default: store_new_state! exactly, slots 2-3 of zeta and psi shifted too),
    "slot1" (QG_KEEP_ORDER_SLOT1: slot 1 of zeta and psi and all of f_store, the values the
    reference's loop reads, newest after every call; one slot copy per step instead of four)
    or "slot1_deferred" (QG_KEEP_ORDER_SLOT1_DEFERRED: as "slot1", the copy of the new zeta
    into slot 1 done by the next evolve_psi!'s first solver pass -- slot 1 of zeta is stale
    between evolve_zeta! and evolve_psi!, which the reference's loop never reads there)."""
    if mode not in ("all", "slot1", "slot1_deferred"):
        raise ValueError("mode must be 'all', 'slot1' or 'slot1_deferred'")
    _DROPIN_SLOTS[0] = mode


def _bound_state(m, zeta, psi, f_store):
    """The library context bound to a caller's (zeta, psi, f_store) arrays, created on first
    use and cached by their addresses (the reference-signature calls below).  The context
    keeps the reference's slot order on every call (qg_set_keep_order), as store_new_state!
    does.  A different model for the same arrays replaces the cached context."""
    key = (zeta.data_ptr(), psi.data_ptr(), f_store.data_ptr())
    st = _BOUND.get(key)
    if st is None or st.model != m:
        if st is not None:  # settle and release the old context (its failure is raised after)
            st = None
            unbind(zeta, psi, f_store)
        st = _BOUND[key] = State(m, device=zeta.device, dtype=zeta.dtype, arrays=(zeta, psi, f_store))
        st.set_keep_order(True, slot1_only=_DROPIN_SLOTS[0] != "all",
                          deferred=_DROPIN_SLOTS[0] == "slot1_deferred")
    return st


def unbind(zeta=None, psi=None, f_store=None):
    """Release the cached contexts of the reference-signature calls: the one bound to these
    arrays, or all of them (no arguments).  The contexts hold references to the arrays, so
    without this the arrays stay alive as long as the process.  Every selected context is
    released even if settling one fails (e.g. a deferred PCG certificate that failed,
    QG_ERR_NOT_CONVERGED); the first such error is raised after all of them are released."""
    if zeta is None:
        keys = list(_BOUND)
    else:
        keys = [k for k in _BOUND if k[0] == zeta.data_ptr()
                and (psi is None or k[1] == psi.data_ptr())
                and (f_store is None or k[2] == f_store.data_ptr())]
    err = None
    for k in keys:
        st = _BOUND.pop(k)
        try:
            st.synchronize()
        except Exception as e:  # noqa: BLE001 -- re-raised below, after every release
            err = err or e
        finally:
            st.close()
            del st
    if err is not None:
        raise err
    return len(keys)


def evolve_zeta_(m, *args):
    """evolve_zeta!(model, zeta, psi, timestep, f_store) (model.jl:155-158).

    Two forms: ``evolve_zeta_(m, state, timestep)`` on a :class:`State` (slots rotate, no
    copies), and the reference's own signature ``evolve_zeta_(m, zeta, psi, timestep,
    f_store)`` on (3, 2, P+2, M+2) device tensors, which leaves the arrays in the reference's
    slot order after the call (slot 1 = newest, as store_new_state! leaves them)."""
    if len(args) == 2:
        state, timestep = args
        state.evolve_zeta_(timestep)
        return
    zeta, psi, timestep, f_store = args
    st = _bound_state(m, zeta, psi, f_store)
    st.evolve_zeta_(timestep)  # (keep-order context: the arrays stay in reference order)


class SolverHandle:
    """Stands in for SparseArrays.CHOLMOD.Factor in evolve_psi!'s signature.  The state's
    context owns the actual solver (both systems are solved together on the device)."""

    def __init__(self, kind, M, P, dx, alpha):
        self.kind, self.M, self.P, self.dx, self.alpha = kind, M, P, dx, alpha


def get_poisson_cholesky(M, P, dx):  # laplacian.jl:66-75
    return SolverHandle("poisson", M, P, dx, 0.0)


def get_helmholtz_cholesky(M, P, dx, alpha):  # laplacian.jl:60-64
    return SolverHandle("helmholtz", M, P, dx, alpha)


def evolve_psi_(m, *args):
    """evolve_psi!(model, zeta, psi, poisson_cholesky, helmholtz_cholesky) (model.jl:172-199).

    ``evolve_psi_(m, state[, poisson, helmholtz])`` on a :class:`State`, or the reference's
    signature ``evolve_psi_(m, zeta, psi, poisson, helmholtz)`` on device tensors already
    bound by :func:`evolve_zeta_` (which knows their f_store)."""
    if isinstance(args[0], State):
        state, poisson, helmholtz = (tuple(args) + (None, None))[:3]
    else:
        zeta, psi, poisson, helmholtz = args
        hits = [st for k, st in _BOUND.items() if k[:2] == (zeta.data_ptr(), psi.data_ptr())]
        if len(hits) != 1:
            raise ValueError("evolve_psi_: call evolve_zeta_ on these arrays first (it binds them "
                             "with their f_store)")
        state = hits[0]
        if state.model != m:
            raise ValueError("evolve_psi_: these arrays are bound to a different model (call "
                             "evolve_zeta_ with this model first, or unbind them)")
    for h, kind in ((poisson, "poisson"), (helmholtz, "helmholtz")):
        if h is not None and (h.kind != kind or h.M != m.M or h.P != m.P or h.dx != m.dx):
            raise ValueError(f"{kind} handle does not match the model")
    if helmholtz is not None and helmholtz.alpha != S_eig(m):
        raise ValueError("helmholtz handle alpha != S_eig(model)")
    state.evolve_psi_()


def run_model_no_output(m, nsteps=None, seeds=(SEED_LAYER1, SEED_LAYER2), **kw):
    """run_model_no_output.jl:3-16: init, total_steps = floor(T/dt) steps; returns State."""
    st = initialise_model(m, seeds, **kw)
    total = int(np.floor(m.T / m.dt)) if nsteps is None else int(nsteps)
    st.run(1, total)
    return st


# ---- stateless operators on (P+2, M+2) device matrices -----------------------------------
def _dims(u):
    P2, M2 = u.shape[-2:]
    return M2 - 2, P2 - 2


def laplace_5p(u, dx):
    torch = _torch()
    M, P = _dims(u)
    _check_field(u, M, P)
    out = torch.empty_like(u)
    call("qg_laplace_5p", _ptr(u), _ptr(out), M, P, float(dx), _stream_ptr())
    return out


def cd(u, dx):
    torch = _torch()
    M, P = _dims(u)
    _check_field(u, M, P)
    out = torch.empty_like(u)
    call("qg_cd", _ptr(u), _ptr(out), M, P, float(dx), _stream_ptr())
    return out


def J(dx, zeta, psi):
    torch = _torch()
    M, P = _dims(zeta)
    _check_field(zeta, M, P)
    _check_field(psi, M, P)
    out = torch.empty_like(zeta)
    call("qg_arakawa_J", _ptr(zeta), _ptr(psi), _ptr(out), M, P, float(dx), _stream_ptr())
    return out


def update_doubly_periodic_bc_(b):
    M, P = _dims(b)
    _check_field(b, M, P)
    call("qg_fill_ghosts", _ptr(b), M, P, _stream_ptr())
    return b


class PairSolver:
    """qg_solver handle: A_s x_s = proj_in . f for s = 0 (optionally pinned Poisson), 1."""

    def __init__(self, M, P, dx, alpha, pinned=(0, 0), proj_in=(1, 0, 0, 1), proj_out=(1, 0, 0, 1),
                 kind=_lib.QG_SOLVER_SPECTRAL, precond=_lib.QG_PRECOND_SPECTRAL):
        torch = _torch()
        self.M, self.P = M, P
        self._h = C.c_void_p()
        call("qg_solver_create", int(M), int(P), float(dx), (C.c_double * 2)(*alpha),
             (C.c_int * 2)(*pinned), (C.c_double * 4)(*proj_in), (C.c_double * 4)(*proj_out),
             int(kind), int(precond), int(torch.cuda.current_device()), _stream_ptr(), C.byref(self._h))

    def solve(self, f1, f2=None, out1=None, out2=None):
        torch = _torch()
        _check_field(f1, self.M, self.P)
        out1 = torch.empty_like(f1) if out1 is None else out1
        call("qg_solver_solve", self._h, _ptr(f1), _ptr(f2) if f2 is not None else None, _ptr(out1),
             _ptr(out2) if out2 is not None else None)
        return out1 if out2 is None else (out1, out2)

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.qg_solver_destroy(self._h)
            self._h = None


def sp_solve_modified_helmholtz(M, P, dx, f, alpha, **kw):
    """laplacian.jl:78-86: solution x of construct_spA(M,P,dx,alpha) x = f, with ghosts."""
    s = PairSolver(M, P, dx, (float(alpha), -1.0), (0, 0), (1, 0, 0, 0), (1, 0, 0, 0), **kw)
    return s.solve(f)


def sp_solve_poisson(M, P, dx, f, **kw):
    """laplacian.jl:100-111: the pinned Poisson solve (x = 0 at interior (1,1))."""
    s = PairSolver(M, P, dx, (0.0, -1.0), (1, 0), (1, 0, 0, 0), (1, 0, 0, 0), **kw)
    return s.solve(f)
