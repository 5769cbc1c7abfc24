"""The caller side of the hot path: ``run_model`` with snapshot output, ``log_model_params`` and
``create_metadata`` (src/run_model.jl:6-95).

The reference writes a JLD (HDF5) file: keys ``zeta_0``, ``psi_0``, ``metadata`` (a Dict) and
``zeta_$t`` / ``psi_$t`` = ``zeta[:,:,:,1]`` / ``psi[:,:,:,1]`` ((M+2, P+2, 2) Float64) every
``sample_timestep = 2*floor(DAY/dt)`` steps (run_model.jl:59, 85-90), while ``metadata``
records ``floor(DAY/dt)`` (run_model.jl:8; the plotting code doubles it again,
plotting/animation.jl:21).  No HDF5 library is available here, so the same keys go into an
``.npz`` (a zip of ``.npy`` members, written incrementally; ``numpy.load`` reads it without
pickling): arrays in Julia index order (M+2, P+2, 2), ``metadata`` as a JSON string.  A Julia
caller writes JLD itself from the same host buffers.

Snapshots leave the GPU without stalling the time loop: ``qg_snapshot`` copies the newest
fields into a device staging buffer in stream order and a copy stream moves them to
page-locked host memory while the next steps run; a writer thread stores each snapshot while
the GPU keeps stepping (two host buffers in rotation).
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import re
import time
import zipfile

import numpy as np

from ._lib import call
from .model import (DAY, SEED_LAYER1, SEED_LAYER2, S1_plus, S2_minus, State, _torch, beta_1, beta_2,
                    ratio_term)


def create_metadata(m):
    """run_model.jl:6-20."""
    sample_interval = 1.0 * DAY
    return {"dt": float(m.dt), "T": float(m.T), "sample_interval": sample_interval,
            "sample_timestep": int(np.floor(sample_interval / m.dt)),
            "total_steps": int(np.floor(m.T / m.dt))}


def julia_repr(x) -> str:
    """``print(x::Float64)`` as Julia writes it (Base.Ryu.writeshortest, compact=false):
    the shortest round-trip digits (the same digits as Python's ``repr``), in decimal form
    when the decimal point position ``pt`` satisfies -4 < pt <= 6 and otherwise as
    ``d.ddde±n`` — e.g. ``4.0e6``, ``1.0e-6``, ``123456.0``, ``0.0001``, ``2.52288e8``.
    Integers print as themselves."""
    if isinstance(x, (int, np.integer)) and not isinstance(x, bool):
        return str(int(x))
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Inf" if x > 0 else "-Inf"
    if x == 0.0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))  # shortest round-trip digits
    m = re.fullmatch(r"(\d+)(?:\.(\d*))?(?:e([+-]?\d+))?", r)
    ip, fp, ex = m.group(1), m.group(2) or "", int(m.group(3) or 0)
    digits = (ip + fp).lstrip("0")
    # decimal exponent of the digit string: value = 0.digits * 10^pt
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    pt = len(ip) + ex - lead_zeros
    digits = digits.rstrip("0") or "0"
    olength = len(digits)
    nexp = pt - olength  # value = digits * 10^nexp
    if -4 < pt <= 6 and not (pt >= olength and abs((abs(x) + 0.05) % 10.0 ** (pt - olength) - 0.05) > 0.05):
        if pt <= 0:
            body = "0." + "0" * (-pt) + digits
        elif pt >= olength:
            body = digits + "0" * (pt - olength) + ".0"
        else:
            body = digits[:pt] + "." + digits[pt:]
    else:
        body = digits[0] + "." + (digits[1:] or "0") + "e" + str(nexp + olength - 1)
    return sign + body


def log_model_params(m, out=print):
    """run_model.jl:22-39 (same lines, same order; numbers printed as Julia's ``println``
    prints a Float64 / Int, see :func:`julia_repr`)."""
    total_steps = int(np.floor(m.T / m.dt))
    j = julia_repr
    out("Parameters:")
    out(f"Lx = {j(m.Lx)}")
    out(f"Ly = {j(m.Ly)}")
    out(f"(f_0^2 / N^2): {j(ratio_term(m))}")
    out(f"S1 = {j(S1_plus(m))}")
    out(f"S2 = {j(S2_minus(m))}")
    out(f"Beta_1 = {j(beta_1(m))}")
    out(f"Beta_2 = {j(beta_2(m))}")
    out(f"M = {j(m.M)}")
    out(f"P = {j(m.P)}")
    out(f"dt = {j(m.dt)}")
    out(f"T = {j(m.T)}")
    out(f"U = {j(m.U)}")
    out(f"Initial kick = {j(m.initial_kick)}")
    out(f"Total steps = {total_steps}\n")


def update_max(current_max: float, matrix) -> float:
    """run_model.jl:41-46 (``matrix``: numpy / torch array, or a qg_diagnostics maximum)."""
    m = float(matrix.max()) if hasattr(matrix, "max") else float(matrix)
    return m if m > current_max else current_max


def update_min(current_min: float, matrix) -> float:
    """run_model.jl:48-53."""
    m = float(matrix.min()) if hasattr(matrix, "min") else float(matrix)
    return m if m < current_min else current_min


class SnapshotWriter:
    """Incremental .npz writer fed by qg_snapshot (see module docstring)."""

    def __init__(self, state: State, file_name: str):
        torch = _torch()
        self.st = state
        shape = (2, state.P_local + 2, state.model.M + 2)  # = Julia (M+2, P+2, 2)
        self.bufs = [tuple(torch.empty(shape, dtype=state.dtype, pin_memory=True) for _ in range(2))
                     for _ in range(2)]
        self.zf = zipfile.ZipFile(file_name, "w", compression=zipfile.ZIP_STORED, allowZip64=True)
        self.pool = cf.ThreadPoolExecutor(max_workers=1)
        self.writes = [None, None]  # pending write of each host buffer
        self.outstanding = None     # (label, buffer index) copied but not yet handed to the writer
        self.k = 0

    def _put(self, name, arr):
        with self.zf.open(name + ".npy", "w", force_zip64=True) as f:
            arr = np.asarray(arr)
            np.lib.format.write_array(f, arr if arr.ndim == 0 else np.ascontiguousarray(arr), allow_pickle=False)

    def _write(self, label, b):
        z, p = self.bufs[b]
        self._put(f"zeta_{label}", z.numpy().transpose(2, 1, 0))
        self._put(f"psi_{label}", p.numpy().transpose(2, 1, 0))

    def _hand_over(self):
        if self.outstanding is not None:
            call("qg_snapshot_wait", self.st._ctx)
            label, b = self.outstanding
            self.writes[b] = self.pool.submit(self._write, label, b)
            self.outstanding = None

    def add(self, label):
        """Snapshot the state's newest zeta / psi under ``zeta_<label>`` / ``psi_<label>``."""
        self._hand_over()
        b = self.k % 2
        if self.writes[b] is not None:
            self.writes[b].result()  # this host buffer is still being written out
        z, p = self.bufs[b]
        call("qg_snapshot", self.st._ctx, z.data_ptr(), p.data_ptr())
        self.outstanding = (label, b)
        self.k += 1

    def metadata(self, md):
        self.pool.submit(self._put, "metadata", np.array(json.dumps(md))).result()

    def close(self):
        self._hand_over()
        for w in self.writes:
            if w is not None:
                w.result()
        self.pool.shutdown()
        self.zf.close()


def run_model(m, file_name: str, save_results: bool, nsteps=None, seeds=(SEED_LAYER1, SEED_LAYER2),
              log=print, monitor=None, **kw):
    """run_model(model, file_name, save_results) (run_model.jl:55-95) on the GPU.  Returns the
    State (its newest zeta / psi are the reference's return values).  ``monitor(t, diag)``, if
    given, receives State.diagnostics() at step 0 and at every sample step."""
    torch = _torch()
    log_model_params(m, log)
    t0 = time.perf_counter()
    st = State(m, **kw)  # the solver tables: the analogue of the two factorisations
    torch.cuda.synchronize()
    log(f"Time to set up the Poisson / modified Helmholtz solver: {time.perf_counter() - t0:.6f} s")
    sample_timestep = 2 * int(np.floor(1.0 * DAY / m.dt))
    total = int(np.floor(m.T / m.dt)) if nsteps is None else int(nsteps)
    st.initialise(seeds)
    writer = None
    if save_results:
        writer = SnapshotWriter(st, file_name)
        writer.metadata(create_metadata(m))
        writer.add("0")
    if monitor is not None:
        monitor(0, st.diagnostics())
    log("Running simulation... \n")
    try:
        for t in range(1, total + 1):
            st.step(t)
            if t % sample_timestep == 0:
                if writer is not None:
                    writer.add(str(t))
                if monitor is not None:
                    monitor(t, st.diagnostics())
    finally:
        if writer is not None:
            writer.close()
    return st
