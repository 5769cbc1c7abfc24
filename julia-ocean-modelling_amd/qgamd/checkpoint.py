"""Checkpoint / resume of a run (the reference itself cannot resume).

The reference keeps its whole state in three caller-owned arrays (``zeta``, ``psi``,
``f_store``, each (M+2, P+2, 2, 3), model.jl:155-199) and the step counter of its loop
(run_model_no_output.jl:10-13).  AB3 (model.jl:129-136) reads the two previous tendencies,
so a faithful resume must carry ``f_store`` as well as the snapshot fields -- the JLD
snapshots of run_model.jl:85-90 (zeta[:,:,:,1], psi[:,:,:,1]) are not enough.

A checkpoint is an ``.npz`` (no pickling) holding the three arrays in the reference's slot
order and Julia index order, the model parameters, the solver options and the last completed
timestep.  A resumed run continues bit for bit (both solvers start from x0 = 0 each step, so
no solver state is needed).  Multi-GPU: each rank saves / loads its own slab file; attach the
transport (``comm_init``) after loading, before stepping.
"""
from __future__ import annotations

import dataclasses
import json

import numpy as np

from . import _lib
from .model import BaroclinicModel, State, _torch

FORMAT = "qgmi355-checkpoint-1"


def save_checkpoint(state: State, path: str, timestep: int) -> None:
    """Write ``state`` after ``timestep`` completed steps (synchronises; multi-GPU: all ranks
    call it, each with its own ``path``).  The slot rotation is canonicalised first, so the
    device arrays are in the reference's order afterwards as well."""
    state.canonicalize()
    state.synchronize()
    p = state.params
    meta = {
        "format": FORMAT,
        "timestep": int(timestep),
        "model": dataclasses.asdict(state.model),
        "rank": int(state.rank), "nranks": int(state.nranks), "P_local": int(state.P_local),
        "dtype": "f32" if p.dtype == _lib.QG_F32 else "f64",
        "solver": int(p.solver), "precond": int(p.precond), "pcg_rtol": float(p.pcg_rtol),
        "pcg_maxit": int(p.pcg_maxit), "chunk_rows": int(p.chunk_rows), "P_fwd": [float(x) for x in p.P_fwd],
        "wind": [float(p.wind_tau0), float(p.wind_rho0)],
    }
    arrays = {n: getattr(state, n).permute(3, 2, 1, 0).contiguous().cpu().numpy()
              for n in ("zeta", "psi", "f_store")}
    with open(path, "wb") as f:
        np.savez(f, meta=np.array(json.dumps(meta)), **arrays)


def read_checkpoint(path: str):
    """(meta dict, {"zeta", "psi", "f_store"} numpy arrays (M+2, P+2, 2, 3))."""
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z["meta"]))
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} file")
        return meta, {n: z[n] for n in ("zeta", "psi", "f_store")}


def load_checkpoint(path: str, device=None, **overrides):
    """Rebuild the State saved by :func:`save_checkpoint`.  Returns ``(state, next_timestep)``:
    continue with ``state.run(next_timestep, n)`` (after ``comm_init`` on multi-GPU ranks).
    ``overrides`` replace saved State options (e.g. ``solver``)."""
    torch = _torch()
    meta, arrays = read_checkpoint(path)
    m = BaroclinicModel(**meta["model"])
    kw = {"solver": meta["solver"], "precond": meta["precond"], "pcg_rtol": meta["pcg_rtol"],
          "pcg_maxit": meta["pcg_maxit"], "chunk_rows": meta["chunk_rows"], "P_fwd": meta["P_fwd"],
          "P_local": meta["P_local"], "rank": meta["rank"], "nranks": meta["nranks"],
          "dtype": torch.float32 if meta["dtype"] == "f32" else torch.float64}
    if meta.get("wind", [0.0])[0] != 0.0:  # the wind-forcing extension was on
        kw["wind"] = tuple(meta["wind"])
    kw.update(overrides)
    st = State(m, device=device, **kw)
    for n, a in arrays.items():
        t = getattr(st, n)
        if tuple(a.shape[::-1]) != tuple(t.shape):
            raise ValueError(f"{path}: {n} has shape {a.shape}, the model needs {tuple(t.shape[::-1])}")
        t.copy_(torch.from_numpy(np.ascontiguousarray(a.transpose(3, 2, 1, 0))).to(t.dtype))
    st.set_heads([0, 0, 0])
    return st, int(meta["timestep"]) + 1
