"""qgamd -- MI355X-native two-layer Phillips (baroclinic QG) hot path.

Host mirror of the reference's operator surface (src/model.jl, src/schemes/*.jl,
src/run_model_no_output.jl of JSLeadbetter/julia-ocean-modelling) over the HIP C-ABI in
include/qg_mi355.h.  See model.py for the mapping.
"""
from . import _lib
from ._lib import LIB_PATH, QGError, lib
from .model import *  # noqa: F401,F403
from .model import (BaroclinicModel, PairSolver, State, bench_model, cd, device_zeros,
                    evolve_psi_, evolve_zeta_, get_helmholtz_cholesky, get_poisson_cholesky,
                    initialise_model, J, laplace_5p, make_model, run_model_no_output,
                    set_dropin_slots, sp_solve_modified_helmholtz, sp_solve_poisson, unbind,
                    update_doubly_periodic_bc_)
from .checkpoint import load_checkpoint, read_checkpoint, save_checkpoint
from .run import SnapshotWriter, create_metadata, log_model_params, run_model, update_max, update_min

__all__ = ["BaroclinicModel", "PairSolver", "State", "bench_model", "cd", "device_zeros",
           "evolve_psi_", "evolve_zeta_", "get_helmholtz_cholesky", "get_poisson_cholesky",
           "initialise_model", "J", "laplace_5p", "make_model", "run_model_no_output", "set_dropin_slots",
           "sp_solve_modified_helmholtz", "sp_solve_poisson", "unbind", "update_doubly_periodic_bc_",
           "run_model", "update_max", "update_min", "create_metadata", "log_model_params", "SnapshotWriter",
           "save_checkpoint", "load_checkpoint", "read_checkpoint", "LIB_PATH", "QGError", "lib"]
