"""Exploration: F32 state vs the F64 C oracle (relative RMS per field after k steps)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
import torch, qgamd
from oracle import qg_oracle as O, qg_ref as R
O.build()
for N, steps, dt in ((64, 10, 1800.0), (256, 10, 1800.0), (1024, 10, 1800.0), (128, 48, 1800.0)):
    m = qgamd.bench_model(N, dt=dt)
    st = qgamd.run_model_no_output(m, nsteps=steps, dtype=torch.float32)
    d = qgamd.run_model_no_output(m, nsteps=steps)
    ref = O.State(R.bench_model(N, dt=dt)).run(steps)
    for n in ("psi", "zeta"):
        a = st.to_numpy(n)[:, :, :, 0].astype(np.float64); b = getattr(ref, n)[:, :, :, 0]
        e32 = np.linalg.norm(a - b) / np.linalg.norm(b)
        e64 = np.linalg.norm(d.to_numpy(n)[:, :, :, 0] - b) / np.linalg.norm(b)
        print(f"N={N} steps={steps} {n}: f32 rel {e32:.3e}   f64 rel {e64:.3e}", flush=True)
