"""P = 2 slabs: device vs the C oracle and the modal residuals (diagnostic for r05)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd"), os.path.join(ROOT, "tests")]
import qgamd as qg
from oracle import qg_ref as R, qg_oracle as O
from test_gpu_edge import modal_residuals
def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))
for M, P in [(8, 2), (64, 2), (5000, 2), (8192, 2), (16384, 2), (20000, 2), (20000, 3)]:
    st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=60.0), nsteps=2)
    ref = O.State(R.bench_model(M, P=P, dt=60.0)).run(2)
    m = R.bench_model(M, P=P, dt=60.0)
    print(M, P, "psi vs oracle", rel(st.to_numpy("psi"), ref.psi), "dev res", modal_residuals(R, m, st.to_numpy("zeta"), st.to_numpy("psi")),
          "oracle res", modal_residuals(R, m, ref.zeta, ref.psi), flush=True)
