"""Residuals of the Bluestein-row solve for a list of sizes (diagnostic for r05)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd"), os.path.join(ROOT, "tests")]
import qgamd as qg
from oracle import qg_ref as R
from test_gpu_edge import modal_residuals
for M, P in [(20000, 2), (50001, 4), (40000, 4), (32769, 4), (50000, 4), (33000, 4), (70000, 2)]:
    st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=60.0), nsteps=2)
    m = R.bench_model(M, P=P, dt=60.0)
    print(M, P, modal_residuals(R, m, st.to_numpy("zeta"), st.to_numpy("psi")), flush=True)
