"""Plain CG (QG_PRECOND_NONE) at 256^2: relres target vs the reached residual, iterations and the
psi error against the C oracle after 2 steps -- the measurement behind test_plain_cg_256's bar."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
import qgamd as qg  # noqa: E402
from oracle import qg_oracle as O, qg_ref as R  # noqa: E402

O.build()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ref = O.State(R.bench_model(N)).run(2)
for rtol in (1e-12, 1e-13, 1e-14, 3e-15, 1e-15):
    st = qg.initialise_model(qg.bench_model(N), solver=1, precond=0, pcg_rtol=rtol, pcg_maxit=6000)
    its = []
    for t in (1, 2):
        try:
            st.step(t)
            ok = "ok"
        except qg.QGError as e:
            ok = f"status {e.status}"
        s = st.stats()
        its.append((s["iters"], s["relres"], ok))
    torch.cuda.synchronize()
    ep = np.linalg.norm(st.to_numpy("psi")[:, :, :, 0] - ref.psi[:, :, :, 0]) / np.linalg.norm(ref.psi[:, :, :, 0])
    ez = np.linalg.norm(st.to_numpy("zeta")[:, :, :, 0] - ref.zeta[:, :, :, 0]) / np.linalg.norm(ref.zeta[:, :, :, 0])
    print(f"N {N} rtol {rtol:.0e}: steps {its}  psi err {ep:.3e}  zeta err {ez:.3e}", flush=True)
