"""The Float32 tendency's two-points-per-thread kernel (`tendency_pair_kernel`, the F32
default) against the one-point kernel it replaces (`tendency_kernel`, QG_TEND_PAIR=0): the
same arithmetic in the same order per point, so every field must be bit-identical after
several Euler + AB3 steps.  Grids above the direct kernel's cut-off (1.2 M points per layer)
so the LDS-ring kernels run; M = 1500 leaves a partial last strip (F32 states need even M), the
rows of whole strips run the 5-per-CU kernel, M = 1024 / 512 with every strip (one) an edge strip.  The kernel choice
is read once per process, so each variant runs in its own child process."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = """
import sys, numpy as np, torch
sys.path.insert(0, {pkg!r})
import qgamd
M, P, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
st = qgamd.run_model_no_output(qgamd.bench_model(M, P=P, dt=600.0), nsteps=5, dtype=torch.float32)
np.savez(out, **{{n: st.to_numpy(n) for n in ("zeta", "psi", "f_store")}})
"""


@pytest.mark.parametrize("M,P", [(2048, 1024), (1500, 1024), (1024, 1536), (512, 4096)])
def test_pair_kernel_bitwise_vs_one_point(M, P, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    code = CHILD.format(pkg=os.path.join(ROOT, "julia-ocean-modelling_amd"))
    res = {}
    for pair in ("1", "0"):
        env = dict(os.environ, QG_TEND_PAIR=pair)
        out = tmp_path / f"pair{pair}.npz"
        r = subprocess.run([sys.executable, "-c", code, str(M), str(P), str(out)], env=env,
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res[pair] = np.load(out)
    for n in ("zeta", "psi", "f_store"):
        a, b = res["1"][n], res["0"][n]
        assert a.shape == b.shape and a.dtype == b.dtype
        assert a.tobytes() == b.tobytes(), (n, M, P, float(np.abs(a.astype(np.float64) - b).max()))
