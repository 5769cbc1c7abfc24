"""The Float32 tendency's two-points-per-thread kernel (`tendency_pair_kernel`, the F32
default) against the one-point kernel it replaces (`tendency_kernel`, selected with
qg_set_form(QG_FORM_TENDENCY, QG_TEND_ONE_POINT)): the same arithmetic in the same order per
point, so every field must be bit-identical after several Euler + AB3 steps.  Grids above the
direct kernel's cut-off (1.2 M points per layer) so the LDS-ring kernels run; M = 1500 leaves a
partial last strip (F32 states need even M), the rows of whole strips run the 5-per-CU kernel,
M = 1024 / 512 with every strip (one) an edge strip."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]


@pytest.mark.parametrize("M,P", [(2048, 1024), (1500, 1024), (1024, 1536), (512, 4096)])
def test_pair_kernel_bitwise_vs_one_point(M, P):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd as qg

    def run():
        st = qg.run_model_no_output(qg.bench_model(M, P=P, dt=600.0), nsteps=5, dtype=torch.float32)
        out = {n: st.to_numpy(n) for n in ("zeta", "psi", "f_store")}
        st.close()
        return out

    pair = run()
    with qg.forced_form(qg._lib.QG_FORM_TENDENCY, qg._lib.QG_TEND_ONE_POINT):
        one = run()
    for n in ("zeta", "psi", "f_store"):
        a, b = pair[n], one[n]
        assert a.shape == b.shape and a.dtype == b.dtype
        assert a.tobytes() == b.tobytes(), (n, M, P, float(np.abs(a.astype(np.float64) - b).max()))
