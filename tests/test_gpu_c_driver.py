"""The C-ABI on its own: a plain-C driver (julia-ocean-modelling_amd/examples/run_no_output.c,
built with gcc against include/qg_mi355.h, HIP runtime memory, no Python / torch) runs
run_model_no_output and must produce BIT-identical zeta and psi to the Python binding on the
same model, for both solvers."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "julia-ocean-modelling_amd")


@pytest.fixture(scope="module")
def driver():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    subprocess.run(["make", "-s", "-C", PKG, "examples"], check=True)
    return os.path.join(PKG, "build", "run_no_output")


@pytest.mark.parametrize("M,P,steps,solver", [(64, 64, 20, 0), (96, 32, 7, 0), (64, 48, 6, 1)])
def test_c_driver_matches_python_binding(driver, tmp_path, M, P, steps, solver):
    import qgamd
    out = tmp_path / "state.bin"
    r = subprocess.run([driver, str(M), str(P), str(steps), str(solver), str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    raw = np.fromfile(out, dtype=np.float64).reshape(2, 2, P + 2, M + 2)  # [zeta|psi][layer][j][i]
    st = qgamd.run_model_no_output(qgamd.bench_model(M, P=P), nsteps=steps, solver=solver)
    z = st.to_numpy("zeta")[:, :, :, 0]
    p = st.to_numpy("psi")[:, :, :, 0]
    assert np.array_equal(raw[0].transpose(2, 1, 0), z)
    assert np.array_equal(raw[1].transpose(2, 1, 0), p)
    d = st.diagnostics()
    assert rec["psi_max"] == d["psi_max"] and rec["zeta_sum"] == d["zeta_sum"]
    if solver == 1:
        assert rec["pcg_iters"][0] >= 1
