"""run_model with snapshot output (src/run_model.jl:55-95) on the GPU: the file holds the
reference's keys (zeta_0, psi_0, metadata, zeta_$t, psi_$t every 2*floor(DAY/dt) steps),
each snapshot equals the C oracle's state after that many steps (relative RMS < 1e-10;
the initial conditions bit for bit), and the time loop is not changed by snapshotting."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-10


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    from oracle import qg_oracle, qg_ref
    qg_oracle.build()
    return torch, qgamd, qg_oracle, qg_ref


@pytest.mark.parametrize("N,P", [(32, 24), (64, 64)])
def test_run_model_snapshots_match_oracle(env, tmp_path, N, P):
    torch, qg, O, R = env
    dt, T = 21600.0, 4 * qg.model.DAY  # sample every 2*floor(DAY/dt) = 8 steps; 16 steps
    m = qg.bench_model(N, dt=dt, T=T, P=P)
    path = tmp_path / "run.npz"
    lines = []
    st = qg.run_model(m, str(path), True, log=lines.append)
    assert lines[0] == "Parameters:" and "Total steps = 16\n" in lines
    data = np.load(path)  # no pickles
    assert sorted(data.files) == sorted(["metadata", "zeta_0", "psi_0", "zeta_8", "psi_8", "zeta_16", "psi_16"])
    md = json.loads(str(data["metadata"]))
    assert md == {"dt": dt, "T": T, "sample_interval": 86400.0, "sample_timestep": 4, "total_steps": 16}
    rm = R.bench_model(N, dt=dt, T=T, P=P)
    for t in (0, 8, 16):
        ref = O.State(rm).run(t)
        z, p = data[f"zeta_{t}"], data[f"psi_{t}"]
        assert z.shape == (N + 2, P + 2, 2)
        if t == 0:
            assert np.array_equal(p, ref.psi[:, :, :, 0]) and np.array_equal(z, ref.zeta[:, :, :, 0])
        else:
            assert rel(p, ref.psi[:, :, :, 0]) < TOL and rel(z, ref.zeta[:, :, :, 0]) < TOL
    # the returned state is the last step's, identical to a run without output
    assert np.array_equal(st.to_numpy("psi")[:, :, :, 0], data["psi_16"])
    plain = qg.run_model_no_output(m)
    assert np.array_equal(plain.to_numpy("psi"), st.to_numpy("psi"))


def test_run_model_without_output(env, tmp_path):
    torch, qg, O, R = env
    m = qg.bench_model(32, dt=21600.0, T=2 * qg.model.DAY)
    path = tmp_path / "none.npz"
    st = qg.run_model(m, str(path), False, log=lambda s: None)
    assert not path.exists()
    ref = O.State(R.bench_model(32, dt=21600.0, T=2 * qg.model.DAY)).run(8)
    assert rel(st.to_numpy("psi"), ref.psi) < TOL
