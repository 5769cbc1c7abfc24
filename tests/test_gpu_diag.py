"""qg_diagnostics (include/qg_mi355.h) on the GPU: the update_max / update_min of
run_model.jl:41-53 and the monitoring sums, against oracle.qg_ref.diagnostics on the same
device state; circulation conservation over a long run; the run_model monitor hook.
Max / min are exact (the same values); sums differ only by summation order (rel 1e-12)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    from oracle import qg_ref
    return torch, qgamd, qg_ref


def _check(diag, want):
    for k, v in want.items():
        got = np.atleast_1d(diag[k])
        v = np.atleast_1d(v)
        if k.endswith("_max") or k.endswith("_min"):
            assert np.array_equal(got, v), (k, got, v)
        else:
            np.testing.assert_allclose(got, v, rtol=1e-12, atol=0, err_msg=k)


@pytest.mark.parametrize("M,P,steps,dtype", [(64, 64, 7, "f64"), (32, 48, 3, "f64"), (128, 64, 12, "f64"),
                                             (64, 64, 5, "f32")])
def test_diagnostics_match_oracle(env, M, P, steps, dtype):
    torch, qgamd, qg_ref = env
    kw = {} if dtype == "f64" else {"dtype": torch.float32}
    st = qgamd.run_model_no_output(qgamd.bench_model(M, P=P), nsteps=steps, **kw)
    d = st.diagnostics()
    z = st.to_numpy("zeta").astype(np.float64)
    p = st.to_numpy("psi").astype(np.float64)
    _check(d, qg_ref.diagnostics(z, p, st.model.dx))


def test_diagnostics_after_initialise_only(env):
    torch, qgamd, qg_ref = env
    st = qgamd.initialise_model(qgamd.bench_model(64))
    z, p = st.to_numpy("zeta"), st.to_numpy("psi")
    _check(st.diagnostics(), qg_ref.diagnostics(z, p, st.model.dx))


def test_circulation_conserved(env):
    """Every term of zeta_f1 / zeta_f2 (model.jl:139-153) sums to zero over the periodic grid
    (Arakawa J, the 5-point Laplacians, the centred x-differences), so sum(zeta) dx^2 changes
    only by roundoff over a long run, while enstrophy and energy change."""
    torch, qgamd, _ = env
    st = qgamd.initialise_model(qgamd.bench_model(128))
    d0 = st.diagnostics()
    z = st.to_numpy("zeta")[1:-1, 1:-1, :, 0]
    scale = np.abs(z).sum(axis=(0, 1)) * st.model.dx ** 2
    st.run(1, 300)
    d1 = st.diagnostics()
    for l in range(2):
        assert abs(d1["zeta_sum"][l] - d0["zeta_sum"][l]) < 1e-11 * scale[l], (l, d0, d1)
        assert d1["enstrophy"][l] != d0["enstrophy"][l]


def test_run_model_monitor(env, tmp_path):
    torch, qgamd, _ = env
    m = qgamd.bench_model(32, dt=21600.0, T=4 * 86400.0)  # sample_timestep = 2*floor(DAY/dt) = 8
    seen = []
    qgamd.run_model(m, str(tmp_path / "out.npz"), False, log=lambda *a: None,
                    monitor=lambda t, d: seen.append((t, qgamd.update_max(-np.inf, d["psi_max"][0]))))
    assert [t for t, _ in seen] == [0, 8, 16]
    assert all(np.isfinite(v) for _, v in seen)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_nan_propagates_to_extrema(env, dtype):
    """A diverged state must not report finite extrema: Julia's maximum / minimum (what
    update_max / update_min of run_model.jl:41-53 fold) return NaN when the matrix holds one."""
    torch, qgamd, _ = env
    kw = {} if dtype == "f64" else {"dtype": torch.float32}
    st = qgamd.initialise_model(qgamd.bench_model(64, P=48), **kw)
    st.current("zeta", 2)[17, 23] = float("nan")  # layer 2 only
    st.synchronize()
    d = st.diagnostics()
    assert np.isnan(d["zeta_max"][1]) and np.isnan(d["zeta_min"][1])
    assert np.isfinite(d["zeta_max"][0]) and np.isfinite(d["zeta_min"][0])
    assert np.all(np.isfinite(d["psi_max"])) and np.all(np.isfinite(d["psi_min"]))
