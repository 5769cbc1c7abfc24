"""Checkpoint / resume (qgamd.checkpoint): a run saved after step k and
resumed in a fresh State continues BIT FOR BIT like the uninterrupted run -- every slot of
zeta, psi and f_store -- across the Euler -> AB3 switch (k = 1, 2) and later, for both
solvers and the F32 state."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def qg():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import qgamd
    return qgamd


def _all(st):
    return {n: st.to_numpy(n) for n in ("zeta", "psi", "f_store")}


@pytest.mark.parametrize("k,solver,dtype", [(1, 0, "f64"), (2, 0, "f64"), (9, 0, "f64"), (3, 1, "f64"),
                                            (5, 0, "f32")])
def test_resume_is_bitwise(qg, tmp_path, k, solver, dtype):
    import torch
    total = 14
    m = qg.bench_model(64, P=48)
    kw = {"solver": solver}
    if dtype == "f32":
        kw["dtype"] = torch.float32
    straight = qg.run_model_no_output(m, nsteps=total, **kw)
    want = _all(straight)

    a = qg.initialise_model(m, **kw)
    a.run(1, k)
    a.step(k + 1)  # leave the slot rotation non-canonical before saving
    path = str(tmp_path / "ck.npz")
    qg.save_checkpoint(a, path, k + 1)
    del a
    b, t = qg.load_checkpoint(path)
    assert t == k + 2 and b.heads() == [0, 0, 0] and b.dtype == straight.dtype
    b.run(t, total - t + 1)
    got = _all(b)
    for n in want:
        assert np.array_equal(got[n], want[n]), n


def test_checkpoint_contents(qg, tmp_path):
    m = qg.bench_model(32)
    st = qg.run_model_no_output(m, nsteps=4)
    want = _all(st)
    path = str(tmp_path / "ck.npz")
    qg.save_checkpoint(st, path, 4)
    meta, arr = qg.read_checkpoint(path)
    assert meta["timestep"] == 4 and meta["model"]["M"] == 32 and meta["P_fwd"] == [1.0, -1.0, 1.0, 1.0]
    for n in want:  # reference slot order, Julia index order (M+2, P+2, 2, 3)
        assert arr[n].shape == (34, 34, 2, 3)
        assert np.array_equal(arr[n], want[n])
    with np.load(path, allow_pickle=False) as z:  # plain arrays: loadable without pickling
        assert set(z.files) == {"meta", "zeta", "psi", "f_store"}
