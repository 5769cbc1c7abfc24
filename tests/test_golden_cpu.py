"""The C oracle reproduces the committed golden fixtures (made by the scipy oracle)."""
import json
import os

import numpy as np
import pytest

from oracle import qg_oracle as O
from oracle import qg_ref as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def test_golden_32x32_full_state():
    g = np.load(os.path.join(GOLDEN, "qg_32x32.npz"))
    st = O.State(R.bench_model(32))
    for t in (1, 2, 3, 10):
        st.run(t - st.t)
        for name, arr in (("psi", st.psi), ("zeta", st.zeta), ("f_store", st.f_store)):
            assert _rel(arr, g[f"{name}_{t}"]) < 1e-12, (name, t)


def test_golden_rectangular():
    g = np.load(os.path.join(GOLDEN, "qg_64x32.npz"))
    st = O.State(R.bench_model(64, P=32)).run(6)
    assert _rel(st.psi, g["psi_6"]) < 1e-12
    assert _rel(st.zeta, g["zeta_6"]) < 1e-12


def test_golden_128_one_day():
    g = np.load(os.path.join(GOLDEN, "qg_128x128_T1day.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))["qg_128x128_T1day.npz"]
    m = R.bench_model(128)
    assert int(np.floor(m.T / m.dt)) == meta["steps"][0] == 48
    st = O.State(m).run(48)
    assert _rel(st.psi[:, :, :, 0], g["psi_48"]) < 1e-12
    assert _rel(st.zeta[:, :, :, 0], g["zeta_48"]) < 1e-12
