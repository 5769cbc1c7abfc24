"""Generate the committed golden fixtures from the scipy oracle (oracle/qg_ref.py).

The reference (Julia) cannot run in this environment, so the fixtures are produced by the
oracle, which is itself pinned to the reference's own known answers (tests/test_oracle_kat.py).
Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import qg_ref as R  # noqa: E402


def run_record(m, record_steps, nsteps):
    snaps = {}

    def cb(t, zeta, psi, f_store):
        if t in record_steps:
            snaps[f"zeta_{t}"] = zeta.copy()
            snaps[f"psi_{t}"] = psi.copy()
            snaps[f"f_store_{t}"] = f_store.copy()

    R.run_model_no_output(m, nsteps=nsteps, callback=cb)
    return snaps


def meta(m, **extra):
    d = {k: getattr(m, k) for k in m.__dataclass_fields__}
    d.update(seeds=[R.SEED_LAYER1, R.SEED_LAYER2], P_matrix="P_matrix(H_1,H_1)", **extra)
    return d


def main():
    out = {}
    # 32x32, full 4-D state after the two Euler steps, the first AB3 step and step 10
    m = R.bench_model(32)
    s = run_record(m, {1, 2, 3, 10}, 10)
    np.savez_compressed(os.path.join(HERE, "qg_32x32.npz"), **s)
    out["qg_32x32.npz"] = meta(m, steps=[1, 2, 3, 10])
    # rectangular 64x32 (M != P), 6 steps
    m = R.bench_model(64, P=32)
    s = run_record(m, {6}, 6)
    np.savez_compressed(os.path.join(HERE, "qg_64x32.npz"), **s)
    out["qg_64x32.npz"] = meta(m, steps=[6])
    # config 1 of BASELINE.json: 128x128, dt = 30 min, T = 1 day = 48 steps; current slot only
    m = R.bench_model(128)
    snaps = {}

    def cb(t, zeta, psi, f_store):
        if t == 48:
            snaps["zeta_48"] = zeta[:, :, :, 0].copy()
            snaps["psi_48"] = psi[:, :, :, 0].copy()

    R.run_model_no_output(m, callback=cb)
    np.savez_compressed(os.path.join(HERE, "qg_128x128_T1day.npz"), **snaps)
    out["qg_128x128_T1day.npz"] = meta(m, steps=[48], slots="current slot only, (M+2,P+2,2)")
    # manufactured-solution known answers (test.jl / scheme_validation.ipynb)
    out["kat"] = {
        "arakawa_slope_notebook": -2.0171,
        "helmholtz_slope_notebook": -2.0495,
        "note": "slopes printed in notebooks/jupyter/scheme_validation.ipynb plot legends",
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
