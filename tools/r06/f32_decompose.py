"""F32 state vs F64 decomposition probe; the model is tests/f32_model.py.
usage: python tools/r06/f32_decompose.py M P_total steps [mc]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd"), os.path.join(ROOT, "tests")]
from f32_model import EPS32, decompose  # noqa: E402


def main():
    import torch
    import qgamd
    M, P, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    mc = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    m = qgamd.bench_model(M, P=P, dt=60.0)
    r = decompose(qgamd, torch, m, steps, mc)
    for k, v in r.items():
        if isinstance(v, list):
            v = "[" + ", ".join(f"{x:.3e}" for x in v) + "]"
        elif isinstance(v, float):
            v = f"{v:.3e}"
        print(f"{k:16s} {v}")
    print(f"eps32 = {EPS32:.3e}; psi_err / eps32 = {r['psi_err'] / EPS32:.1f}, "
          f"e_solve / eps32 = {r['e_solve'] / EPS32:.1f}, zeta_err / eps32 = {r['zeta_err'] / EPS32:.1f}")


if __name__ == "__main__":
    main()
