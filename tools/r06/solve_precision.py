"""How far each F64 solver is from the exact solution of the same F64 input:
the C oracle's DFT solve and (with --device) the device's spectral solve, against the
long-double DFT solve of oracle/qg_ref.solve_longdouble, for the pinned Poisson and the
Helmholtz systems of evolve_psi! on white-noise right-hand sides of long grids.
usage: python tools/r06/solve_precision.py [--device] M:P [M:P ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
from oracle import qg_oracle as O  # noqa: E402
from oracle import qg_ref as R  # noqa: E402


def rel(a, b):
    b = np.asarray(b, dtype=np.longdouble)
    return float(np.linalg.norm((np.asarray(a, dtype=np.longdouble) - b)[1:-1, 1:-1]) /
                 np.linalg.norm(b[1:-1, 1:-1]))


def main():
    dev = "--device" in sys.argv
    grids = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:] if ":" in a]
    if dev:
        import torch
        import qgamd
    for M, P in grids:
        dx = 4e6 / M
        f = R.update_doubly_periodic_bc(R.seeded_rand(M, P, 17) - 0.5) * 1e-9
        for name, alpha, pinned in (("poisson", 0.0, True), ("helmholtz", -6.25e-10, False)):
            t0 = time.time()
            x = R.solve_longdouble(M, P, dx, alpha, f, pinned=pinned, workers=os.cpu_count())
            tl = time.time() - t0
            xc = O.solve(M, P, dx, alpha, f, pinned=pinned)
            line = f"{M}x{P} {name:9s} C-oracle {rel(xc, x):.3e}"
            if dev:
                t = torch.from_numpy(np.ascontiguousarray(f.T)).cuda()
                xd = (qgamd.sp_solve_poisson(M, P, dx, t) if pinned else
                      qgamd.sp_solve_modified_helmholtz(M, P, dx, t, alpha)).cpu().numpy().T
                line += f"  device {rel(xd, x):.3e}  device-vs-C {rel(xd, xc):.3e}"
            print(line + f"  (long double {tl:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
