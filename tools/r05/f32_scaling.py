"""How the F32 state's error against the F64 path grows with the grid (white-noise initial
field, the reference's rand; bench parameters, dt = 60 s, 10 steps): relative RMS of psi and
zeta (slot 1, both layers) for M = 256 ... 8192, square grids.  The DESIGN §4 model: zeta
carries ~eps_32 relative rounding; psi = A^-1 zeta amplifies it in the gravest modes
relative to the grid-scale energy of white noise by ~(M / 2 pi)^2 / (spectral weight), so the
psi error should grow ~ M^2 until it saturates.  Prints one line per M and the fitted slope."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd


def rel(a, b):
    d = torch.linalg.vector_norm((a.double() - b.double()).reshape(-1))
    return float(d / torch.linalg.vector_norm(b.double().reshape(-1)))


steps = 10
rows = []
for M in (256, 512, 1024, 2048, 4096, 8192):
    m = qgamd.bench_model(M, dt=60.0)
    a = qgamd.run_model_no_output(m, nsteps=steps)
    b = qgamd.run_model_no_output(m, nsteps=steps, dtype=torch.float32)
    torch.cuda.synchronize()
    e = {n: max(rel(b.current(n, l), a.current(n, l)) for l in (1, 2)) for n in ("psi", "zeta")}
    rows.append((M, e["psi"], e["zeta"]))
    print(f"M {M:5d}  psi {e['psi']:.3e}  zeta {e['zeta']:.3e}  psi / (eps32 (M/2pi)^2) {e['psi'] / (2 ** -24 * (M / (2 * math.pi)) ** 2):.3e}", flush=True)
    del a, b
    torch.cuda.empty_cache()
xs = [math.log(r[0]) for r in rows]
for k, name in ((1, "psi"), (2, "zeta")):
    ys = [math.log(r[k]) for r in rows]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    print(f"{name}: log-log slope vs M = {slope:.2f}")
