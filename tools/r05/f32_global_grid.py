"""Config 5's global grid (8192 x 65536) on ONE GPU: the F32 state against the F64 path after 3
steps (white-noise field), the yardstick for the 8-slab-vs-one-GPU F32 comparison of
tests/test_gpu_rccl_multirank.py (two F32 runs can differ by up to the sum of their distances
to the F64 result)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd


def rel(a, b):
    d = torch.linalg.vector_norm((a.double() - b.double()).reshape(-1))
    return float(d / torch.linalg.vector_norm(b.double().reshape(-1)))


N, G, steps = 8192, 8, 3
m = qgamd.bench_model(N, P=G * N, dt=60.0)
a = qgamd.run_model_no_output(m, nsteps=steps)
torch.cuda.synchronize()
ref = {n: [a.current(n, l).cpu() for l in (1, 2)] for n in ("psi", "zeta")}
del a
torch.cuda.empty_cache()
b = qgamd.run_model_no_output(m, nsteps=steps, dtype=torch.float32)
torch.cuda.synchronize()
e = {n: [rel(b.current(n, l).cpu(), ref[n][l - 1]) for l in (1, 2)] for n in ("psi", "zeta")}
print(f"{N} x {G * N}, {steps} steps, F32 vs F64 on one GPU: psi {e['psi']}, zeta {e['zeta']}")
