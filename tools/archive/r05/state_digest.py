"""sha256 of zeta / psi after a few steps (library from QGMI355_LIB): compares two builds bit for
bit.  usage: state_digest.py M f32|f64 [steps]"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd

M = int(sys.argv[1])
dt = torch.float32 if sys.argv[2] == "f32" else torch.float64
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
st = qgamd.run_model_no_output(qgamd.bench_model(M, dt=60.0), nsteps=steps, dtype=dt)
torch.cuda.synchronize()
h = hashlib.sha256()
for x in (st.zeta, st.psi):
    h.update(x.detach().cpu().numpy().tobytes())
print(M, sys.argv[2], steps, h.hexdigest()[:32])
