"""Phase timing of spec_carry from a stamp build (tools/stamps/add_stamps_carry.py ->
lib/exp/stampC.so; not part of the product).  usage: stamps_carry.py M f32|f64"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd

M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dt = torch.float32 if (len(sys.argv) > 2 and sys.argv[2] == "f32") else torch.float64
st = qgamd.run_model_no_output(qgamd.bench_model(M, dt=60.0), nsteps=6, dtype=dt)
torch.cuda.synchronize()
L = qgamd._lib.lib()
NS = 1024 * 8
buf = (C.c_ulonglong * NS)()
assert L.qg_debug_stamps(buf, NS) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
nwg = int((a[:, 0] > 0).sum())
a = a[:nwg]
us = lambda x: x / 100.0
t0 = a[:, 0].min()
reg = a[:, 1] > 0
print("M", M, dt, "workgroups", nwg, "regular", int(reg.sum()))
print("kernel span us %.1f" % us(a[:, 6].max() - t0))
st_ = a[:, 0] - t0
print("start us: median %.2f max %.2f; late starters (> 5 us): %d" % (us(np.median(st_)), us(st_.max()), int((st_ > 500).sum())))
names = ["summaries arrive", "segment combine", "backward pass", "forward pass", "closure", "store drain"]
r = a[reg]
for k, n in enumerate(names):
    d = r[:, k + 1] - r[:, k]
    print("%-18s median %.2f us  max %.2f" % (n, us(np.median(d)), us(d.max())))
ex = a[~reg]
for i in range(len(ex)):
    print("extra-column workgroup: start %.2f us, duration %.2f us" % (us(ex[i, 0] - t0), us(ex[i, 6] - ex[i, 0])))
tot = a[:, 6] - a[:, 0]
print("workgroup duration us: median %.2f max %.2f" % (us(np.median(tot)), us(tot.max())))
