"""Phase timing of spec_passB<4096> from a stamp build (tools/stamps/add_stamps.py -> lib/exp/stampB.so, built from
a copy of csrc with wall_clock64 stamps; not part of the product).  Prints per-phase medians."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd

M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
st = qgamd.run_model_no_output(qgamd.bench_model(M), nsteps=12)
torch.cuda.synchronize()
L = qgamd._lib.lib()
buf = (C.c_ulonglong * (1024 * 64))()
assert L.qg_debug_stamps(buf, 1024 * 64) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64).astype(np.int64)
nwg = int((a[:, 0] > 0).sum())
a = a[:nwg]
rows = 16
t0 = a[:, 0].min()
print("workgroups", nwg, "kernel span us", (a[:, 63].max() - t0) / 100.0)
print("start skew us: median %.2f max %.2f" % (np.median(a[:, 0] - t0) / 100, (a[:, 0] - t0).max() / 100))
print("head (set-up) us: median %.2f max %.2f" % (np.median(a[:, 1] - a[:, 0]) / 100, (a[:, 1] - a[:, 0]).max() / 100))
prev = a[:, 1]
rec, fft, sto = [], [], []
for r in range(rows):
    x2, x3, x4 = a[:, 2 + 3 * r], a[:, 3 + 3 * r], a[:, 4 + 3 * r]
    rec.append(np.median(x2 - prev)); fft.append(np.median(x3 - x2)); sto.append(np.median(x4 - x3))
    prev = x4
print("per row us (median over wgs): recurrence+wait", np.round(np.array(rec) / 100, 2))
print("  fft", np.round(np.array(fft) / 100, 2))
print("  store issue", np.round(np.array(sto) / 100, 2))
print("tail (store drain) us: median %.2f" % (np.median(a[:, 63] - prev) / 100))
print("end skew us: median %.2f max %.2f" % (np.median(a[:, 63] - t0) / 100, (a[:, 63] - t0).max() / 100))
