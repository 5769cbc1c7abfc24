"""Phase timing from a stamp build (not part of the product): the wide-row pass A
(tools/stamps/add_stamps_half.py -> lib/exp/stampAH.so) or the 4096-point pass B
(add_stamps_pb4k.py -> lib/exp/stampB4.so).  Runs M^2 for a few steps and prints per-phase
medians over workgroups and rows.  usage: stamps_phases.py M f32|f64 A|B"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "julia-ocean-modelling_amd"))
import qgamd

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dt = torch.float32 if (len(sys.argv) < 3 or sys.argv[2] == "f32") else torch.float64
m = qgamd.bench_model(M, dt=60.0)
st = qgamd.run_model_no_output(m, nsteps=6, dtype=dt)
torch.cuda.synchronize()
L = qgamd._lib.lib()
NS = 1024 * 256
buf = (C.c_ulonglong * NS)()
assert L.qg_debug_stamps(buf, NS) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 256).astype(np.int64)
nwg = int((a[:, 0] > 0).sum())
a = a[:nwg]
rows = int(((a[0, 2:162] > 0).sum()) // 5)
t0 = a[:, 0].min()
us = lambda x: x / 100.0  # wall_clock64: 100 MHz
print("M", M, dt, "workgroups", nwg, "rows per workgroup", rows)
print("kernel span us %.1f" % us(a[:, 255].max() - t0))
print("start us: median %.2f max %.2f (two rounds of workgroups when > 256)" % (us(np.median(a[:, 0] - t0)), us((a[:, 0] - t0).max())))
print("set-up us: median %.2f" % us(np.median(a[:, 1] - a[:, 0])))
kind = sys.argv[3] if len(sys.argv) > 3 else "A"
names = (["wait+projection", "stage1+T1 write", "transform rest", "split+recurrence+stores", "to next row"]
         if kind == "A" else ["u wait+convert", "recurrence (coef wait)", "exchange+transform", "stores+coef issue",
                              "to next row"])
ph = np.zeros((nwg, rows, 5))
for r in range(rows):
    b = 2 + 5 * r
    for k in range(4):
        ph[:, r, k] = a[:, b + k + 1] - a[:, b + k]
    nxt = a[:, b + 5] if r + 1 < rows else a[:, 255]
    ph[:, r, 4] = nxt - a[:, b + 4]
for k, n in enumerate(names):
    per_row = np.median(ph[:, :, k], axis=0)
    print("%-24s median %.2f us  (rows 0-3: %s, last: %.2f)" % (n, us(np.median(ph[:, 1:, k])), np.round(us(per_row[:4]), 2), us(per_row[-1])))
tot = us(np.median(ph[:, 1:, :].sum(axis=2)))
print("row total median %.2f us" % tot)
print("tail (after last row, store drain) us: median %.2f" % us(np.median(a[:, 255] - a[:, 2 + 5 * (rows - 1) + 4])))
