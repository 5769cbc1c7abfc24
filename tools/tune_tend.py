"""Time the tendency kernel (qg_evolve_zeta) and the solve at N^2 for the strip tile given as
"WxR" (qg_set_form(QG_FORM_TENDENCY_TILE, (W << 16) | R); tuning helper, not part of the
product).  usage: python tools/tune_tend.py [N] [WxR]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
import torch
import qgamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
tile = sys.argv[2] if len(sys.argv) > 2 else ""
if tile:
    w, r = (int(x) for x in tile.split("x"))
    qgamd.set_form(qgamd._lib.QG_FORM_TENDENCY_TILE, (w << 16) | r)
K = 20
dtype = torch.float32 if os.environ.get("QG_TUNE_DTYPE") == "f32" else torch.float64
st = qgamd.State(qgamd.bench_model(n, dt=60.0), dtype=dtype).initialise()
for t in range(1, 6):
    st.step(t)
torch.cuda.synchronize()
ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
t = 6
for k in range(K):
    ev[k][0].record(); st.evolve_zeta_(t); ev[k][1].record(); st.evolve_psi_(); ev[k][2].record(); t += 1
torch.cuda.synchronize()
tz = sorted(e[0].elapsed_time(e[1]) for e in ev)
tp = sorted(e[1].elapsed_time(e[2]) for e in ev)
gb = (96 if dtype == torch.float64 else 48) * n * n / 1e9
import hashlib
zsha = hashlib.sha1(st.to_numpy("zeta").tobytes()).hexdigest()
print(json.dumps({"zeta_sha1": zsha, "tile": tile, "tend_ms_med": tz[K // 2], "tend_ms_min": tz[0],
                  "tend_TBs": gb / tz[K // 2], "solve_ms_med": tp[K // 2]}))
