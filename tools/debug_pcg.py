import os, sys, numpy as np, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), 'julia-ocean-modelling_amd')]
import qgamd
st = qgamd.initialise_model(qgamd.bench_model(64), solver=1, precond=1, pcg_maxit=20)
for t in range(1, 7):
    try:
        st.step(t); ok = True
    except qgamd.QGError:
        ok = False
    print(t, ok, st.stats(), flush=True)
