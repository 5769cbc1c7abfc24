import sys, torch
sys.path.insert(0, 'julia-ocean-modelling_amd')
import qgamd
m = qgamd.bench_model(8192, dt=60.0)
st = qgamd.State(m, dtype=torch.float32)
st.initialise()
st.run(1, 6)
torch.cuda.synchronize()
