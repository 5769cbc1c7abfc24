"""Steps/s of qg_run (graph replay of AB3 steps) against a qg_step loop, per grid size
(single GPU, F64, spectral).  usage: python tools/graph_bench.py [N ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
os.environ["QG_GRAPH"] = "1"
import torch  # noqa: E402
import qgamd  # noqa: E402

for n in [int(x) for x in sys.argv[1:]] or [128, 256, 512, 1024, 2048, 4096]:
    K = max(60, min(3000, int(3e9 / (n * n * 160))))
    K -= K % 3
    st = qgamd.State(qgamd.bench_model(n, dt=60.0)).initialise()
    st.run(1, 30)  # (captures the graphs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(31, 31 + K):
        st.step(t)
    torch.cuda.synchronize()
    t_step = (time.perf_counter() - t0) / K
    st.run(31 + K, K)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.run(31 + 2 * K, K)
    torch.cuda.synchronize()
    t_run = (time.perf_counter() - t0) / K
    print(json.dumps({"n": n, "steps": K, "step_loop_steps_per_s": 1 / t_step, "run_graph_steps_per_s": 1 / t_run,
                      "speedup": t_step / t_run}), flush=True)
