"""MG-PCG iteration counts and residuals per step: one GPU vs G slabs (ThreadRing), two targets."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
import torch  # noqa: E402
import qgamd  # noqa: E402
from qgamd.hostcomm import ThreadRing  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = 3
for rtol in (1e-12, 1e-13):
    for G in (1, 2, 4, 8):
        m = qgamd.bench_model(N)
        Pl = N // G
        ring = ThreadRing(G) if G > 1 else None
        ranks = []
        for r in range(G):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                st = qgamd.State(m, P_local=Pl, solver=1, precond=2, pcg_rtol=rtol, pcg_maxit=300)
            if ring:
                ring.attach(st, r)
            ranks.append((st, s))
        log = [[] for _ in range(G)]

        def work(r):
            st, s = ranks[r]
            with torch.cuda.stream(s):
                st.initialise()
                for t in range(1, steps + 1):
                    st.step(t)
                    x = st.stats()
                    log[r].append((x["iters"][0], max(x["relres"])))
                st.synchronize()

        if ring:
            ThreadRing.run_all([lambda r=r: work(r) for r in range(G)])
        else:
            work(0)
        print(f"N {N} rtol {rtol:.0e} G {G}: " + ", ".join(f"{k} ({e:.1e})" for k, e in log[0]), flush=True)
