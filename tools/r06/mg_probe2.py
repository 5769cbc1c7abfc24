"""MG-PCG convergence curve of the first solve (relres after k iterations, k = maxit) for one
GPU and G slabs: a floor or an oscillation shows where the slab cycle departs from the global."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
import torch  # noqa: E402
import qgamd  # noqa: E402
from qgamd.hostcomm import ThreadRing  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
STEPS = int(sys.argv[3]) if len(sys.argv) > 3 else 1
KS = [int(x) for x in (sys.argv[4].split(",") if len(sys.argv) > 4 else "4,8,10,12,14,16,20,30")]
for G in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "1,2,4")]:
    row = []
    for k in KS:
        m = qgamd.bench_model(N)
        Pl = N // G
        ring = ThreadRing(G) if G > 1 else None
        ranks = []
        for r in range(G):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                st = qgamd.State(m, P_local=Pl, solver=1, precond=2, pcg_rtol=1e-30, pcg_maxit=k)
            if ring:
                ring.attach(st, r)
            ranks.append((st, s))
        out = [None] * G

        def work(r):
            st, s = ranks[r]
            with torch.cuda.stream(s):
                st.initialise()
                out[r] = []
                for t in range(1, STEPS + 1):
                    try:
                        st.step(t)
                    except qgamd.QGError:
                        pass
                    out[r].append(st.stats())

        if ring:
            ThreadRing.run_all([lambda r=r: work(r) for r in range(G)])
        else:
            work(0)
        row.append("|".join(f"{x['iters'][0]}:{x['relres'][0]:.1e}/{x['relres'][1]:.1e}" for x in out[0]))
        del ranks
        torch.cuda.synchronize()
    print(f"N {N} G {G}: " + "  ".join(row), flush=True)
