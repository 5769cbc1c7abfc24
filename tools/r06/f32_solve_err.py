"""The F32 state's own solve error per row-transform path: evolve_psi! of an F32 State on a
white-noise F32 zeta against the F64 solve (PairSolver) of the same zeta, relative to psi.
usage: python tools/r06/f32_solve_err.py M:P ..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]
EPS32 = 2.0 ** -24


def main():
    import torch
    import qgamd
    for a in sys.argv[1:]:
        M, P = (int(x) for x in a.split(":"))
        m = qgamd.bench_model(M, P=P, dt=60.0)
        st = qgamd.State(m, dtype=torch.float32)
        st.initialise()
        st.run(1, 1)
        st.synchronize()
        h = st.slot("zeta", 1)
        z = [st.zeta[h, l].double() for l in (0, 1)]
        st.evolve_psi_()
        st.synchronize()
        p32 = [st.current("psi", l).double() for l in (1, 2)]
        Pi = tuple(float(x) for x in np.asarray(qgamd.P_inv_matrix(m), float).reshape(-1))
        S = qgamd.PairSolver(M, P, m.dx, (0.0, qgamd.S_eig(m)), (1, 0), Pi, (1.0, -1.0, 1.0, 1.0))
        o = [torch.empty_like(z[0]), torch.empty_like(z[0])]
        S.solve(z[0], z[1], o[0], o[1])
        torch.cuda.synchronize()
        n = lambda t: float(torch.linalg.vector_norm(t[1:-1, 1:-1]))  # noqa: E731
        e = [n(p32[l] - o[l]) / n(o[l]) for l in (0, 1)]
        # per x-band of the difference
        d = p32[0] - o[0]
        X = torch.fft.rfft(d[1:-1, 1:-1], dim=-1)
        E = (X.real ** 2 + X.imag ** 2).sum(dim=0)
        tot = float(E.sum())
        print(f"{M}x{P}: e_solve layers {e[0]:.3e} {e[1]:.3e} ({e[0] / EPS32:.1f} / {e[1] / EPS32:.1f} eps32); "
              f"energy share kx=0 {float(E[0]) / tot:.3f}, kx<=8 {float(E[1:9].sum()) / tot:.3f}", flush=True)


if __name__ == "__main__":
    main()
