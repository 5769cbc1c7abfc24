"""8192^2 F64 (the widest square grid of the size sweep): the device against the C oracle after
3 steps, and against itself with another chunk size (another summation order of the same exact
solve), with the compatibility residue each run's pin injected.  usage: python tools/r06/f64_8192_probe.py [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "julia-ocean-modelling_amd")]


def main():
    import torch
    import qgamd
    from oracle import qg_oracle as O
    from oracle import qg_ref as R
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    steps = 3
    m = qgamd.bench_model(N, dt=60.0)
    runs = {}
    for L in (0, 8):
        st = qgamd.run_model_no_output(m, nsteps=steps, chunk_rows=L)
        st.synchronize()
        runs[L] = ({n: np.stack([st.current(n, l).cpu().numpy().T for l in (1, 2)], axis=-1) for n in ("psi", "zeta")},
                   st.stats()["delta"])
        del st
        torch.cuda.empty_cache()
    ref = O.State(R.bench_model(N, dt=60.0)).run(steps)
    rel = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))  # noqa: E731
    for n in ("psi", "zeta"):
        want = getattr(ref, n)[:, :, :, 0]
        print(f"{N}^2 F64, {steps} steps, {n}: device vs C oracle {rel(runs[0][0][n], want):.3e}; "
              f"chunk 8 vs default {rel(runs[8][0][n], runs[0][0][n]):.3e}", flush=True)
    print(f"Sigma b residue (delta): default {runs[0][1]:.3e}, chunk 8 {runs[8][1]:.3e}")


if __name__ == "__main__":
    main()
