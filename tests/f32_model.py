"""F32 state vs F64: where the psi error comes from -- test infrastructure
shared by tests/test_gpu_configs.py and tools/r06/f32_decompose.py.

Both runs start from the same seeded model (F64 and F32 state).  After `steps` steps, with
zeta^32 / psi^32 (F32 run) and zeta^64 / psi^64 (F64 run) in slot 1:

  psi' = solve64(zeta^32)                  the exact (F64) evolve_psi! of the F32 run's zeta
  e_solve = psi^32 - psi'                  the F32 path's own solve error (U stored in F32,
                                           psi rounded to F32)
  L dz = psi' - psi^64 = solve64(dzeta)    the image of the F32 zeta error under the solve
                                           (linear: the pinned solve is a linear map, its
                                           compatibility shift and pin included)

so psi^32 - psi^64 = L dz + e_solve exactly.  L dz is split by x-wavenumber kx of the rows:
(a) kx = 0 (the x-mean line, with the pin's constant), (b) 1 <= kx <= 8, (c) kx > 8, each
relative to ||psi^64||.  The white-noise model of the zeta error predicts each part: a modal
white noise per system with the measured variance, through the same solve (Monte Carlo on the
device): E ||(L w)_S||^2.  Also recorded: the compatibility residue delta = -sum(b) that the
pin injects at interior (1,1) (model.jl:185, qg_get_stats) in both runs.
"""
import numpy as np

EPS32 = 2.0 ** -24


def parts(torch, x, kb=8):
    """Energies of the rows' x-wavenumber bands of a (P+2, M+2) field's interior:
    [kx = 0, 1 <= kx <= kb, kx > kb] (Parseval over rfft along x)."""
    X = torch.fft.rfft(x[1:-1, 1:-1].double(), dim=-1)
    M = x.shape[-1] - 2
    w = torch.full((X.shape[-1],), 2.0, dtype=torch.float64, device=x.device)
    w[0] = 1.0
    if M % 2 == 0:
        w[-1] = 1.0
    e = (X.real ** 2 + X.imag ** 2).sum(dim=0) * w / M
    del X
    return [float(e[0]), float(e[1:kb + 1].sum()), float(e[kb + 1:].sum())]


def decompose(qgamd, torch, m, steps, mc=8, seed=5):
    a = qgamd.run_model_no_output(m, nsteps=steps)
    a.synchronize()
    d64 = a.stats()["delta"]
    z64 = [a.current("zeta", l).clone() for l in (1, 2)]
    p64 = [a.current("psi", l).clone() for l in (1, 2)]
    del a
    torch.cuda.empty_cache()
    b = qgamd.run_model_no_output(m, nsteps=steps, dtype=torch.float32)
    b.synchronize()
    d32 = b.stats()["delta"]
    z32 = [b.current("zeta", l).double() for l in (1, 2)]
    p32 = [b.current("psi", l).double() for l in (1, 2)]
    del b
    torch.cuda.empty_cache()
    Pi = np.asarray(qgamd.P_inv_matrix(m), float).reshape(-1)
    Pf = np.array([1.0, -m.H_1 / m.H_1, 1.0, 1.0])  # P_matrix(H_1, H_1) (model.jl:173)
    S = qgamd.PairSolver(m.M, m.P, m.dx, (0.0, qgamd.S_eig(m)), (1, 0), tuple(Pi), tuple(Pf))
    pp = [torch.empty_like(z32[0]), torch.empty_like(z32[0])]
    S.solve(z32[0], z32[1], pp[0], pp[1])
    torch.cuda.synchronize()
    nrm = lambda t: float(torch.linalg.vector_norm(t[1:-1, 1:-1]))  # noqa: E731
    psi_n = np.hypot(nrm(p64[0]), nrm(p64[1]))
    zeta_n = np.hypot(nrm(z64[0]), nrm(z64[1]))
    out = {"M": m.M, "P": m.P, "steps": steps, "delta64": d64, "delta32": d32}
    out["psi_err"] = np.hypot(nrm(p32[0] - p64[0]), nrm(p32[1] - p64[1])) / psi_n
    out["zeta_err"] = np.hypot(nrm(z32[0] - z64[0]), nrm(z32[1] - z64[1])) / zeta_n
    out["e_solve"] = np.hypot(nrm(p32[0] - pp[0]), nrm(p32[1] - pp[1])) / psi_n
    L = [pp[l] - p64[l] for l in (0, 1)]
    E = np.sum([parts(torch, L[l]) for l in (0, 1)], axis=0)
    out["L_parts"] = list(np.sqrt(E) / psi_n)
    out["L_total"] = float(np.sqrt(E.sum()) / psi_n)
    Ed = np.sum([parts(torch, p32[l] - p64[l]) for l in (0, 1)], axis=0)
    out["dpsi_parts"] = list(np.sqrt(Ed) / psi_n)
    # modal zeta error (the solve's inputs): dz~_s = Pinv[s] . dz, its variance per point
    dz = [z32[l] - z64[l] for l in (0, 1)]
    N = m.M * m.P
    sig = []
    for s in (0, 1):
        t = Pi[2 * s] * dz[0] + Pi[2 * s + 1] * dz[1]
        sig.append(nrm(t) / np.sqrt(N))
        del t
    out["sigma_modal"] = sig
    out["dz_parts"] = list(np.sqrt(np.sum([parts(torch, dz[l]) for l in (0, 1)], axis=0)) / zeta_n)
    del z32, z64, dz, L, pp, p32
    torch.cuda.empty_cache()
    # white-noise prediction through the same solve (inputs already modal: proj_in = I)
    Sm = qgamd.PairSolver(m.M, m.P, m.dx, (0.0, qgamd.S_eig(m)), (1, 0), (1, 0, 0, 1), tuple(Pf))
    g = torch.Generator(device="cuda").manual_seed(seed)
    acc, draws = np.zeros(3), []
    f = [torch.zeros_like(p64[0]), torch.zeros_like(p64[0])]
    o = [torch.empty_like(p64[0]), torch.empty_like(p64[0])]
    for _ in range(mc):
        for s in (0, 1):
            f[s][1:-1, 1:-1].normal_(0.0, sig[s], generator=g)
        Sm.solve(f[0], f[1], o[0], o[1])
        e = np.sum([parts(torch, o[l]) for l in (0, 1)], axis=0)
        acc += e
        draws.append(list(np.sqrt(e) / psi_n))
    out["pred_parts_rms"] = list(np.sqrt(acc / mc) / psi_n)
    out["pred_draws"] = draws
    out["ratio_to_pred"] = [x / y for x, y in zip(out["L_parts"], out["pred_parts_rms"])]
    return out


