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
KB = 8  # band (b): 1 <= kx <= KB


def parts(torch, x, kb=KB):
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
    return np.array([float(e[0]), float(e[1:kb + 1].sum()), float(e[kb + 1:].sum())])


def _nrm(torch, t):
    return float(torch.linalg.vector_norm(t[1:-1, 1:-1].double()))


def _projections(qgamd, m):
    Pi = tuple(float(x) for x in np.asarray(qgamd.P_inv_matrix(m), float).reshape(-1))
    Pf = (1.0, -m.H_1 / m.H_1, 1.0, 1.0)  # P_matrix(H_1, H_1) (model.jl:173)
    return Pi, Pf


def compare(qgamd, torch, m, z_a, p_a, z_b, p_b, mc=8, seed=5):
    """State a (zeta / psi layers, slot 1) against state b, both models m: the psi difference
    attributed as above.  Returns a dict of relative (to ||psi_b|| or ||zeta_b||) norms."""
    Pi, Pf = _projections(qgamd, m)
    z_a = [z.double() for z in z_a]
    S = qgamd.PairSolver(m.M, m.P, m.dx, (0.0, qgamd.S_eig(m)), (1, 0), Pi, Pf)
    pp = [torch.empty_like(z_a[0]), torch.empty_like(z_a[0])]
    S.solve(z_a[0], z_a[1], pp[0], pp[1])  # psi' = solve64(zeta_a)
    torch.cuda.synchronize()
    psi_n = np.hypot(_nrm(torch, p_b[0]), _nrm(torch, p_b[1]))
    zeta_n = np.hypot(_nrm(torch, z_b[0]), _nrm(torch, z_b[1]))
    out = {"M": m.M, "P": m.P}
    out["psi_err"] = np.hypot(*[_nrm(torch, p_a[l].double() - p_b[l].double()) for l in (0, 1)]) / psi_n
    out["zeta_err"] = np.hypot(*[_nrm(torch, z_a[l] - z_b[l].double()) for l in (0, 1)]) / zeta_n
    out["e_solve"] = np.hypot(*[_nrm(torch, p_a[l].double() - pp[l]) for l in (0, 1)]) / psi_n
    E = sum(parts(torch, pp[l] - p_b[l].double()) for l in (0, 1))
    out["L_parts"] = list(np.sqrt(E) / psi_n)
    out["L_total"] = float(np.sqrt(E.sum()) / psi_n)
    del pp
    dz = [z_a[l] - z_b[l].double() for l in (0, 1)]
    out["dz_parts"] = list(np.sqrt(sum(parts(torch, dz[l]) for l in (0, 1))) / zeta_n)
    N = m.M * m.P
    sig, mean0 = [], 0.0
    for s in (0, 1):
        t = Pi[2 * s] * dz[0] + Pi[2 * s + 1] * dz[1]
        sig.append(_nrm(torch, t) / np.sqrt(N))
        if s == 0:  # the compatibility residue of the zeta error: sum(b) that the pin moves to (1,1)
            mean0 = float(t[1:-1, 1:-1].sum()) / N
        del t
    del dz, z_a
    out["sigma_modal"] = sig
    out["sum_b_residue"] = mean0 * N
    # the residue's part of L dz: the pinned solve of the constant mean0 is exactly the
    # response to the point source -sum(b) at (1,1) that get_poisson_cholesky's pin makes of it
    Sm = qgamd.PairSolver(m.M, m.P, m.dx, (0.0, qgamd.S_eig(m)), (1, 0), (1, 0, 0, 1), Pf)
    f = [torch.zeros_like(p_b[0], dtype=torch.float64), torch.zeros_like(p_b[0], dtype=torch.float64)]
    o = [torch.empty_like(f[0]), torch.empty_like(f[0])]
    f[0][1:-1, 1:-1] = mean0
    Sm.solve(f[0], f[1], o[0], o[1])
    torch.cuda.synchronize()
    out["L_sum_b"] = np.hypot(_nrm(torch, o[0]), _nrm(torch, o[1])) / psi_n
    # white-noise prediction through the same solve (modal inputs: proj_in = I)
    g = torch.Generator(device=f[0].device).manual_seed(seed)
    acc, draws = np.zeros(3), []
    for _ in range(mc):
        for s in (0, 1):
            f[s][1:-1, 1:-1].normal_(0.0, sig[s], generator=g)
        Sm.solve(f[0], f[1], o[0], o[1])
        e = sum(parts(torch, o[l]) for l in (0, 1))
        acc += e
        draws.append(list(np.sqrt(e) / psi_n))
    del f, o
    torch.cuda.empty_cache()
    out["pred_parts_rms"] = list(np.sqrt(acc / mc) / psi_n)
    out["pred_total_rms"] = float(np.sqrt(acc.sum() / mc) / psi_n)
    out["pred_draws_max"] = [max(d[i] for d in draws) for i in range(3)]
    out["ratio_to_pred"] = [x / y for x, y in zip(out["L_parts"], out["pred_parts_rms"])]
    return out


def decompose(qgamd, torch, m, steps, mc=8, seed=5, chunk_rows=0):
    """The F32 run of model m against the F64 run after `steps` steps (compare above), plus the
    compatibility residue delta = -sum(b) each run's pin injected (qg_get_stats).  chunk_rows:
    the F32 run's solver chunk (0 = automatic) -- another chunk is another summation order of
    the scans, the singular kx = 0 line's included: another realisation of the F32 roundoff."""
    a = qgamd.run_model_no_output(m, nsteps=steps)
    a.synchronize()
    d64 = a.stats()["delta"]
    z64 = [a.current("zeta", l).clone() for l in (1, 2)]
    p64 = [a.current("psi", l).clone() for l in (1, 2)]
    del a
    torch.cuda.empty_cache()
    b = qgamd.run_model_no_output(m, nsteps=steps, dtype=torch.float32, chunk_rows=chunk_rows)
    b.synchronize()
    d32 = b.stats()["delta"]
    z32 = [b.current("zeta", l).clone() for l in (1, 2)]
    p32 = [b.current("psi", l).clone() for l in (1, 2)]
    del b
    torch.cuda.empty_cache()
    out = compare(qgamd, torch, m, z32, p32, z64, p64, mc=mc, seed=seed)
    out.update(steps=steps, delta64=d64, delta32=d32)
    return out


def bars(r, k=5.0, e_solve_bar=8 * EPS32):
    """The mechanism's bars: each band of L dz within k times its white-noise prediction, the
    F32 solve's own error within e_solve_bar, and the total psi error within the sum.  A band's
    energy is a weighted sum of independent chi-square variables (one per mode, 1 or 2 degrees
    of freedom); the heaviest tail is one real mode carrying it all, so P(band > k x its RMS)
    <= P(chi2_1 > k^2) = 5.7e-7 at k = 5, whichever modes the roundoff happens to hit."""
    part = [k * p for p in r["pred_parts_rms"]]
    return {"parts": part, "e_solve": e_solve_bar, "psi": float(np.sqrt(sum(x * x for x in part))) + e_solve_bar}


def check(r, k=5.0, e_solve_bar=8 * EPS32, zeta_bar=16 * EPS32):
    """Assert the mechanism's bars on a compare()/decompose() record."""
    b = bars(r, k, e_solve_bar)
    assert r["zeta_err"] < zeta_bar, ("zeta", r["zeta_err"], zeta_bar)
    assert r["e_solve"] < b["e_solve"], ("e_solve", r["e_solve"], b["e_solve"])
    for i, (x, y) in enumerate(zip(r["L_parts"], b["parts"])):
        assert x < y, ("band", "abc"[i], x, y)
    assert r["psi_err"] < b["psi"], ("psi", r["psi_err"], b["psi"])
    return b


def fmt(r):
    def f(v):
        if isinstance(v, (list, tuple)):
            return "[" + ", ".join(f"{x:.3e}" for x in v) + "]"
        return f"{v:.3e}" if isinstance(v, float) else str(v)
    return ", ".join(f"{k}={f(v)}" for k, v in r.items())
