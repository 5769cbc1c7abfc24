"""A numpy restatement of the multigrid preconditioner of csrc/qg_mg.hip (QG_PRECOND_MULTIGRID)
and of the PCG around it (csrc/qg_pcg.hip) -- test infrastructure: the CPU suite checks the
design (symmetry, grid-independent iteration counts, the slab form's equality with the global
cycle) without a GPU; the GPU tests check the kernels against the C oracle.

Operator per level: B = -(cx (E + W - 2) + cy (N + S - 2) + alpha), x periodic, y periodic on
the global grid.  V(2,2): damped Jacobi (omega 0.8) from zero, full-weighting restriction,
rediscretised coarse operator, bilinear prolongation; coarsest grid (<= 64 points) by
min(512, 8 max(M, P)) Jacobi sweeps.  Pinned Poisson: z = T^T V T r (T r = r - sum(r) e_pin,
T^T z = z - z_pin).  Slab form: levels of each rank's rows with ghost rows copied from the
neighbouring slabs before every stencil, gathered into the global grid below MG_AGG_POINTS.
Fields are (P, M) arrays (row j = y index), the pin at [0, 0].
"""
import numpy as np

OMEGA = 0.8
AGG_POINTS = 4096


def plan(M, P, G=1):
    """[(M, P, rx, ry, slab, agg)] as plan_levels builds them."""
    lv = [(M, P, 0, 0, G > 1, 0)]
    while True:
        m, p, _, _, slab, _ = lv[-1]
        rx, ry = m % 2 == 0 and m >= 8, p % 2 == 0 and p >= 8
        if slab:
            if m * p > AGG_POINTS and ry:
                lv.append((m // 2 if rx else m, p // 2, rx, 1, 1, 0))
            else:
                lv.append((m, p * G, 0, 0, 0, 1))
        else:
            if m * p <= 64 or not (rx or ry):
                break
            lv.append((m // 2 if rx else m, p // 2 if ry else p, rx, ry, 0, 0))
    return lv


def spacings(lv, dx):
    out, hx, hy = [], dx, dx
    for (_, _, rx, ry, _, _) in lv:
        hx, hy = hx * (2 if rx else 1), hy * (2 if ry else 1)
        out.append((1 / hx ** 2, 1 / hy ** 2))
    return out


def apply_b(z, cx, cy, al, ghost=None):
    """B z; ghost = (row below, row above) for a slab, else y wraps."""
    if ghost is None:
        s, n = np.roll(z, 1, 0), np.roll(z, -1, 0)
    else:
        s, n = np.vstack([ghost[0][None], z[:-1]]), np.vstack([z[1:], ghost[1][None]])
    return -(cx * ((np.roll(z, 1, 1) + np.roll(z, -1, 1)) - 2 * z) + cy * ((s + n) - 2 * z) + al * z)


def _restrict(t, rx, ry, below=None):
    """Full weighting; below: the slab's ghost row -1 of t (None: y wraps)."""
    if rx:
        t = 0.5 * t + 0.25 * (np.roll(t, 1, 1) + np.roll(t, -1, 1))
        t = t[:, 0::2]
        if below is not None:
            below = (0.5 * below + 0.25 * (np.roll(below, 1) + np.roll(below, -1)))[0::2]
    if ry:
        prev = np.roll(t, 1, 0) if below is None else np.vstack([below[None], t[:-1]])
        t = (0.5 * t + 0.25 * (prev + np.roll(t, -1, 0)))[0::2]
    return t


def _prolong(e, rx, ry, above=None):
    """Bilinear interpolation; above: the slab's coarse ghost row P_c (None: y wraps)."""
    if ry:
        nxt = np.roll(e, -1, 0) if above is None else np.vstack([e[1:], above[None]])
        f = np.zeros((2 * e.shape[0], e.shape[1]))
        f[0::2], f[1::2] = e, 0.5 * (e + nxt)
        e = f
    if rx:
        f = np.zeros((e.shape[0], 2 * e.shape[1]))
        f[:, 0::2], f[:, 1::2] = e, 0.5 * (e + np.roll(e, -1, 1))
        e = f
    return e


def _coarsest(r, cx, cy, al):
    wd = OMEGA / (2 * cx + 2 * cy - al)
    z = wd * r
    for _ in range(min(512, 8 * max(r.shape)) - 1):
        z = z + wd * (r - apply_b(z, cx, cy, al))
    return z


def _vglobal(lv, hs, l, r, al):
    cx, cy = hs[l]
    if l == len(lv) - 1:
        return _coarsest(r, cx, cy, al)
    wd = OMEGA / (2 * cx + 2 * cy - al)
    _, _, rx, ry, _, _ = lv[l + 1]
    z = wd * (2 * r - wd * apply_b(r, cx, cy, al))  # the two pre-sweeps from zero (mg_pre)
    e = _vglobal(lv, hs, l + 1, _restrict(r - apply_b(z, cx, cy, al), rx, ry), al)
    z = z + _prolong(e, rx, ry)
    t = z + wd * (r - apply_b(z, cx, cy, al))
    return t + wd * (r - apply_b(t, cx, cy, al))


def _halo(fs):
    """Ghost rows (below, above) of each slab from its ring neighbours."""
    G = len(fs)
    return [(fs[(g - 1) % G][-1], fs[(g + 1) % G][0]) for g in range(G)]


def _vslab(lv, hs, l, rs, al):
    """One level of the slab cycle; rs: each rank's rows."""
    G = len(rs)
    _, _, rx, ry, _, agg = lv[l + 1]
    if agg:
        Z = _vglobal(lv, hs, l + 1, np.vstack(rs), al)
        P = rs[0].shape[0]
        return [Z[g * P:(g + 1) * P] for g in range(G)]
    cx, cy = hs[l]
    wd = OMEGA / (2 * cx + 2 * cy - al)
    hr = _halo(rs)
    z = [wd * (2 * rs[g] - wd * apply_b(rs[g], cx, cy, al, hr[g])) for g in range(G)]
    hz = _halo(z)
    t = [rs[g] - apply_b(z[g], cx, cy, al, hz[g]) for g in range(G)]
    ht = _halo(t)
    e = _vslab(lv, hs, l + 1, [_restrict(t[g], rx, ry, ht[g][0]) for g in range(G)], al)
    he = _halo(e)
    z = [z[g] + _prolong(e[g], rx, ry, he[g][1]) for g in range(G)]
    hz = _halo(z)
    t = [z[g] + wd * (rs[g] - apply_b(z[g], cx, cy, al, hz[g])) for g in range(G)]
    ht = _halo(t)
    return [t[g] + wd * (rs[g] - apply_b(t[g], cx, cy, al, ht[g])) for g in range(G)]


def vcycle(r, dx, al, G=1):
    """V r on the global (P, M) grid, computed in the G-slab form when G > 1."""
    P, M = r.shape
    lv = plan(M, P // G, G)
    hs = spacings(lv, dx)
    if G == 1:
        return _vglobal(lv, hs, 0, r, al)
    Pl = P // G
    return np.vstack(_vslab(lv, hs, 0, [r[g * Pl:(g + 1) * Pl] for g in range(G)], al))


def precond(r, dx, al, pinned, G=1):
    """z = T^T V T r (pinned Poisson) or V r; r has r[0, 0] = 0 when pinned."""
    if not pinned:
        return vcycle(r, dx, al, G)
    rt = r.copy()
    rt[0, 0] = -r.sum()
    z = vcycle(rt, dx, al, G)
    return z - z[0, 0]


def pinned_apply(x, dx, al, pinned):
    """The reference's matrix (construct_spA, pinned as get_poisson_cholesky pins it), negated."""
    idx2 = 1 / dx ** 2
    if not pinned:
        return apply_b(x, idx2, idx2, al)
    xx = x.copy()
    xx[0, 0] = 0
    y = apply_b(xx, idx2, idx2, al)
    y[0, 0] = x[0, 0]
    return y


def pcg(b, dx, al, pinned, G=1, rtol=1e-13, maxit=200):
    """PCG as qg_pcg.hip runs it: x0 = 0, stop at ||r|| <= rtol ||b||; returns (x, iterations,
    relres history)."""
    r = b.copy()
    if pinned:
        r[0, 0] = 0.0
    x = np.zeros_like(b)
    bb = float((r * r).sum())
    z = precond(r, dx, al, pinned, G)
    if pinned:
        z[0, 0] = r[0, 0]
    p, rz, hist = z.copy(), float((r * z).sum()), []
    for it in range(1, maxit + 1):
        q = pinned_apply(p, dx, al, pinned)
        a = rz / float((p * q).sum())
        x += a * p
        r -= a * q
        hist.append(np.sqrt(float((r * r).sum()) / bb))
        if hist[-1] <= rtol:
            return x, it, hist
        z = precond(r, dx, al, pinned, G)
        if pinned:
            z[0, 0] = r[0, 0]
        rz2 = float((r * z).sum())
        p = z + (rz2 / rz) * p
        rz = rz2
    return x, maxit, hist
