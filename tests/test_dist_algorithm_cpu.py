"""The multi-rank FACR algorithm (per-rank pass A, all-gathered rank records, redundant
cross-rank closure + pin, per-rank pass B) run as world_size 1, 2, 4 and 8 gloo processes on the
CPU, through tests/facr_model.py (the step-for-step numpy model of the device kernels),
checked against the exact DFT solve of the C oracle on the global grid."""
import os
import socket
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(M, P):
    rng = np.random.default_rng(7)
    f1 = rng.standard_normal((M, P)) * 1e-9 + 3e-10  # nonzero mean: exercises delta
    f2 = rng.standard_normal((M, P)) * 1e-9
    return f1, f2


def _worker(rank, world, port, M, P, L, outdir):
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    import facr_model as F

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dx = 4e6 / M
    alphas = (0.0, -6.25e-10)
    f1, f2 = _problem(M, P)
    Pl = P // world
    sl = slice(rank * Pl, (rank + 1) * Pl)
    rec, st = F.rank_pass_a(f1[:, sl], f2[:, sl], M, dx, alphas, True, L, Pl, P)
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    x1, x2 = F.rank_pass_b(recs, rank, st, M, dx, True, L, Pl, P, np.eye(2))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), x1=x1, x2=x2)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,M,P,L", [(1, 32, 48, 8), (2, 32, 48, 8), (4, 16, 64, 4), (2, 64, 32, 16), (8, 16, 64, 4)])
def test_multirank_facr_matches_exact_solve(world, M, P, L):
    import torch.multiprocessing as mp

    from oracle import qg_oracle as O

    O.build()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, M, P, L, d)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
        assert all(p.exitcode == 0 for p in ps)
        x1 = np.concatenate([np.load(os.path.join(d, f"r{r}.npz"))["x1"] for r in range(world)], axis=1)
        x2 = np.concatenate([np.load(os.path.join(d, f"r{r}.npz"))["x2"] for r in range(world)], axis=1)
    dx = 4e6 / M
    f1, f2 = _problem(M, P)
    F1 = np.zeros((M + 2, P + 2))
    F1[1:-1, 1:-1] = f1
    F2 = np.zeros((M + 2, P + 2))
    F2[1:-1, 1:-1] = f2
    r1 = O.solve(M, P, dx, 0.0, F1, pinned=True)[1:-1, 1:-1]
    r2 = O.solve(M, P, dx, -6.25e-10, F2)[1:-1, 1:-1]
    assert np.abs(x1 - r1).max() < 1e-12 * np.abs(r1).max()
    assert np.abs(x2 - r2).max() < 1e-12 * np.abs(r2).max()
