import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'julia-ocean-modelling_amd'))
import qgamd
from oracle import qg_ref as R
M = P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dx = 4e6 / M
f = R.update_doubly_periodic_bc(R.seeded_rand(M, P, 5) - 0.5) * 1e-9
F = torch.from_numpy(np.ascontiguousarray(f.T)).cuda()
ref = R.sp_solve_modified_helmholtz(M, P, dx, f, -6.25e-10)
for dummy in (-6.25e-10, -1.0, -1e-8):
    s = qgamd.PairSolver(M, P, dx, (-6.25e-10, dummy), (0, 0), (1, 0, 0, 0), (1, 0, 0, 0))
    out = s.solve(F).cpu().numpy().T
    print('dummy', dummy, 'nan?', np.isnan(out).any(), 'rel', np.linalg.norm(out - ref) / np.linalg.norm(ref))
# pair with both systems live
s = qgamd.PairSolver(M, P, dx, (-6.25e-10, -6.25e-10), (0, 0), (1, 0, 0, 1), (1, 0, 0, 1))
o1, o2 = s.solve(F, F, torch.empty_like(F), torch.empty_like(F))
print('pair', np.linalg.norm(o1.cpu().numpy().T - ref) / np.linalg.norm(ref), np.linalg.norm(o2.cpu().numpy().T - ref) / np.linalg.norm(ref))
print(out[:3, :3], ref[:3, :3])
