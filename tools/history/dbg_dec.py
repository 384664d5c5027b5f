import sys, numpy as np
sys.path.insert(0, '.')
from tests.test_decomposition_gpu import run_decomposed, to_np
from tests.iw_helpers import device_params, perturbed, solver
for (world, W, H, nit, lit) in [(4,256,200,1,1),(4,256,200,1,2),(4,256,200,1,10),(4,256,200,3,10),(2,256,200,3,10)]:
    w = perturbed(W, H, seed=21 + world)
    s = solver(W, H); prm = device_params(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    ref = s.profiled_solve(prm)
    costs, O, A = run_decomposed(w, world, nit, lit)
    Ar = to_np(prm[1]); Or = to_np(prm[0])
    dA = np.abs(A - Ar).reshape(H, W); dO = np.abs(O - Or).reshape(H, 2*W)
    ia = np.unravel_index(dA.argmax(), dA.shape); io = np.unravel_index(dO.argmax(), dO.shape)
    rowmax = dA.max(axis=1)
    print(world, nit, lit, "cost rel", max(abs(a-b)/b for a,b in zip(costs[0], ref)), "dA", dA.max(), ia, "A there", Ar.reshape(H,W)[ia], "dO", dO.max(), io)
    print("   rows with largest dA:", np.argsort(rowmax)[-8:], rowmax[np.argsort(rowmax)[-8:]])
