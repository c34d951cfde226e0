import faulthandler, importlib, sys
faulthandler.enable()
sys.path.insert(0, ".")
D = importlib.import_module("ddpca-admm_amd")
import numpy as np
P = D.Problem('beam', 8, 2, 2, 2, 1, 1, 1).ESTABLISH()
G = P.grid(0)
L = G.maxiLeve
nn = [int(x) for x in P.array("leveCount", 0)]
flag = np.asarray(G.consFlag)
fd = np.flatnonzero(flag[: 3 * nn[L]])
M = D.MGPIS.from_csr([nn[L]], [fd], [G.consStif(L)], [], table_mode=0, precond_fp32=0)
x, it, rr, bd = M.BiCGSTAB_SOLV(0, G.consForc)
print("single-level BiCGSTAB(0):", it, rr, flush=True)
