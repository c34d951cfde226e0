"""Stencil-coded vs column-indexed V-cycle copies on one headline subdomain (GPU): MULT_VCYC of a
random residual under both, per option set, with the row-split kernel off (DDPCA_SPLIT_CHUNKS=0)."""
import importlib
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")
gl = int(sys.argv[1]) if len(sys.argv) > 1 else 3
os.environ["DDPCA_SPLIT_CHUNKS"] = "0"
P = D.headline_problem(gl=gl).ESTABLISH()
r = np.random.default_rng(1).standard_normal(len(P.grid(0).consForc))
for name in ("HEADLINE_OPTIONS", "HEADLINE_OPTIONS_SMALL"):
    out = {}
    for coded in ("1", "0", "2"):
        os.environ["DDPCA_CODED"] = coded
        M = D.MGPIS.from_problem(P, 0, **getattr(D, name))
        out[coded] = (M.MULT_VCYC(r), M.spmv(r))
        del M
    z1, z0 = out["1"][0], out["0"][0]
    nd = int(np.sum(z1 != z0))
    print(f"{name}: vcycle differing entries {nd} of {len(z1)}, max |dz| {np.max(np.abs(z1 - z0)):.3e} "
          f"(|z| {np.max(np.abs(z0)):.3e}); fine spmv equal {np.array_equal(out['1'][1], out['0'][1])}", flush=True)
    z2 = out["2"][0]
    print(f"  coded levels + column-indexed colour chunks vs all column-indexed: differing {int(np.sum(z2 != z0))}", flush=True)
    if nd:
        idx = np.nonzero(z1 != z0)[0][:10]
        print("  first differing dofs", idx.tolist(), (z1[idx] - z0[idx]).tolist())
