"""Diagnostics of the multicolour smoother (smoother = 3) on the headline's subdomains.

    python profiles/gs_debug.py GL mgpis            MGPIS iterations per subdomain (random b, capped)
    python profiles/gs_debug.py GL admm SM NU MUSC  ADMM steps of the device loop (the bench's
                                                    problem, coarse space MUSC) with every
                                                    subdomain's PCG count per step
Run the admm mode under DDPCA_PCG_MAXIT=... so a stagnating solve ends instead of running to
maxit = rows."""
import importlib
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")
gl = int(sys.argv[1]) if len(sys.argv) > 1 else 3
mode = sys.argv[2] if len(sys.argv) > 2 else "mgpis"
if mode == "mgpis":
    P = D.headline_problem(gl=gl).ESTABLISH()
    rng = np.random.default_rng(1)
    for tv in range(P.nsub):
        b = rng.standard_normal(len(P.grid(tv).consForc))
        for sm, nu in ((1, 1), (3, 2)):
            M = D.MGPIS.from_problem(P, tv, smoother=sm, nu=nu, omega=-1.7, precond_fp32=2, table_mode=0)
            t = time.time()
            try:
                x, it, rr = M.CG_SOLV(1, b, maxit=300)
            except Exception as e:  # the cap reached is reported as an error code
                print(tv, sm, nu, "error", e, flush=True)
                continue
            print(f"tv {tv} smoother {sm} nu {nu}: {it} iterations, relres {rr:.2e} ({time.time() - t:.2f} s)", flush=True)
else:
    sm, nu, musc = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    P = D.headline_problem(gl=gl)
    if musc:
        P.set_coarse(musc, [1] * P.nsub)
    P.ESTABLISH()
    o = dict(D.HEADLINE_OPTIONS, smoother=sm, nu=nu)
    mc = D.MCONTACT(P, **o)
    for k in range(4):
        t = time.time()
        try:
            mc.CONTACT_ANALYSIS(1, check=False)
        except Exception as e:
            print(f"smoother {sm} nu {nu} musc {musc} ADMM step {k}: {e}; pcg {list(mc.get('pcg_iters'))}", flush=True)
            break
        print(f"smoother {sm} nu {nu} musc {musc} ADMM step {k}: pcg {list(mc.get('pcg_iters'))} {time.time() - t:.2f} s",
              flush=True)
