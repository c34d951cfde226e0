"""One subdomain per GPU (what each rank holds at N = 8): the MGPIS solve of one full-size subdomain
of the bench chain (worm and wheel, 1.22M dof, 6 levels) under the multicolour option set and under
the block-Jacobi small-batch set, alternating, best of 5 timed solves each (host copies of b and x
included, the same for both).  The worm's consForc is zero at iteration 0, so both take a fixed
pseudo-random right-hand side.

    python profiles/one_sub_probe.py OUT.json [--variants]
"""
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")


def main():
    P = D.Problem("dehw", 1, 3, 2, 2, 5, 0.2).ESTABLISH()
    rows = []
    sets = [("multicolour", D.HEADLINE_OPTIONS), ("block-jacobi", D.HEADLINE_OPTIONS_SMALL)]
    if "--variants" in sys.argv:  # exact solve one level higher, Chebyshev smoothing
        sets += [("block-jacobi, exact level 2", dict(D.HEADLINE_OPTIONS_SMALL, coarse_level=2)),
                 ("multicolour, exact level 2", dict(D.HEADLINE_OPTIONS, coarse_level=2)),
                 ("chebyshev nu 2", dict(D.HEADLINE_OPTIONS_SMALL, smoother=2, nu=2)),
                 ("block-jacobi nu 2", dict(D.HEADLINE_OPTIONS_SMALL, nu=2))]
    for tv in ((1,) if "--variants" in sys.argv else (0, 1)):
        n = len(P.grid(tv).consForc)
        b = ((np.arange(n) * 7919 + 13) % 2003) / 2003.0 - 0.5
        for rep in range(2):
            for name, opts in sets:
                M = D.MGPIS.from_problem(P, tv, **opts)
                M.CG_SOLV(1, b)  # warm-up (graph capture)
                best, its = 1e300, 0
                for _ in range(5):
                    t = time.perf_counter()
                    _, its, rr = M.CG_SOLV(1, b)
                    best = min(best, time.perf_counter() - t)
                    assert rr <= 1e-14
                del M
                r = dict(subdomain=tv, dof=n, set=name, rep=rep, ms_per_solve=1e3 * best, pcg_iters=its)
                rows.append(r)
                print(json.dumps(r), flush=True)
    with open(sys.argv[1], "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
