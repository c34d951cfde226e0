"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

CPU price of one full ADMM iteration of MCONTACT::CONTACT_ANALYSIS (MCONTACT.h:2493-2723) for
bench.py's `cpu_baseline` leg, computed by the SGS-faithful port (oracle.cpp: MGPIS::CG_SOLV with
SGS V(1,1), OpenMP SpMV) on the bench's own operators, at the state the device run reached (its
u / aux / lambda after the timed iterations), so the subdomain solves see a late-iteration
right-hand side, not iteration 0's:

  body balance   (2511-2533)  CG_SOLV(1) of each subdomain with consForc + consOper
                              (systTran_pena aux - systTran lambda) -- sampled: solves run until
                              `budget_s` is spent (>= 2 of them), priced as nsub x their mean
  coarse space   (2578-2612)  globTran_1 lambda, globTran_D_1 u, the factorised globCoup_1 solve
                              (scipy SuperLU; the reference's SimplicialLDLT is factorised at setup
                              too), accuProl -- all of them, timed
  interface      (2629-2704)  gamma, projection, aux and lambda with the factorised surface mass
                              matrices (the reference's LDLT below 120000 rows) -- all interfaces,
                              timed
Text output (OUTP_SUB2 / OUTPUT_PRTR every iteration in the reference) is left out.
"""
from __future__ import annotations

import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from oracle import oracle as O


def price_iteration(P, mc, budget_s: float = 20.0) -> dict:
    nsub, nint = P.nsub, P.nint
    u = [mc.get("resuDisp", tv) for tv in range(nsub)]
    aux = [[mc.get("inteAuxi", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    lam = [[mc.get("inteLagr", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    ops = [[{n: O.csr64(P.csr(n, 2 * ts + s)) for n in P.IFACE_OPS} for s in range(2)] for ts in range(nint)]
    body = [tuple(int(b) for b in P.array("iface_body", ts)) for ts in range(nint)]
    fric = [float(P.array("iface_param", ts)[0]) for ts in range(nint)]
    # ---- body balance: sampled subdomain solves (wheels first: they carry the load)
    order = [tv for tv in range(1, nsub, 2)] + [tv for tv in range(0, nsub, 2)]
    solve_s, iters, ndof, used = [], [], 0, []
    for tv in order:
        G = P.grid(tv)
        L = G.maxiLeve
        M = O.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
        flag = G.consFlag == 1
        f = np.zeros(len(flag))
        for ts in range(nint):
            for s in range(2):
                if body[ts][s] == tv:  # ADDITIONAL_FORCE, MCONTACT.h:2520-2524
                    O.csr_matvec(ops[ts][s]["systTran_pena"], aux[ts][s], f)
                    f -= O.csr_matvec(ops[ts][s]["systTran"], lam[ts][s])
        b = G.consForc + f[flag]
        t = time.perf_counter()
        x, it, _ = M.CG_SOLV(1, b)
        solve_s.append(time.perf_counter() - t)
        iters.append(int(it))
        used.append(tv)
        ndof = len(b)
        del M
        if len(solve_s) >= 2 and sum(solve_s) >= budget_s:
            break
    t_body = nsub * float(np.mean(solve_s))
    # ---- coarse-space correction (muscSett = 2)
    t_coarse = 0.0
    try:
        gc = P.csr("globCoup_1")
    except Exception:  # noqa: BLE001 -- no coarse space in this problem
        gc = None
    if gc is not None and gc.shape[0] > 0:
        lu = spla.splu(sp.csc_matrix(gc))
        gt = [[O.csr64(P.csr("globTran_1", 2 * ts + s)) for s in range(2)] for ts in range(nint)]
        gd = [O.csr64(P.csr("globTran_D_1", tv)) for tv in range(nsub)]
        ap = [O.csr64(P.csr("accuProl", tv)) for tv in range(nsub)]
        base = P.array("baseReco")
        t = time.perf_counter()
        g = P.array("globForc_1").copy()
        for ts in range(nint):
            for s in range(2):
                O.csr_matvec(gt[ts][s], lam[ts][s], g)
        for tv in range(nsub):
            g -= O.csr_matvec(gd[tv], u[tv])
        xc = lu.solve(g)
        for tv in range(nsub):
            O.csr_matvec(ap[tv], xc[base[tv]:base[tv + 1]])
        t_coarse = time.perf_counter() - t
    # ---- interface step, every interface
    mfac = [[(spla.factorized(sp.csc_matrix(ops[ts][s]["inteMass_pena"])), spla.factorized(sp.csc_matrix(ops[ts][s]["inteMass"])))
             for s in range(2)] for ts in range(nint)]
    tTp = [[O.csr64(ops[ts][s]["systTran_pena"].T) for s in range(2)] for ts in range(nint)]
    t = time.perf_counter()
    nip = 0
    for ts in range(nint):
        op = ops[ts]
        gam = 0.5 * (O.csr_matvec(op[0]["inpoLagr"], lam[ts][0]) - O.csr_matvec(op[1]["inpoLagr"], lam[ts][1])
                     + O.csr_matvec(op[0]["pemaInpo_r"], u[body[ts][0]]) - O.csr_matvec(op[1]["pemaInpo_r"], u[body[ts][1]]))
        gam -= 0.5 * P.array("pemaDiag", ts) * P.array("inpoNgap", ts)
        comp = 1 if fric[ts] == 0.0 else 3
        gam = O._project(gam, comp, fric[ts])[0]
        nip += len(gam) // comp
        for s in range(2):
            Tt_u = O.csr_matvec(tTp[ts][s], u[body[ts][s]])
            a = mfac[ts][s][0](Tt_u + O.csr_matvec(op[s]["inteMass"], lam[ts][s]) + O.csr_matvec(op[s]["inteInpo"], gam))
            lam[ts][s] = lam[ts][s] + mfac[ts][s][1](Tt_u - O.csr_matvec(op[s]["inteMass_pena"], a))
    t_iface = time.perf_counter() - t
    total = t_body + t_coarse + t_iface
    return {
        "value": 1.0 / total,
        "unit": "ADMM it/s",
        "cores": O.threads(),
        "kind": "port",
        "sample": f"one ADMM iteration at the device run's final state: {len(solve_s)} of {nsub} subdomain "
                  f"CG_SOLV(1) solves sampled (subdomains {used}, {ndof} DOF each, {iters} SGS-MGPIS iterations, "
                  f"{sum(solve_s):.1f} s; body balance priced {t_body:.1f} s), coarse-space correction {t_coarse:.2f} s, "
                  f"interface step over all {nint} interfaces / {nip} integration points {t_iface:.2f} s",
        "body_s": t_body,
        "coarse_s": t_coarse,
        "iface_s": t_iface,
        "dof_iter_per_s": ndof * sum(iters) / sum(solve_s),
    }
