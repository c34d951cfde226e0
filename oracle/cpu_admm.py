"""ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.

CPU price of one full ADMM iteration of MCONTACT::CONTACT_ANALYSIS (MCONTACT.h:2493-2723) for
bench.py's `cpu_baseline` leg, computed by the SGS-faithful port (oracle.cpp: MGPIS::CG_SOLV with
SGS V(1,1), OpenMP SpMV) on the bench's own operators, at the state the device run reached (its
u / aux / lambda after the timed iterations), so the subdomain solves see a late-iteration
right-hand side, not iteration 0's.  Bounded sample:

  per subdomain (sampled: a wheel and a worm, more while `budget_s` lasts; priced x nsub / sample)
    body balance (2511-2533)  CG_SOLV(1) with consForc + consOper (systTran_pena aux - systTran lambda)
    coarse space (2578-2612)  its part of globTran_D_1 u in factored form -- consStif[L] u (one SpMV;
                              the reference multiplies the assembled globTran_D_1, more entries, so
                              this is favourable to the CPU) -- and accuProl x_c
  once (timed in full)
    coarse space              globTran_1 lambda, the globCoup_1 solve (scipy SuperLU, factorised
                              beforehand like the reference's SimplicialLDLT)
    interface    (2629-2704)  gamma, projection, aux and lambda with the factorised surface mass
                              matrices (the reference's LDLT below 120000 rows), every interface
Text output (OUTP_SUB2 / OUTPUT_PRTR every iteration in the reference) is left out.
"""
from __future__ import annotations

import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from oracle import oracle as O


def _log(msg: str) -> None:
    print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)


def price_iteration(P, mc, budget_s: float = 20.0) -> dict:
    nsub, nint = P.nsub, P.nint
    body = [tuple(int(b) for b in P.array("iface_body", ts)) for ts in range(nint)]
    fric = [float(P.array("iface_param", ts)[0]) for ts in range(nint)]
    u = [mc.get("resuDisp", tv) for tv in range(nsub)]
    aux = [[mc.get("inteAuxi", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    lam = [[mc.get("inteLagr", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    try:
        has_coarse = P.csr("globCoup_1").shape[0] > 0
    except Exception:  # noqa: BLE001 -- no coarse space in this problem
        has_coarse = False
    base = P.array("baseReco") if has_coarse else None
    # ---- per-subdomain work, sampled (wheels carry the load: a wheel, a worm, then alternate)
    order = [x for pair in zip(range(1, nsub, 2), range(0, nsub, 2)) for x in pair]
    solve_s, spmv_s, prol_s, iters, used, ndof = [], [], [], [], [], 0
    t_sample0 = time.perf_counter()
    for tv in order:
        G = P.grid(tv)
        L = G.maxiLeve
        M = O.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
        flag = G.consFlag == 1
        f = np.zeros(len(flag))
        for ts in range(nint):
            for s in range(2):
                if body[ts][s] == tv:  # ADDITIONAL_FORCE, MCONTACT.h:2520-2524
                    O.csr_matvec(O.csr64(P.csr("systTran_pena", 2 * ts + s)), aux[ts][s], f)
                    f -= O.csr_matvec(O.csr64(P.csr("systTran", 2 * ts + s)), lam[ts][s])
        b = G.consForc + f[flag]
        t = time.perf_counter()
        x, it, _ = M.CG_SOLV(1, b)
        solve_s.append(time.perf_counter() - t)
        iters.append(int(it))
        if has_coarse:
            t = time.perf_counter()
            M.SPMV(L, x)
            spmv_s.append(time.perf_counter() - t)
            A = O.csr64(P.csr("accuProl", tv))
            xc = np.ones(A.shape[1])
            t = time.perf_counter()
            O.csr_matvec(A, xc)
            prol_s.append(time.perf_counter() - t)
        used.append(tv)
        ndof = len(b)
        del M
        _log(f"subdomain {tv}: CG_SOLV(1) {iters[-1]} iterations, {solve_s[-1]:.2f} s")
        if len(solve_s) >= 2 and time.perf_counter() - t_sample0 >= budget_s:
            break
    scale = nsub / len(solve_s)
    t_body = scale * sum(solve_s)
    t_coarse = scale * (sum(spmv_s) + sum(prol_s))
    # ---- coarse solve and globTran_1 lambda, once
    if has_coarse:
        lu = spla.splu(sp.csc_matrix(P.csr("globCoup_1")))
        gt = [[O.csr64(P.csr("globTran_1", 2 * ts + s)) for s in range(2)] for ts in range(nint)]
        t = time.perf_counter()
        g = P.array("globForc_1").copy()
        for ts in range(nint):
            for s in range(2):
                O.csr_matvec(gt[ts][s], lam[ts][s], g)
        lu.solve(g)
        t_coarse += time.perf_counter() - t
    # ---- interface step, every interface
    ops = [[{n: O.csr64(P.csr(n, 2 * ts + s)) for n in P.IFACE_OPS} for s in range(2)] for ts in range(nint)]
    mfac = [[(spla.factorized(sp.csc_matrix(ops[ts][s]["inteMass_pena"])), spla.factorized(sp.csc_matrix(ops[ts][s]["inteMass"])))
             for s in range(2)] for ts in range(nint)]
    tTp = [[O.csr64(ops[ts][s]["systTran_pena"].T.tocsr()) for s in range(2)] for ts in range(nint)]
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
    _log(f"interface step {t_iface:.2f} s ({nip} integration points)")
    total = t_body + t_coarse + t_iface
    return {
        "value": 1.0 / total,
        "unit": "ADMM it/s",
        "cores": O.threads(),
        "kind": "port",
        "sample": f"one ADMM iteration at the device run's final state: {len(solve_s)} of {nsub} subdomains sampled "
                  f"(subdomains {used}, {ndof} DOF each: CG_SOLV(1) {iters} SGS-MGPIS iterations in "
                  f"{sum(solve_s):.1f} s, priced x{scale:g} = {t_body:.1f} s), coarse-space correction {t_coarse:.2f} s "
                  f"(fine SpMV + accuProl sampled, globTran_1 and the coarse solve in full), interface step over all "
                  f"{nint} interfaces / {nip} integration points {t_iface:.2f} s",
        "body_s": t_body,
        "coarse_s": t_coarse,
        "iface_s": t_iface,
        "dof_iter_per_s": ndof * sum(iters) / sum(solve_s),
    }
