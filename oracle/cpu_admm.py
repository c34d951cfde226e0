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

`reference_cg_solv` times the reference's OWN MGPIS::CG_SOLV(1) (MGPIS.h:163-225, compiled from
/root/reference into oracle/_ref/ref_harness_portable, `time_cg_ops`) on a worm's and a wheel's
consStif[l] / realProl[l] and the same right-hand side, handed over as raw files; bench.py reports
it as `reference_measured`, the body balance priced by those solves and the rest of the
iteration by the port.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from oracle import oracle as O


def _log(msg: str) -> None:
    print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)


def _state(P, mc):
    nsub, nint = P.nsub, P.nint
    body = [tuple(int(b) for b in P.array("iface_body", ts)) for ts in range(nint)]
    aux = [[mc.get("inteAuxi", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    lam = [[mc.get("inteLagr", 2 * ts + s) for s in range(2)] for ts in range(nint)]
    return nsub, nint, body, aux, lam


def _rhs(P, G, tv, body, aux, lam):
    """consForc + consOper (systTran_pena aux - systTran lambda) of subdomain tv: the body
    balance's right-hand side (ADDITIONAL_FORCE, MCONTACT.h:2520-2524), condensed."""
    flag = G.consFlag == 1
    f = np.zeros(len(flag))
    for ts in range(len(body)):
        for s in range(2):
            if body[ts][s] == tv:
                O.csr_matvec(O.csr64(P.csr("systTran_pena", 2 * ts + s)), aux[ts][s], f)
                f -= O.csr_matvec(O.csr64(P.csr("systTran", 2 * ts + s)), lam[ts][s])
    return G.consForc + f[flag]


def reference_cg_solv(P, mc, exe, subdomains=(1, 0), threads: int | None = None, timeout_s: float = 300.0) -> dict:
    """Wall time of the reference's own MGPIS::CG_SOLV(1) on the given subdomains (default: a
    wheel, then a worm) at the device run's final state: each hierarchy is written to a scratch
    directory as raw CSR files and `exe time_cg_ops` reads it into the reference's MGPIS
    (consStif / realProl members, MGPIS::ESTABLISH untimed) and times CG_SOLV(1) once."""
    nsub, nint, body, aux, lam = _state(P, mc)
    env = dict(os.environ)
    if threads:
        env["OMP_NUM_THREADS"] = str(threads)
    out = []
    for tv in subdomains:
        G = P.grid(tv)
        L = G.maxiLeve
        d = tempfile.mkdtemp(prefix="ddpca_refcg_")
        try:
            meta = [str(L + 1)]
            for kind, n in (("K", L + 1), ("P", L)):
                for l in range(n):
                    base = "K" if kind == "K" else "P"
                    shape = P.array(f"{base}:shape", tv, l)
                    ptr = P.array(f"{base}:ptr", tv, l)
                    meta.append(f"{int(shape[0])} {int(shape[1])} {int(ptr[-1])}")
                    np.ascontiguousarray(ptr, dtype=np.int64).tofile(f"{d}/{kind}{l}.ptr")
                    np.ascontiguousarray(P.array(f"{base}:col", tv, l), dtype=np.int32).tofile(f"{d}/{kind}{l}.col")
                    np.ascontiguousarray(P.array(f"{base}:val", tv, l), dtype=np.float64).tofile(f"{d}/{kind}{l}.val")
            b = _rhs(P, G, tv, body, aux, lam)
            np.ascontiguousarray(b, dtype=np.float64).tofile(f"{d}/b.f64")
            with open(f"{d}/meta.txt", "w") as f:
                f.write("\n".join(meta) + "\n")
            r = subprocess.run([str(exe), "time_cg_ops", d, "1"], capture_output=True, text=True, timeout=timeout_s, env=env)
            if r.returncode != 0:
                raise RuntimeError(f"{exe} time_cg_ops: exit {r.returncode}: {r.stderr[-500:]}")
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rec["subdomain"] = tv
            out.append(rec)
            _log(f"reference CG_SOLV(1) subdomain {tv}: {rec['iters']} iterations, {rec['cg_s']:.2f} s "
                 f"({rec['threads']} threads, true relres {rec['true_relres']:.1e})")
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return {"solves": out, "threads": out[0]["threads"] if out else None}


def price_iteration(P, mc, budget_s: float = 20.0, ref_exe=None, ref_threads: int | None = None) -> dict:
    nsub, nint, body, aux, lam = _state(P, mc)
    fric = [float(P.array("iface_param", ts)[0]) for ts in range(nint)]
    u = [mc.get("resuDisp", tv) for tv in range(nsub)]
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
        b = _rhs(P, G, tv, body, aux, lam)
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
    ref = None
    if ref_exe is not None:
        # the reference's own CG_SOLV(1) on a wheel and a worm: the body balance priced by its
        # solves (x nsub / 2), the coarse space and the interface step by the port as above
        rc = reference_cg_solv(P, mc, ref_exe, (1, 0), ref_threads)
        solves = rc["solves"]
        t_body_ref = nsub / len(solves) * sum(x["cg_s"] for x in solves)
        ref = {"value": 1.0 / (t_body_ref + t_coarse + t_iface), "unit": "ADMM it/s", "cores": rc["threads"],
               "kind": "reference",
               "sample": f"the reference's own MGPIS::CG_SOLV(1) (oracle/_ref/ref_harness_portable time_cg_ops) on "
                         f"subdomains {[x['subdomain'] for x in solves]} ({[x['n'] for x in solves]} DOF, "
                         f"{[x['iters'] for x in solves]} iterations, {[round(x['cg_s'], 2) for x in solves]} s) "
                         f"priced x{nsub / len(solves):g} = {t_body_ref:.1f} s; coarse space {t_coarse:.2f} s and "
                         f"interface step {t_iface:.2f} s by the port",
               "body_s": t_body_ref, "solves": solves,
               "port_over_reference_cg": sum(solve_s[:2]) / max(sum(x["cg_s"] for x in solves), 1e-30)}
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
        "reference_measured": ref,
    }
