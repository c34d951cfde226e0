"""The reference's own ADMM loop on the bench workload's operators (oracle/ref_admm_time.cpp,
profiles/ref_admm_time.py; bench.py's `cpu_baseline.reference_full_iteration`).

The harness fills the reference's MCONTACT with the operators the library exports (subdomain
hierarchies, mortar operators, the interface-eliminated coarse space) and runs the reference's
unmodified CONTACT_ANALYSIS (MCONTACT.h:2493-2845).  Before its timings are trusted, its first
iterations from the zero state must be the CPU oracle's on the same operators (oracle.admm,
MCONTACT.h:2493-2845 restated; subdomain solves by the SGS-faithful oracle CG): resuMoni rows within
1e-7 -- which pins every member the dump hands over (a wrong mapping is O(1))."""
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "oracle" / "_ref" / "ref_admm_time"


@pytest.mark.skipif(not EXE.exists(), reason="oracle/_ref/ref_admm_time is built only where the reference is")
def test_reference_admm_on_dumped_operators_matches_oracle(ddpca, oracle, tmp_path):
    import importlib
    import sys
    sys.path.insert(0, str(ROOT / "profiles"))
    R = importlib.import_module("ref_admm_time")
    M = ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem(gl=2)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    d = tmp_path / "dump"
    d.mkdir()
    R.dump(P, str(d))
    k = 3
    res = R.run(EXE, str(d), stop=k, threads=4)
    rows = np.asarray(res["resuMoni"])
    assert len(res["iteration_s"]) == k and rows.shape[0] >= k, res.keys()
    # the oracle on the same operators (exact subdomain solves)
    subs = []
    for tv in range(P.nsub):
        G = P.grid(tv)
        subs.append(dict(consForc=G.consForc, solve=oracle.DenseSolver(G.consStif(G.maxiLeve)), consFlag=G.consFlag,
                         presc=np.zeros(len(G.consFlag))))
    names = ["systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr", "pemaInpo_r", "inteInpo"]
    ifaces = []
    for ts in range(P.nint):
        fric, pn, pf = P.array("iface_param", ts)
        ifaces.append(dict(body=tuple(int(b) for b in P.array("iface_body", ts)), fric=float(fric),
                           comp=1 if fric == 0.0 else 3, pemaDiag=P.array("pemaDiag", ts),
                           inpoNgap=P.array("inpoNgap", ts),
                           ops=[{n: P.csr(n, 2 * ts + s) for n in names} for s in range(2)]))
    coarse = dict(globCoup_1=P.csr("globCoup_1"), globForc_1=P.array("globForc_1"), baseReco=P.array("baseReco"),
                  globTran_1=[[P.csr("globTran_1", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D_1=[P.csr("globTran_D_1", tv) for tv in range(P.nsub)],
                  accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    ref = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=coarse)["rows"]
    a, b = rows[:k], np.asarray(ref)[:k]
    scale = np.abs(b).max(axis=0, keepdims=True)
    rel = (np.abs(a - b) / np.maximum(np.abs(b), 1e-12 * scale)).max()
    print(f"reference CONTACT_ANALYSIS on the dumped operators vs oracle: worst resuMoni rel {rel:.2e}, "
          f"iterations {res['iteration_s']} s")
    assert rel <= 1e-7, rel
