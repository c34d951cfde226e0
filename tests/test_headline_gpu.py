"""Parity of the exact option set the headline number is measured with.

bench.py runs MCONTACT on the synthetic DEHW chain with ``HEADLINE_OPTIONS`` (ddpca-admm_amd/
__init__.py: block-Jacobi V(1,1), damping 1.7/lambda_max, fp32 V-cycle levels with block-exponent
fp16 on the two finest, streamed rows (table_mode 0), automatic exact-solve level, 4 PCG
iterations per hipGraph replay) and ``HEADLINE_MUSC`` (interface-eliminated coarse space,
muscSett = 2, doleMcsc = 1).  These tests run that same set:

* reduced chain: ``Problem("dehw", 4, 3, 2, 2, 3, 0.2)`` -- the bench's 8-subdomain batch, 4
  frictional contacts and 6 glued interfaces, 4 MG levels (21k dof per subdomain), so the automatic
  exact-solve level lands on level 1 exactly as at the bench's size, and the fine and next level
  run the fp16 smoother copies.  A fixed-k trajectory (20 ADMM iterations) against the CPU oracle
  (oracle.admm, MCONTACT.h:2493-2845, with exact subdomain solves: the SGS-faithful oracle CG to
  1e-14) on the same host operators: resuMoni rows within 1e-6 relative, displacements 1e-7.
* full size: the bench's own problem (8 x 1.22M dof, 6 levels), one batched ADMM iteration without
  the coarse space; every subdomain's solution of that iteration is the MGPIS solve of its consForc
  (MCONTACT.h:2513-2533 with aux = lambda = 0) and is compared with the oracle's CG_SOLV(1)
  (oracle.cpp, pinned to the reference by test_oracle.py) at 1e-8.  The worms' load is
  zero at that iteration, so their solutions must be exactly zero.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows_close(rows, ref, k, rtol, floor=1e-12):
    a, b = rows[:k], ref[:k]
    scale = np.abs(ref[:k]).max(axis=0, keepdims=True)
    err = np.abs(a - b)
    ok = err <= rtol * np.abs(b) + floor * scale
    return ok.all(), (err / np.maximum(np.abs(b), floor * scale)).max()


def _oracle_problem(P, oracle):
    """Subdomain solves by the SGS-faithful oracle PCG (1e-14, exact to the trajectory tolerance)."""
    subs = []
    for tv in range(P.nsub):
        G = P.grid(tv)
        L = G.maxiLeve
        M = oracle.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
        subs.append(dict(consForc=G.consForc, solve=(lambda b, M=M: M.CG_SOLV(1, b)[0]), consFlag=G.consFlag,
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
    return subs, ifaces, coarse


def test_headline_options_trajectory_matches_oracle(ddpca, oracle, gpu):
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    P = ddpca.Problem("dehw", 4, 3, 2, 2, 3, 0.2)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    assert P.nsub == 8 and P.nint == 10
    mc = ddpca.MCONTACT(P, **H)
    k = 20
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    its = mc.get("pcg_iters")
    subs, ifaces, coarse = _oracle_problem(P, oracle)
    res = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=coarse)
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-6)
    print(f"headline options, reduced chain: last PCG iterations {list(its)}, worst resuMoni rel {worst:.2e}")
    assert ok, worst
    for tv in range(P.nsub):
        u, ur = mc.get("resuDisp", tv), res["u"][tv]
        assert np.linalg.norm(u - ur) <= 1e-7 * np.linalg.norm(ur), tv
    for ts in range(P.nint):
        g, gr = mc.get("inpoGamm", ts), res["gamma"][ts]
        assert np.linalg.norm(g - gr) <= 1e-6 * max(np.linalg.norm(gr), 1e-300), ts


def test_headline_fullsize_batched_solves_match_oracle(ddpca, oracle, gpu):
    H = ddpca.HEADLINE_OPTIONS
    P = ddpca.Problem("dehw", 4, 3, 2, 2, 5, 0.2).ESTABLISH()  # the bench's problem, muscSett = 0
    assert P.nsub == 8
    mc = ddpca.MCONTACT(P, **H)
    assert mc.CONTACT_ANALYSIS(1, check=False) == 1
    its = mc.get("pcg_iters")
    for tv in range(P.nsub):
        G = P.grid(tv)
        flag = G.consFlag
        u = mc.get("resuDisp", tv)
        b = G.consForc
        assert len(b) > 1_000_000
        if not np.any(b):
            assert not np.any(u), tv
            continue
        L = G.maxiLeve
        O = oracle.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
        xo, ito, _ = O.CG_SOLV(1, b)
        del O
        x = u[flag == 1]
        err = np.linalg.norm(x - xo) / np.linalg.norm(xo)
        print(f"subdomain {tv}: device {its[tv]} PCG its (oracle SGS {ito}), rel err {err:.2e}")
        assert err <= 1e-8, (tv, err)


@pytest.mark.parametrize("env", [("DDPCA_STREAMS", "1"), ("DDPCA_FUSE_JAC0", "1")], ids=["one-stream", "fused-jac0"])
def test_schedule_variants_are_bit_identical(ddpca, gpu, monkeypatch, env):
    """Schedule-only variants of the headline path must not change a bit: the two-stream split of
    the body-balance batch and of the mass CG (MgpisDevice / MassBatch ::set_split, default on)
    against one stream, and the V-cycle's first fine sweep fused into k_axpy (k_axpy_jac0, opt-in)
    against the separate k_jac0 (default).  ADMM trajectory, displacements and PCG iteration counts equal
    bit for bit (8 ADMM iterations, reduced chain, headline option set)."""
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    out = {}
    for variant in ("default", "alt"):
        if variant == "alt":
            monkeypatch.setenv(*env)
        else:
            monkeypatch.delenv(env[0], raising=False)
        P = ddpca.Problem("dehw", 4, 3, 2, 2, 3, 0.2)
        P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
        P.ESTABLISH()
        mc = ddpca.MCONTACT(P, **H)
        assert mc.CONTACT_ANALYSIS(8, check=False) == 8
        out[variant] = (mc.monitor().copy(), [mc.get("resuDisp", tv).copy() for tv in range(P.nsub)],
                        np.array(mc.get("pcg_iters")).copy())
        del mc
    assert np.array_equal(out["default"][0], out["alt"][0])
    for a, b in zip(out["default"][1], out["alt"][1]):
        assert np.array_equal(a, b)
    assert np.array_equal(out["default"][2], out["alt"][2])
