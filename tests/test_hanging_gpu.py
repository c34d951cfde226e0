"""Hanging level (MULTIGRID.h:836-848, 884-910; OUTP_SUB1 1279, ADDITIONAL_FORCE 1257-1261) on the
device ADMM loop, pinned by the CPU oracle.

Locally refined meshes (the reference's CYLINDER) keep hanging nodes -- and coupled nodes -- on a
level past the MGPIS hierarchy: their values are rows of prolOper[maxiLeve] applied to the fine
level's vector, the interface operators see them like any other node, the body-balance RHS folds
their rows back with prolOper^T, and MONITOR's norms include them.  Here a synthetic hanging level
is grafted onto a host-built DEHW-shaped chain: some hanging nodes copy a coupled surface node and
take half of its interface coupling (so u on the MGPIS level is unchanged, the fold is exercised),
others are rotated averages of two nodes (generic 3x3 blocks).  The device run is compared with
the oracle's restatement (oracle.admm with `hang`) at the fixed-k trajectory tolerance, the MGPIS
level's u with the run without the hanging level, and the hanging values with hang @ u.
The reference-built CYLINDER case is tests/test_mcontact_gpu.py::test_cylinder_known_answer.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


def _rot(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def _graft(subs, ifaces, tv, rng, latin=None):
    """Add a hanging level to subdomain tv; returns the hanging prolongation H."""
    s = subs[tv]
    nL = int(s["nnodes"][-1])
    n3 = 3 * nL
    # coupled surface nodes of tv: rows of systTran with entries
    coupled = set()
    for f in ifaces:
        for side in range(2):
            if f["body"][side] == tv:
                T = f["ops"][side]["systTran"].tocsr()
                coupled |= {r // 3 for r in np.flatnonzero(np.diff(T.indptr))}
    coupled = sorted(coupled)
    copies = [coupled[i] for i in rng.choice(len(coupled), size=min(40, len(coupled)), replace=False)]
    nh = len(copies) + 24
    rows, cols, vals = [], [], []
    for k, c in enumerate(copies):  # copy of node c: identity block
        for a in range(3):
            rows.append(3 * k + a), cols.append(3 * c + a), vals.append(1.0)
    for k in range(len(copies), nh):  # rotated average of two nodes
        p, q = rng.choice(nL, size=2, replace=False)
        R = _rot(rng.uniform(0, np.pi))
        for a in range(3):
            for b in range(3):
                rows.append(3 * k + a), cols.append(3 * p + b), vals.append(0.5 * R[a, b])
            rows.append(3 * k + a), cols.append(3 * q + a), vals.append(0.5)
    H = sp.csr_matrix((vals, (rows, cols)), shape=(3 * nh, n3))
    # move half of each copied node's coupling onto its hanging copy
    move = sp.lil_matrix((3 * nh + n3, n3))
    keep = np.ones(n3)
    for k, c in enumerate(copies):
        for a in range(3):
            keep[3 * c + a] = 0.5
            move[n3 + 3 * k + a, 3 * c + a] = 0.5
    Mrow = (sp.vstack([sp.diags(keep), sp.csr_matrix((3 * nh, n3))]) + move.tocsr()).tocsr()  # (n3+3nh) x n3
    for f in ifaces:
        for side in range(2):
            if f["body"][side] != tv:
                continue
            op = f["ops"][side]
            for name in ("systTran", "systTran_pena"):
                op[name] = (Mrow @ op[name]).tocsr()
            op["pemaInpo_r"] = (op["pemaInpo_r"] @ Mrow.T).tocsr()
    if latin is not None:
        for ts, f in enumerate(ifaces):
            for side in range(2):
                if f["body"][side] == tv:
                    latin["globTran_D"][ts][side] = (latin["globTran_D"][ts][side] @ Mrow.T).tocsr()
    s["hang"] = (nL + nh, H)
    return H


@pytest.mark.parametrize("opts", ["default", "HEADLINE_OPTIONS"])
@pytest.mark.parametrize("musc", [0, 1])
def test_hanging_level_matches_oracle(ddpca, oracle, gpu, musc, opts):
    """opts HEADLINE_OPTIONS: the multicolour Gauss-Seidel fine level on operators handed over
    without coordinates (reference node order, colours of a general graph)."""
    O = {} if opts == "default" else dict(getattr(ddpca, opts))
    from test_mcontact_gpu import _oracle_problem, _rows_close
    P = ddpca.Problem("dehw", 2, 2, 2, 1, 2, 0.3)
    if musc:
        P.set_coarse(1, [1] * P.nsub)
    P.ESTABLISH()
    subs, ifaces = P.export_operators()
    coarse = None
    if musc:
        coarse = dict(latin=True, globCoup=P.csr("globCoup_1"), baseReco=P.array("baseReco"),
                      doleMcsc=P.array("doleMcsc"),
                      globTran=[[P.csr("globTran", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                      globTran_pena=[[P.csr("globTran_pena", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                      globTran_D=[[P.csr("globTran_D", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                      accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    k = 30
    base = ddpca.MCONTACT(ddpca.Problem.from_operators(subs, ifaces, coarse=coarse), **O)
    assert base.CONTACT_ANALYSIS(k, check=False) == k
    u_base = [base.get("resuDisp", tv) for tv in range(P.nsub)]
    rng = np.random.default_rng(20251017)
    Hs = {tv: _graft(subs, ifaces, tv, rng, latin=coarse) for tv in (0, 3)}
    Q = ddpca.Problem.from_operators(subs, ifaces, coarse=coarse)
    mc = ddpca.MCONTACT(Q, **O)
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    osubs, oifaces = _oracle_problem(P)
    for tv, H in Hs.items():
        osubs[tv]["hang"] = H
    for ts, f in enumerate(ifaces):
        for side in range(2):
            oifaces[ts]["ops"][side] = f["ops"][side]
    res = oracle.admm(osubs, oifaces, maxit=k, check=False, coarse=coarse)
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-6)
    assert ok, worst
    for tv in range(P.nsub):
        u = mc.get("resuDisp", tv)
        n3 = len(u_base[tv])
        assert np.linalg.norm(u - res["u"][tv]) <= 1e-7 * np.linalg.norm(res["u"][tv])
        # the MGPIS level is the run without the hanging level (same operators after the fold)
        assert np.linalg.norm(u[:n3] - u_base[tv]) <= 1e-9 * np.linalg.norm(u_base[tv])
        if tv in Hs:
            assert len(u) == n3 + Hs[tv].shape[0]
            assert np.abs(u[n3:] - Hs[tv] @ u[:n3]).max() <= 1e-13 * np.abs(u).max()
