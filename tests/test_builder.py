"""Operator-level builder (ddpca_problem_empty / set_subdomain / set_interface / finalize): the
drop-in entry for a caller that already holds the reference's operators.  CPU-only checks:
exact round trip of every operator the device path reads, and argument validation."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def pair(ddpca):
    P = ddpca.Problem("dehw", 2, 2, 2, 1, 1, 0.3).ESTABLISH()
    subs, ifaces = P.export_operators()
    return P, subs, ifaces


def test_round_trip_is_exact(ddpca, pair):
    P, subs, ifaces = pair
    Q = ddpca.Problem.from_operators(subs, ifaces)
    assert (Q.nsub, Q.nint) == (P.nsub, P.nint)
    for tv in range(P.nsub):
        G, H = P.grid(tv), Q.grid(tv)
        assert G.maxiLeve == H.maxiLeve
        for l in range(G.maxiLeve + 1):
            assert abs(G.consStif(l) - H.consStif(l)).max() == 0.0
        for l in range(G.maxiLeve):
            assert abs(G.realProl(l) - H.realProl(l)).max() == 0.0
        assert np.array_equal(G.consForc, H.consForc)
        assert np.array_equal(G.consFlag, H.consFlag)
        assert np.array_equal(G.nodeCoor, H.nodeCoor)
    for ts in range(P.nint):
        assert np.array_equal(P.array("pemaDiag", ts), Q.array("pemaDiag", ts))
        assert np.array_equal(P.array("inpoNgap", ts), Q.array("inpoNgap", ts))
        for s in range(2):
            for n in ddpca.Problem.IFACE_OPS:
                assert abs(P.csr(n, 2 * ts + s) - Q.csr(n, 2 * ts + s)).max() == 0.0, n


def test_shape_errors_are_reported(ddpca, pair):
    P, subs, ifaces = pair
    bad = [dict(f, ops=[dict(o) for o in f["ops"]]) for f in ifaces]
    bad[0]["ops"][0]["inteMass"] = bad[0]["ops"][0]["inteMass"][:-1, :-1]
    with pytest.raises(ddpca.DdpcaError, match="inteMass"):
        ddpca.Problem.from_operators(subs, bad)


def test_unset_members_are_reported(ddpca):
    import ctypes as C
    L = ddpca.lib()
    h = C.c_void_p()
    assert L.ddpca_problem_empty(1, 1, C.byref(h)) == 0
    try:
        assert L.ddpca_problem_finalize(h) < 0
        assert b"subdomain 0" in L.ddpca_last_error()
    finally:
        L.ddpca_problem_destroy(h)
    with pytest.raises(ddpca.DdpcaError):
        ddpca.Problem.from_operators([], [])


def test_realprol_handover_equals_stencils(ddpca, pair):
    """ddpca_problem_set_subdomain_prol (the reference's realProl instead of scalProl, for rotated
    hierarchies) rebuilds the same stencils on a plain hierarchy: realProl read back is exact."""
    P, subs, ifaces = pair
    subs_p = []
    for tv, s in enumerate(subs):
        G = P.grid(tv)
        d = {k: v for k, v in s.items() if k != "S"}
        d["P"] = [G.realProl(l) for l in range(G.maxiLeve)]
        subs_p.append(d)
    Q = ddpca.Problem.from_operators(subs_p, ifaces)
    for tv in range(P.nsub):
        G, H = P.grid(tv), Q.grid(tv)
        for l in range(G.maxiLeve):
            assert abs(G.realProl(l) - H.realProl(l)).max() == 0.0


def test_hanging_level_shapes(ddpca, pair):
    """The hanging level widens the subdomain's nodal space: interface operators must then have
    3 nnodes_all rows / columns, and the hanging prolongation 3 (nnodes_all - N) x 3 N."""
    import scipy.sparse as sp
    P, subs, ifaces = pair
    nL = int(subs[0]["nnodes"][-1])
    H = sp.csr_matrix((np.full(3, 1.0), (np.arange(3), np.arange(3))), shape=(3, 3 * nL))
    s2 = [dict(s) for s in subs]
    s2[0]["hang"] = (nL + 1, H)
    with pytest.raises(ddpca.DdpcaError, match="pemaInpo_r|systTran"):
        ddpca.Problem.from_operators(s2, ifaces)  # operators still 3N wide
    s2[0]["hang"] = (nL + 2, H)
    with pytest.raises(ddpca.DdpcaError, match="hanging prolongation"):
        ddpca.Problem.from_operators(s2, ifaces)


@pytest.mark.parametrize("kc,kg", [(1, 0), (2, 1)])
def test_refined_face_integration(ddpca, kc, kg):
    """Contact / glued faces integrated over 2^k x 2^k polygons each (bench.py's M3 density):
    4^k times the points of the conforming rule, weights summing to the face area, and the
    mortar mass of a contact side equal to the conforming one to the quadrature's accuracy (the
    triangle rule is not exact for the xi^2 eta^2 term of bilinear x bilinear: 0.5 %)."""
    P0 = ddpca.Problem("dehw", 2, 2, 1, 1, 1, 0.2)
    P1 = ddpca.Problem("dehw", 2, 2, 1, 1, 1, 0.2, kc, kg)
    for ts in range(P0.nint):
        k = kc if ts < 2 else kg
        w0, w1 = P0.array("ip_w", ts), P1.array("ip_w", ts)
        assert len(w1) == 4 ** k * len(w0)
        assert abs(w1.sum() - w0.sum()) <= 1e-14 * w0.sum()
    P0.ESTABLISH()
    P1.ESTABLISH()
    M0, M1 = P0.csr("inteMass", 0), P1.csr("inteMass", 0)
    assert abs(M1 - M0).max() <= 1e-2 * abs(M0).max()
