"""Rotated-node transfers (MULTIGRID::nodeRota, the CYLINDER / DEHW hubs): the reference builds
realProl with 3x3 blocks w * R_offspring^T * R_parent where exactly one of the two nodes is rotated
(w * I when both are, "only one pattern of nodeRota"; MULTIGRID.h:1141-1181), and the fine
operator lives in the rotated frame.  ``mgpis_gpu_create_prol`` takes realProl as the reference
holds it; blocks that are not w * I run as block entries (k_prolong_rot / k_restrict_rot).

Hierarchy for the tests: the BEAM golden case's fine operator K_L, rotated on a seeded set of
fully free nodes (K_L' = Q^T K_L Q), realProl' by the reference's rule, coarse operators by the
condensed Galerkin product realProl'^T K' realProl'.  The exact solution is x' = Q^T x with x the
reference's own CG_SOLV result (golden ``x_mg``); tolerance 1e-8 relative L2.
With ONE rotation for every rotated node the rotated hierarchy is orthogonally similar to the
plain one, so the device PCG must also need the same iteration count (+-2: the damping estimate's
power iteration starts from a fixed, not rotated, vector)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import CASE_PARAMS, golden


def _axis_rotation(axis, ang):
    a = np.asarray(axis, float)
    a /= np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _hierarchy(ddpca, rot_mode, case="beam_s1", frac=0.2, seed=20251017):
    """(nn, free_dof, K, P, Qfine, b) with rot_mode 'none', 'one' (a single R) or 'many'."""
    P_ = ddpca.Problem(*CASE_PARAMS[case]).ESTABLISH()
    G = P_.grid(0)
    L = G.maxiLeve
    nn = [int(x) for x in P_.array("leveCount", 0)]
    flag = G.consFlag
    free_dof = [np.flatnonzero(flag[: 3 * nn[l]]).astype(np.int32) for l in range(L + 1)]
    fidx = []
    for l in range(L + 1):
        f = np.full(3 * nn[l], -1, np.int64)
        f[free_dof[l]] = np.arange(len(free_dof[l]))
        fidx.append(f)
    S = [sp.csr_matrix((P_.array("S:w", 0, l), P_.array("S:col", 0, l), P_.array("S:ptr", 0, l)),
                       shape=(nn[l + 1], nn[l])) for l in range(L)]
    rng = np.random.default_rng(seed)
    rot = {}
    if rot_mode != "none":
        full = np.flatnonzero(flag[: 3 * nn[L]].reshape(-1, 3).all(axis=1))
        pick = rng.choice(full, size=int(frac * len(full)), replace=False)
        R1 = _axis_rotation([1.0, 2.0, 3.0], 0.7)
        for n in pick:
            if rot_mode == "one":
                rot[int(n)] = R1
            else:
                q, r = np.linalg.qr(rng.standard_normal((3, 3)))
                q = q * np.sign(np.diag(r))
                rot[int(n)] = q if np.linalg.det(q) > 0 else -q
    # realProl[l] by the reference's rule (MULTIGRID.h:1141-1181, 1246-1249), condensed
    P = []
    for l in range(L):
        rows, cols, vals = [], [], []
        Sl = S[l]
        for i in range(nn[l + 1]):
            for k in range(Sl.indptr[i], Sl.indptr[i + 1]):
                p, w = int(Sl.indices[k]), float(Sl.data[k])
                B = w * np.eye(3)
                if i >= nn[l]:
                    ri, rp = i in rot, p in rot
                    if (ri or rp) and not (ri and rp):
                        if ri:
                            B = B @ rot[i].T
                        if rp:
                            B = B @ rot[p]
                for a in range(3):
                    fr = fidx[l + 1][3 * i + a]
                    if fr < 0:
                        continue
                    for c in range(3):
                        fc = fidx[l][3 * p + c]
                        if fc >= 0:
                            rows.append(fr)
                            cols.append(fc)
                            vals.append(B[a, c])
        P.append(sp.csr_matrix((vals, (rows, cols)), shape=(len(free_dof[l + 1]), len(free_dof[l]))))
    # fine operator in the rotated frame, K' = Q^T K Q (rotated nodes are fully free)
    n = len(free_dof[L])
    qr, qc, qv = list(range(n)), list(range(n)), [1.0] * n
    keep = np.ones(n, bool)
    for node, R in rot.items():
        d = fidx[L][3 * node: 3 * node + 3]
        keep[d] = False
        for a in range(3):
            for c in range(3):
                qr.append(d[a])
                qc.append(d[c])
                qv.append(R[a, c])
    qv = np.asarray(qv)
    qv[:n] = keep  # identity only on unrotated dofs
    Q = sp.csr_matrix((qv, (qr, qc)), shape=(n, n))
    K = [None] * (L + 1)
    K[L] = sp.csr_matrix(Q.T @ G.consStif(L) @ Q)
    for l in range(L - 1, -1, -1):
        K[l] = sp.csr_matrix(P[l].T @ K[l + 1] @ P[l])
    for k in K:
        k.sort_indices()
    return nn, free_dof, K, P, Q, Q.T @ G.consForc


def test_rotation_rule_gives_a_similar_hierarchy(ddpca):
    """Host check of the test hierarchy itself: with one R, realProl' = Q_f^T realProl Q_c."""
    nn, fd, K, P, Q, _ = _hierarchy(ddpca, "one")
    _, _, K0, P0, _, _ = _hierarchy(ddpca, "none")
    L = len(K) - 1
    # Q restricted to level L-1's dofs (level-ordered numbering: coarse dofs first in node order)
    nc = len(fd[L - 1])
    Qc = Q[:nc, :nc]
    assert abs(P[L - 1] - Q.T @ P0[L - 1] @ Qc).max() <= 1e-15
    assert abs(K[L - 1] - Qc.T @ K0[L - 1] @ Qc).max() <= 1e-12 * abs(K0[L - 1]).max()


def test_prol_dropin_rejects_a_non_identity_coarse_row(ddpca):
    """realProl's coarse-node rows must be the identity (MULTIGRID.h:1144-1146): EINVAL on the
    host, before any device call (so this runs without a GPU)."""
    nn, fd, K, P, _, _ = _hierarchy(ddpca, "none")
    bad = [p.copy() for p in P]
    bad[0] = bad[0].tolil()
    bad[0][0, 0] = 0.5
    bad[0] = bad[0].tocsr()
    with pytest.raises(ddpca.DdpcaError) as e:
        ddpca.MGPIS.from_prol(nn, fd, K, bad)
    assert e.value.code == -1


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["beam_s1", "beam_gl1"])
def test_rotated_prol_dropin_one_rotation(ddpca, oracle, gpu, case):
    g = golden(case)
    nn, fd, K, P, Q, b = _hierarchy(ddpca, "one", case)
    n0, f0, K0, P0, _, b0 = _hierarchy(ddpca, "none", case)
    x_ref = Q.T @ g["x_mg"]
    M = ddpca.MGPIS.from_prol(nn, fd, K, P)
    x, it, _ = M.CG_SOLV(1, b)
    M0 = ddpca.MGPIS.from_prol(n0, f0, K0, P0)
    x0, it0, _ = M0.CG_SOLV(1, b0)
    assert np.linalg.norm(x - x_ref) <= 1e-8 * np.linalg.norm(x_ref)
    assert np.linalg.norm(x0 - g["x_mg"]) <= 1e-8 * np.linalg.norm(x_ref)
    assert abs(it - it0) <= 2, (it, it0)
    xo, ito, _ = oracle.MgpisOracle(K, P).CG_SOLV(1, b)
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.gpu
@pytest.mark.parametrize("smoother,nu,fp32", [(1, 1, 0), (0, 1, 0), (2, 2, 0), (1, 1, 1), (1, 1, 2), (2, 2, 2),
                                               (1, 1, 3), (3, 2, 3)])
def test_rotated_prol_dropin_many_rotations(ddpca, oracle, gpu, smoother, nu, fp32):
    """Per-node rotations: the reference's both-rotated rule (w * I) makes the hierarchy a
    different, still valid preconditioner; the solution must still be x' = Q^T x.  Every smoother
    (point / block Jacobi, Chebyshev: the first coarse sweep after a block restriction runs as
    k_jac0) and every V-cycle operator storage (fp64, fp32, the finest levels block-exponent fp16 or
    block-scaled int8; the multicolour fine level on int8)."""
    g = golden("beam_s1")
    nn, fd, K, P, Q, b = _hierarchy(ddpca, "many")
    x_ref = Q.T @ g["x_mg"]
    M = ddpca.MGPIS.from_prol(nn, fd, K, P, smoother=smoother, nu=nu, precond_fp32=fp32)
    x, it, _ = M.CG_SOLV(1, b)
    assert np.linalg.norm(x - x_ref) <= 1e-8 * np.linalg.norm(x_ref)
    xo, ito, _ = oracle.MgpisOracle(K, P).CG_SOLV(1, b)
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
    assert it <= 3 * ito + 10, (it, ito)
    # the V-cycle stays a symmetric positive definite preconditioner with block entries
    rng = np.random.default_rng(7)
    u, v = rng.standard_normal(len(b)), rng.standard_normal(len(b))
    Mu, Mv = M.MULT_VCYC(u), M.MULT_VCYC(v)
    assert abs(v @ Mu - u @ Mv) <= 1e-10 * np.linalg.norm(Mu) * np.linalg.norm(v)
    assert u @ Mu > 0


@pytest.mark.gpu
@pytest.mark.parametrize("gl,variant", [(1, "one"), (2, "one"), (2, "many"), (2, "roller")])
def test_reference_rotated_hierarchy_end_to_end(gpu, gl, variant):
    """The reference itself builds a rotated hierarchy: oracle/ref_bind sets MULTIGRID::nodeRota
    on every fifth node of a BEAM mesh before CONSTRAINT(1) (MULTIGRID.h:1102-1181), solves with
    its own CG_SOLV(1), and hands consStif / realProl over through mgpis_gpu_create_prol
    (oracle/ref_bind.hpp); the device solution must match to 1e-8.  "roller": a
    roller on the tip face constrains local dof 0 only, so coarse nodes there have partly
    constrained dofs whose realProl rows / columns are absent (consOper, MULTIGRID.h:1248)."""
    import json
    import os
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_bind"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_bind is built only where the reference is (travels with the snapshot)")
    env = dict(os.environ)
    out = subprocess.run([str(exe), "rot", str(gl), variant], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.splitlines()[-1])
    assert res["rot_ok"] and res["rotated_prol_entries"] > 0, res
