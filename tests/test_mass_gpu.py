"""The batched surface-mass solver of the ADMM loop (MassBatch; the reference's interface mass
solves, MCONTACT.h:2671-2704: SimplicialLDLT below 120000 rows, 838-847, Eigen CG above,
2680-2682) on its own through ddpca_mass_solve, and its two forms of the CG step length: alpha
summed inside the update kernel (k_mcg_axpy_fa, the default up to 1024 chunks per system) and the
separate k_mcg_fin launch (larger systems, or forced)."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

pytestmark = pytest.mark.gpu


def _mass_like(n, seed):
    """A surface-mass-like SPD system: a 2-D 9-point lattice mass matrix with random positive scaling."""
    m = int(np.ceil(np.sqrt(n)))
    rng = np.random.default_rng(seed)
    T = sp.diags([np.full(m - 1, 1.0), np.full(m, 4.0), np.full(m - 1, 1.0)], [-1, 0, 1]) / 6.0
    A = sp.kron(T, T).tocsr()[:n, :n]
    d = sp.diags(rng.uniform(0.5, 2.0, n))
    return (d @ A @ d).tocsr()


def test_mass_solve_forms_agree_with_direct_solve(ddpca, gpu, monkeypatch):
    """Systems of 37 rows (one chunk) to 70,000 rows (1,094 chunks: past the fused form's limit, so
    the default rule -- per batch: fused only when every system is within 1024 chunks -- takes the
    separate launch for this batch and the fused one for the batch without it).  Both forms against
    scipy's direct solve (1e-10) and against each other (1e-12): the same CG, alpha summed in
    another order.  (The CG alone: the Chebyshev start is off, DDPCA_MASS_CHEB=0.)"""
    monkeypatch.setenv("DDPCA_MASS_CHEB", "0")
    sizes = [37, 4000, 18915, 70000]
    A = [_mass_like(n, 20251017 + i) for i, n in enumerate(sizes)]
    rng = np.random.default_rng(7)
    b = rng.standard_normal(sum(sizes))
    xs = {}
    for fa in (-1, 0, 1):
        x, its = ddpca.mass_solve(A, b, fuse_alpha=fa)
        xs[fa] = x
        o = 0
        for k, n in enumerate(sizes):
            xr = spla.spsolve(A[k].tocsc(), b[o:o + n])
            err = np.linalg.norm(x[o:o + n] - xr) / np.linalg.norm(xr)
            assert err <= 1e-10, (fa, n, err)
            assert 0 < its[k] < 2000
            o += n
    assert np.array_equal(xs[-1], xs[0])  # 70,000 rows: the default takes the separate launch
    assert np.linalg.norm(xs[1] - xs[0]) <= 1e-12 * np.linalg.norm(xs[0])
    small = A[:3]
    nb = sum(sizes[:3])
    xd, _ = ddpca.mass_solve(small, b[:nb], fuse_alpha=-1)
    xf, _ = ddpca.mass_solve(small, b[:nb], fuse_alpha=1)
    assert np.array_equal(xd, xf)  # within the limit the default is the fused form


@pytest.mark.parametrize("fa", [0, 1], ids=["separate-alpha", "fused-alpha"])
def test_mass_solve_breakdown_keeps_last_iterate(ddpca, gpu, fa, monkeypatch):
    """An indefinite system ([[1, 2], [2, 1]], b on its negative eigenvector: p.q = -2 at the first
    step) next to a healthy one: DDPCA_ENUMERIC, the failing system's x stays its last good iterate
    (x0 = 0) in both forms -- every wave of the fused update sees the same p.q and leaves x, r, z
    alone -- and the healthy system is still solved.  (The indefinite system's spectrum estimate is
    not positive, so the batch would skip the Chebyshev start anyway; it is off here.)"""
    monkeypatch.setenv("DDPCA_MASS_CHEB", "0")
    good = _mass_like(500, 3)
    bad = sp.csr_matrix(np.array([[1.0, 2.0], [2.0, 1.0]]))
    rng = np.random.default_rng(11)
    bg = rng.standard_normal(500)
    b = np.concatenate([bg, [1.0, -1.0]])
    with pytest.raises(ddpca.DdpcaError) as ei:
        ddpca.mass_solve([good, bad], b, fuse_alpha=fa)
    e = ei.value
    assert e.code == -6, e
    assert np.array_equal(e.x[500:], [0.0, 0.0]), e.x[500:]
    xr = spla.spsolve(good.tocsc(), bg)
    assert np.linalg.norm(e.x[:500] - xr) <= 1e-10 * np.linalg.norm(xr)


def test_mass_solve_chebyshev_start(ddpca, gpu, monkeypatch):
    """The default surface-mass solve: a fixed-length Chebyshev iteration on D^-1 M (bounds from 60
    Lanczos steps and Gershgorin at setup, one launch per step, no reductions), then the CG
    restarted from its iterate under the same stop rule (||r|| <= 1e-14 ||b||).  Against scipy's
    direct solve 1e-10 and against the CG alone 1e-11; the CG after the Chebyshev steps takes at most
    a handful of iterations.  An indefinite system in the batch turns the Chebyshev start off for the
    batch (DDPCA_ENUMERIC from the CG as before)."""
    sizes = [37, 4000, 18915]
    A = [_mass_like(n, 20251017 + i) for i, n in enumerate(sizes)]
    rng = np.random.default_rng(9)
    b = rng.standard_normal(sum(sizes))
    monkeypatch.setenv("DDPCA_MASS_CHEB", "1")
    xc, itc = ddpca.mass_solve(A, b)
    monkeypatch.setenv("DDPCA_MASS_CHEB", "0")
    xg, itg = ddpca.mass_solve(A, b)
    print("CG iterations after the Chebyshev steps", list(itc), "CG alone", list(itg))
    o = 0
    for k, n in enumerate(sizes):
        xr = spla.spsolve(A[k].tocsc(), b[o:o + n])
        assert np.linalg.norm(xc[o:o + n] - xr) <= 1e-10 * np.linalg.norm(xr), n
        assert np.linalg.norm(xc[o:o + n] - xg[o:o + n]) <= 1e-11 * np.linalg.norm(xg[o:o + n]), n
        assert 0 <= itc[k] <= 5 and itg[k] > 5, (itc, itg)
        o += n
    monkeypatch.setenv("DDPCA_MASS_CHEB", "1")
    bad = sp.csr_matrix(np.array([[1.0, 2.0], [2.0, 1.0]]))
    with pytest.raises(ddpca.DdpcaError) as ei:
        ddpca.mass_solve([A[0], bad], np.concatenate([b[:37], [1.0, -1.0]]))
    assert ei.value.code == -6


def test_admm_trajectory_fused_vs_separate_alpha(ddpca, gpu, monkeypatch):
    """The ADMM loop with the surface-mass CG's alpha fused (the default at the headline's side
    sizes) against the separate k_mcg_fin launch (DDPCA_MCG_FUSE_ALPHA=0): p.q is summed in another
    order, so not bit-identical -- resuMoni rows within 1e-8 relative and displacements within 1e-9
    after 10 ADMM iterations on the reduced headline chain (the CG alone, DDPCA_MASS_CHEB=0)."""
    monkeypatch.setenv("DDPCA_MASS_CHEB", "0")
    _admm_pair(ddpca, monkeypatch, "DDPCA_MCG_FUSE_ALPHA")


def test_admm_trajectory_chebyshev_vs_cg(ddpca, gpu, monkeypatch):
    """The ADMM loop with the Chebyshev-started surface-mass solves (the default) against the CG
    alone (DDPCA_MASS_CHEB=0): both stop at ||r|| <= 1e-14 ||b||, so the trajectories agree to the
    solves' accuracy -- resuMoni rows 1e-8 relative, displacements 1e-9 after 10 ADMM iterations."""
    _admm_pair(ddpca, monkeypatch, "DDPCA_MASS_CHEB")


def _admm_pair(ddpca, monkeypatch, var):
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv(var, v)
        P = ddpca.headline_problem(gl=3)
        P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
        P.ESTABLISH()
        mc = ddpca.MCONTACT(P, **H)
        assert mc.CONTACT_ANALYSIS(10, check=False) == 10
        out[v] = (mc.monitor().copy(), [mc.get("resuDisp", tv).copy() for tv in range(P.nsub)])
        del mc
    a, b = out["0"][0], out["1"][0]
    scale = np.abs(a).max(axis=0, keepdims=True)
    rel = np.abs(a - b) / np.maximum(np.abs(a), 1e-12 * scale)
    du = max(np.linalg.norm(x - y) / np.linalg.norm(y) for x, y in zip(out["0"][1], out["1"][1]) if np.any(y))
    print(f"{var} 0 vs 1: worst resuMoni rel {rel.max():.2e}, displacements {du:.2e}")
    assert rel.max() <= 1e-8
    assert du <= 1e-9
