"""GPU parity of the other MGPIS drivers -- MULT_SOLV (MGPIS.h:130-160), BiCGSTAB_SOLV
(MGPIS.h:350-432), GMRES_SOLV (MGPIS.h:228-348) -- through the C ABI (mgpis_gpu_mult_solve /
_bicgstab / _gmres) against the reference's own runs (tests/golden/beam_s2_solv.npz) and the
oracle restatement (oracle.cpp, pinned by test_oracle.py).

Two kinds of check, stated per test:
* precSwit = 0 (diagonal preconditioner): the device runs the reference's recurrence with the
  same preconditioner bit for bit, so over a bounded number of iterations it follows the
  oracle's trajectory (solution and residual to 1e-9 relative), and GMRES(0) reproduces the
  reference's full capped run.
* precSwit = 1: the device V-cycle smooths with block Jacobi instead of SGS, so
  the trajectory differs; the solution must satisfy the driver's own stop rule and match the
  reference's solution to the accuracy that stop rule delivers.
"""
import numpy as np
import pytest

from conftest import CASE_PARAMS, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(ddpca, gpu):
    P = ddpca.Problem(*CASE_PARAMS["beam_s2"]).ESTABLISH()
    G = P.grid(0)
    return P, G, golden("beam_s2_solv"), golden("beam_s2")


def _rel(x, ref):
    return np.linalg.norm(x - ref) / np.linalg.norm(ref)


def _oracle(G):
    from oracle import oracle
    L = G.maxiLeve
    return oracle.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])


def test_bicgstab_mg_matches_reference(ddpca, setup):
    """BiCGSTAB_SOLV(1): recursive residual <= 1e-14 ||b|| like the reference (59 iterations
    there); solution vs the reference's BiCGSTAB and CG solutions <= 1e-8 (the reference's own
    true residual is 1.7e-9)."""
    P, G, g, g2 = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    x, it, rr, bd = M.BiCGSTAB_SOLV(1, b)
    print("bicgstab(1)", it, rr, _rel(x, g["x_bicg1"]), _rel(x, g2["x_mg"]))
    assert not bd and rr <= 1e-14 and it < len(b)
    assert _rel(x, g["x_bicg1"]) <= 1e-8 and _rel(x, g2["x_mg"]) <= 1e-8


def test_bicgstab_diag_follows_oracle(ddpca, setup):
    """BiCGSTAB_SOLV(0), first 16 iterations: same recurrence, same diagonal preconditioner as
    the oracle -> same iterate to 1e-9.  Diagonally preconditioned BiCGSTAB on this operator
    amplifies rounding ~10^4-fold per 10 iterations (measured: oracle vs a numpy run of the
    same recurrence differ by 2e-14 at 10, 3.5e-10 at 20, 6e-5 at 30 iterations), so only a
    short prefix of the trajectory is reproducible by any implementation.  The full run must end
    like the reference's physically: the reference ends through rho = 0 after 5547 iterations
    at a true residual of 8.3e-9; the device (measured: no breakdown, capped at rows, true
    residual 1.5e-8) must return the reference's solution to 1e-6."""
    P, G, g, _ = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    x, it, rr, bd = M.BiCGSTAB_SOLV(0, b, maxit=16)
    xo, ito, rro, bdo = _oracle(G).BiCGSTAB_SOLV(0, b, maxit=16)
    print("bicgstab(0) 16", it, rr, rro, _rel(x, xo))
    assert it == ito == 16 and not bd
    assert _rel(x, xo) <= 1e-9 and abs(rr - rro) <= 1e-9 * rro
    x, it, rr, bd = M.BiCGSTAB_SOLV(0, b)
    err = _rel(x, g["x_bicg0"])
    print("bicgstab(0) full", it, rr, bd, err, np.linalg.norm(b - G.consStif(G.maxiLeve) @ x) / np.linalg.norm(b))
    assert it <= len(b) and err <= 1e-6


def test_gmres_diag_reproduces_reference_run(ddpca, setup):
    """GMRES_SOLV(0) to the reference's maxit = rows cap: the reference stagnates at a true
    residual of 0.1166 (restarted GMRES(10) with a diagonal preconditioner); the device run
    ends at the same iteration with the same residual and solution to 1e-9."""
    P, G, g, _ = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    x, it, rr = M.GMRES_SOLV(0, b)
    info = g["solv_info"]
    print("gmres(0)", it, rr, info[9], _rel(x, g["x_gmres0"]))
    assert it == int(info[8]) == len(b)
    assert abs(rr - info[9]) <= 1e-9 * info[9] and _rel(x, g["x_gmres0"]) <= 1e-9


def test_gmres_mg_matches_reference(ddpca, setup):
    """GMRES_SOLV(1) bounded to 300 iterations: the reference's true residual stalls at 5.5e-10
    (above the 1e-12 goal and the 1e-10 stagnation band, so it runs to the cap); the device run
    must reach the same level (<= 1e-9) and the reference's solution to 1e-7."""
    P, G, g, g2 = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    x, it, rr = M.GMRES_SOLV(1, b, maxit=300)
    print("gmres(1) 300", it, rr, _rel(x, g["x_gmres1"]), _rel(x, g2["x_mg"]))
    assert rr <= 1e-9
    assert _rel(x, g["x_gmres1"]) <= 1e-7 and _rel(x, g2["x_mg"]) <= 1e-7


def test_mult_solv_stagnation_rule(ddpca, setup):
    """MULT_SOLV: V-cycles until the last five residual norms stagnate (VECT_MEDI_OSCI < 0.1
    median), not until a tolerance, so the accuracy it returns is set by the cycle's contraction.
    The reference's SGS V(1,1) stops after 378 cycles at a relative residual of 4.4e-6 (error
    2.8e-9 vs the converged CG solution).  Measured on the device: block-Jacobi V(2,2) stops after
    383 cycles at 1.7e-6 (error 1.2e-9) -- as accurate as the reference, asserted at 2x its
    error; V(1,1) with the PCG-tuned damping 1.7/lambda_max contracts too slowly as a stationary
    iteration (0.987 per cycle) and the rule stops it after 188 cycles at 8e-2: the rule itself is
    asserted there (more than four cycles, stopped before the cap), which is the reference's
    behaviour for a slowly contracting cycle too.  Use nu >= 2 for stationary solves."""
    P, G, g, g2 = setup
    b = G.consForc
    ref_err = _rel(g["x_mult"], g2["x_mg"])
    M = ddpca.MGPIS.from_problem(P, 0, smoother=1, nu=2)
    x, it, rr = M.MULT_SOLV(b)
    err = _rel(x, g2["x_mg"])
    print("mult_solv V(2,2)", it, rr, err, "ref", int(g["solv_info"][0]), g["solv_info"][1], ref_err)
    assert 4 <= it < 10000 and err <= 2.0 * ref_err
    # the reported residual is the true one (b - Kx cancels to 1.7e-6: summation-order rounding
    # of Kx enters at ~1e-11 of ||b||)
    assert abs(np.linalg.norm(b - G.consStif(G.maxiLeve) @ x) / np.linalg.norm(b) - rr) <= 1e-10
    M = ddpca.MGPIS.from_problem(P, 0, smoother=1, nu=1)
    x, it, rr = M.MULT_SOLV(b)
    print("mult_solv V(1,1)", it, rr)
    assert 4 <= it < 10000 and rr < 1.0


def test_drivers_zero_rhs(ddpca, setup):
    P, G, _, _ = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    z = np.zeros(len(G.consForc))
    for x, it in [M.MULT_SOLV(z)[:2], M.BiCGSTAB_SOLV(1, z)[:2], M.GMRES_SOLV(1, z)[:2]]:
        assert it == 0 and not x.any()


def test_drivers_reject_bad_arguments(ddpca, setup):
    P, G, _, _ = setup
    M = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    with pytest.raises(ddpca.DdpcaError):
        M.BiCGSTAB_SOLV(2, b)
    with pytest.raises(ddpca.DdpcaError):
        M.GMRES_SOLV(1, b, restart=0)
    with pytest.raises(ddpca.DdpcaError):
        M.GMRES_SOLV(1, b, restart=25)
