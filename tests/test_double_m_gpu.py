"""DOUBLE_M_1 (MCONTACT.h:2303-2341): the interface-eliminated coarse problem solved by its own
MGPIS hierarchy instead of a direct factorisation.

The reference switches to it once globCoup_1 has DIRE_MAXI = 120000 rows (PREP.h:69, MCONTACT.h:
1857-1865) and then calls mgpi_1.CG_SOLV(1, ...) every ADMM iteration (2593-2594).  The device
does the same above that size (or above DDPCA_COARSE_MG_MIN): the hierarchy's level l holds level
max(0, doleMcsc - (Lc - l)) of every subdomain, its transfers are the subdomains' realProl
(block-diagonal), its level operators Galerkin products, and the solve is the same batched MGPIS
PCG to the 1e-14 recursive residual.  Checked against the CPU oracle (exact coarse solves) on the
synthetic chain with the switch forced, and against the reference's own DOUBLE_M_1 run on its
TORSION example with doleMcsc at the fine level (126,750 coarse rows)."""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opts", ["default", "HEADLINE_OPTIONS"])
@pytest.mark.parametrize("dole", [1, 2])
def test_double_m_matches_oracle(ddpca, oracle, gpu, monkeypatch, dole, opts):
    """dole 2 = the fine level (the coarse problem is the whole interface-eliminated problem,
    a 3-level coarse hierarchy); dole 1: two levels.  opts HEADLINE_OPTIONS: the coarse problem's
    own MGPIS takes the multicolour smoother on its fine level too (no coordinates there)."""
    O = {} if opts == "default" else dict(getattr(ddpca, opts))
    from test_mcontact_gpu import _oracle_coarse, _oracle_problem, _rows_close
    monkeypatch.setenv("DDPCA_COARSE_MG_MIN", "1")
    P = ddpca.Problem("dehw", 2, 2, 2, 1, 2, 0.3)
    P.set_coarse(2, [dole] * P.nsub)
    P.ESTABLISH()
    mc = ddpca.MCONTACT(P, **O)
    k = 30
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    subs, ifaces = _oracle_problem(P)
    res = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=_oracle_coarse(P))
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-6)
    assert ok, worst
    for tv in range(P.nsub):
        u, ur = mc.get("resuDisp", tv), res["u"][tv]
        assert np.linalg.norm(u - ur) <= 1e-7 * np.linalg.norm(ur)


def test_double_m_reference_torsion(gpu, tmp_path):
    """The reference's TORSION ({1,2,2}, globHomo 2, muscSett 2) with doleMcsc at the fine level:
    globCoup_1 has 126,750 rows, the reference builds DOUBLE_M_1 and solves it with mgpi_1 every
    iteration; the device (no override: the same 120000-row switch) runs its MGPIS coarse solve on
    the handed-over operators.  Iterations +-1, resuDisp 1e-6, end-face displacement as the
    reference's."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_torsion"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_torsion is built only where the reference is (travels with the snapshot)")
    env = {k: v for k, v in os.environ.items() if k != "DDPCA_COARSE_MG_MIN"}
    out = subprocess.run([str(exe), "2", "-1"], capture_output=True, text=True, timeout=280, env=env, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stderr.strip().splitlines()[-1])
    assert res["coarse_rows"] >= 120000, res
    assert abs(res["iters_gpu"] - res["iters_ref"]) <= 1, res
    assert res["resuDisp_rel"] <= 1e-6, res
    assert abs(res["umax_gpu"] - res["umax_ref"]) <= 1e-6 * res["umax_ref"], res


@pytest.mark.parametrize("fric", [0.3, 0.0])
def test_double_m_latin_matches_oracle(ddpca, oracle, gpu, monkeypatch, fric):
    """DOUBLE_M (MCONTACT.h:1538-1670), the LATIN coarse space's multilevel solve (the reference
    switches to it at DIRE_MAXI = 120000 rows, 1229-1237, and calls mgpi.CG_SOLV(1) every
    iteration, 2558-2559): the coarse contact unknowns coarsen with the slave body's scalProl
    (ficoCotr at every level, 1 unknown per node frictionless, 3 otherwise), the displacement
    blocks with the subdomains' realProl.  Forced on the synthetic chain (LATIN coarse space at
    level 1) against the oracle's exact coarse solves: fixed-k trajectory 1e-6, displacements 1e-7."""
    from test_mcontact_gpu import _oracle_problem, _rows_close
    monkeypatch.setenv("DDPCA_COARSE_MG_MIN", "1")
    P = ddpca.Problem("dehw", 2, 2, 2, 1, 2, fric)
    P.set_coarse(1, [1] * P.nsub)
    P.ESTABLISH()
    mc = ddpca.MCONTACT(P)
    k = 30
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    subs, ifaces = _oracle_problem(P)
    coarse = dict(latin=True, globCoup=P.csr("globCoup_1"), baseReco=P.array("baseReco"),
                  doleMcsc=P.array("doleMcsc"),
                  globTran=[[P.csr("globTran", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_pena=[[P.csr("globTran_pena", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D=[[P.csr("globTran_D", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    res = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=coarse)
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-6)
    assert ok, worst
    for tv in range(P.nsub):
        u, ur = mc.get("resuDisp", tv), res["u"][tv]
        assert np.linalg.norm(u - ur) <= 1e-7 * np.linalg.norm(ur)


@pytest.mark.timeout(700)
def test_double_m_latin_reference_torsion(gpu, tmp_path):
    """The reference's TORSION with the LATIN coarse space (muscSett 1) at the fine level: globCoup
    has 130,680 rows (126,750 displacement dofs + the coarse contact unknowns), the reference
    builds DOUBLE_M and solves it with mgpi.CG_SOLV(1) every iteration; oracle/ref_bind.hpp hands
    over the MULTISCALE output with its coarNode (ddpca_problem_set_coarse_nodes) and the device
    takes its DOUBLE_M MGPIS at the same switch.  Measured: 11 vs 10 iterations, resuDisp 4.9e-13."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_torsion"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_torsion is built only where the reference is (travels with the snapshot)")
    env = {k: v for k, v in os.environ.items() if k != "DDPCA_COARSE_MG_MIN"}
    out = subprocess.run([str(exe), "2", "-1", "1"], capture_output=True, text=True, timeout=640, env=env, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stderr.strip().splitlines()[-1])
    assert res["coarse_rows"] >= 120000, res
    assert abs(res["iters_gpu"] - res["iters_ref"]) <= 1, res
    assert res["resuDisp_rel"] <= 1e-6, res
    assert abs(res["umax_gpu"] - res["umax_ref"]) <= 1e-6 * res["umax_ref"], res
