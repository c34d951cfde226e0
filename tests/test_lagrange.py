"""LAGRANGE host assembly (ddpca-admm_amd/csrc/lagrange.cpp) against the reference's own
MCONTACT::LAGRANGE (MCONTACT.h:2847-3701) on its BLOCK example, on the CPU: oracle/_ref/
ref_lagrange_host lets the reference build BLOCK (domaNumb {1,1,1}, globLeve 1: three stacked
blocks and six plates, 8 interfaces) and run its LAGRANGE(1), then runs the restated assembly on the
same hierarchies and integration points with an exact sparse LU in place of the device BiCGSTAB
(the device path: test_lagrange_gpu.py).

Tolerances: the Newton step count, the non-mortar node order and every node's final active-set
state equal; multipliers (resuLagr_<ts>.txt) within 1e-8 of the largest, displacements (OUTP_SUB1,
resuDisp) within 1e-8 relative -- the reference's BiCGSTAB stops at 1e-14 relative residual.
"""
import json
import os
import subprocess
from pathlib import Path

import pytest

EXE = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_lagrange_host"


@pytest.mark.parametrize("fric,tang", [("0", "0"), ("0.2", "2e6")], ids=["frictionless", "coulomb-slip"])
def test_lagrange_assembly_matches_reference(tmp_path, fric, tang):
    """frictionless: the patch test (every active node carries 1e7, converged at step 0);
    coulomb-slip: friction 0.2 on the contact interfaces and a tangential top load of 20 % of
    the normal one -- the reference's semi-smooth Newton changes 60 then 4 node states and
    converges after step 2."""
    if not EXE.exists():
        pytest.skip("oracle/_ref/ref_lagrange_host is built where the reference is (oracle/Makefile)")
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    out = subprocess.run([str(EXE), "1", fric, tang], capture_output=True, text=True, timeout=900, cwd=tmp_path, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stderr.strip().splitlines()[-1])
    print(res)
    assert res["converged"] and res["newton"] == res["newton_ref"], res
    assert res["nodes_equal"] and res["status_equal"], res
    assert res["lambda_rel"] <= 1e-8 and res["resuDisp_rel"] <= 1e-8, res
    if fric != "0":
        assert res["newton"] >= 1 and res["changes"][0] > 0, res
