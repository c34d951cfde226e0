"""Interface-eliminated coarse space (MCONTACT::MULTISCALE_1, MCONTACT.h:1672-2301, and
accuProl, 864-872), host restatement (ddpca-admm_amd/csrc/multiscale.cpp) against the
reference's own operators on identical meshes (golden *_m2 cases, muscSett = 2, doleMcsc = 1).

Tolerance: 1e-12 of each operator's largest entry (the triple products are summed in a
different order than Eigen's); accuProl exactly.  The oracle run on the host-built operators
reproduces the reference's converged ADMM trajectory (iteration count identical).
"""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import CASE_PARAMS, golden, ref_csr

CASES = ["twoblock_f0_m2", "twoblock_f3_m2", "beam_dd_m2"]


def host_problem(ddpca, case):
    """Host-built problem fed with the reference's own integration points (its contact search
    leaves ~1e-18 m of gap noise on coincident faces, which globForc_1 scales by the penalty)."""
    g = golden(case)
    P = ddpca.Problem(*CASE_PARAMS[case])
    for ts in range(P.nint):
        fric, pn, pf = g[f"if{ts}_param"]
        P.set_ips(ts, g[f"if{ts}_ip_node"], g[f"if{ts}_ip_shap"], g[f"if{ts}_ip_basis"], g[f"if{ts}_ip_gap"],
                  g[f"if{ts}_ip_w"], fric, pn, pf)
    P.set_coarse(2, [1] * P.nsub)
    return P.ESTABLISH()


def assert_close(A, B, rtol=1e-12):
    A, B = A.tocsr(), B.tocsr()
    assert A.shape == B.shape
    scale = max(abs(B).max(), 1e-300)
    assert abs(A - B).max() <= rtol * scale


@pytest.mark.parametrize("case", CASES)
def test_coarse_operators_match_reference(ddpca, case):
    g = golden(case)
    P = host_problem(ddpca, case)
    assert np.array_equal(P.array("baseReco"), g["baseReco"])
    assert_close(P.csr("globCoup_1"), ref_csr(g, "globCoup_1"))
    fr = g["globForc_1"]
    assert np.abs(P.array("globForc_1") - fr).max() <= 1e-12 * np.abs(fr).max()
    for tv in range(P.nsub):
        assert_close(P.csr("globTran_D_1", tv), ref_csr(g, f"sd{tv}_globTran_D_1"))
        A, B = P.csr("accuProl", tv), ref_csr(g, f"sd{tv}_accuProl")
        assert A.shape == B.shape and abs(A - B).max() == 0.0
    for ts in range(P.nint):
        for s in range(2):
            assert_close(P.csr("globTran_1", 2 * ts + s), ref_csr(g, f"if{ts}_s{s}_globTran_1"))


@pytest.mark.parametrize("case", CASES)
def test_oracle_on_host_coarse_operators(ddpca, oracle, case):
    """The ADMM oracle with the host-built coarse space follows the reference trajectory."""
    g = golden(case)
    P = host_problem(ddpca, case)
    subs, ifaces = oracle.problem_from_golden(g)
    coarse = dict(globCoup_1=P.csr("globCoup_1"), globForc_1=P.array("globForc_1"), baseReco=P.array("baseReco"),
                  globTran_1=[[P.csr("globTran_1", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D_1=[P.csr("globTran_D_1", tv) for tv in range(P.nsub)],
                  accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    res = oracle.admm(subs, ifaces, maxit=3000, coarse=coarse)
    ref = g["resuMoni"]
    assert res["iters"] == len(ref)
    for tv in range(len(subs)):
        u, ur = res["u"][tv], g[f"sd{tv}_resuDisp"]
        assert np.linalg.norm(u - ur) <= 1e-8 * np.linalg.norm(ur)


def test_set_coarse_rejects_bad_settings(ddpca):
    """muscSett is 0, 1 (MULTISCALE) or 2 (MULTISCALE_1): both bits at once, or out of range, is
    refused (the reference's loop applies either correction, MCONTACT.h:2539-2612)."""
    P = ddpca.Problem(*CASE_PARAMS["twoblock_f0_m2"])
    for bad in (3, 4, -1):
        with pytest.raises(ddpca.DdpcaError):
            P.set_coarse(bad)


def test_rank_local_build_matches_global(ddpca):
    """Each rank of a multi-GPU run builds the coarse rows/columns it owns (ESTABLISH(owner,
    rank)); together they equal the single-process MULTISCALE_1 -- the device sums the RHS
    contributions and the dense rows with RCCL all-reduces."""
    args = ("dehw", 2, 2, 2, 1, 2, 0.3)
    full = ddpca.Problem(*args)
    full.set_coarse(2, [1] * full.nsub)
    full.ESTABLISH()
    base = full.array("baseReco")
    A = full.csr("globCoup_1").toarray()
    f = full.array("globForc_1")
    owner = [0, 1, 0, 1]  # worms on rank 0, wheels on rank 1: every interface crosses ranks
    for rank in range(2):
        P = ddpca.Problem(*args)
        P.set_coarse(2, [1] * P.nsub)
        P.ESTABLISH(owner, rank)
        assert np.array_equal(P.array("baseReco"), base)
        Ar = P.csr("globCoup_1").toarray()
        fr = P.array("globForc_1")
        for tv in range(P.nsub):
            rows = slice(base[tv], base[tv + 1])
            if owner[tv] == rank:
                # bit for bit: every entry sums its own contributions in the same order (the
                # triplet assembly's stable sort), which keeps a multi-rank run's arithmetic equal to
                # the single-rank run's (tests/test_multirank_gpu.py)
                assert np.array_equal(Ar[rows], A[rows])
                assert np.array_equal(fr[rows], f[rows])
                assert abs(P.csr("globTran_D_1", tv) - full.csr("globTran_D_1", tv)).max() == 0.0
            else:
                assert not Ar[rows].any() and not fr[rows].any()
        for ts in range(P.nint):
            body = P.array("iface_body", ts)
            for s in range(2):
                if owner[body[s]] == rank:
                    B = full.csr("globTran_1", 2 * ts + s)
                    assert abs(P.csr("globTran_1", 2 * ts + s) - B).max() == 0.0


@pytest.mark.parametrize("case", ["twoblock_f0_m1", "twoblock_f3_m1"])
def test_latin_operators_match_reference(ddpca, case):
    """LATIN-type coarse space (MCONTACT::MULTISCALE, MCONTACT.h:898-1536, muscSett = 1), host
    restatement (multiscale.cpp MCONTACT::MULTISCALE) against the reference's own operators:
    globCoup (displacement blocks + coarse contact unknowns), globTran / globTran_pena /
    globTran_D per side at 1e-12 of their largest entry, accuProl exactly."""
    g = golden(case)
    P = ddpca.Problem(*CASE_PARAMS[case])
    for ts in range(P.nint):
        fric, pn, pf = g[f"if{ts}_param"]
        P.set_ips(ts, g[f"if{ts}_ip_node"], g[f"if{ts}_ip_shap"], g[f"if{ts}_ip_basis"], g[f"if{ts}_ip_gap"],
                  g[f"if{ts}_ip_w"], fric, pn, pf)
    P.set_coarse(1, [int(x) for x in g["doleMcsc"]])
    P.ESTABLISH()
    assert np.array_equal(P.array("baseReco"), g["baseReco"])
    assert_close(P.csr("globCoup_1"), ref_csr(g, "globCoup"))
    for ts in range(P.nint):
        for s in range(2):
            for name in ("globTran", "globTran_pena", "globTran_D"):
                assert_close(P.csr(name, 2 * ts + s), ref_csr(g, f"if{ts}_s{s}_{name}"))
    for tv in range(P.nsub):
        A, B = P.csr("accuProl", tv), ref_csr(g, f"sd{tv}_accuProl")
        assert A.shape == B.shape and abs(A - B).max() == 0.0


def test_latin_rank_local_build_matches_global(ddpca):
    """Rank-local MULTISCALE (muscSett = 1) builds: each rank assembles its own subdomains' rows
    and its own interface sides' contributions (the coarse contact unknowns of every interface
    are numbered identically on every rank); summed over the ranks -- what the device's RCCL
    all-reduce of the dense rows does -- they equal the single-process operator."""
    args = ("dehw", 2, 2, 2, 1, 2, 0.3)
    full = ddpca.Problem(*args)
    full.set_coarse(1, [1] * full.nsub)
    full.ESTABLISH()
    base = full.array("baseReco")
    A = full.csr("globCoup_1").toarray()
    owner = [0, 1, 0, 1]  # every interface crosses ranks
    total = np.zeros_like(A)
    for rank in range(2):
        P = ddpca.Problem(*args)
        P.set_coarse(1, [1] * P.nsub)
        P.ESTABLISH(owner, rank)
        assert np.array_equal(P.array("baseReco"), base)
        Ar = P.csr("globCoup_1").toarray()
        assert Ar.shape == A.shape
        total += Ar
        for tv in range(P.nsub):
            rows = slice(base[tv], base[tv + 1])
            if owner[tv] == rank:
                assert np.array_equal(Ar[rows], A[rows])
                B = full.csr("accuProl", tv)
                assert abs(P.csr("accuProl", tv) - B).max() == 0.0
            else:
                assert not Ar[rows].any()
        for ts in range(P.nint):
            body = P.array("iface_body", ts)
            for s in range(2):
                if owner[body[s]] == rank:
                    for name in ("globTran", "globTran_pena", "globTran_D"):
                        B = full.csr(name, 2 * ts + s)
                        assert abs(P.csr(name, 2 * ts + s) - B).max() == 0.0
    # the coarse contact rows: one share per side, summed by the setup all-reduce (two terms per
    # entry: the same bits in any order)
    assert np.array_equal(total, A)


@pytest.mark.parametrize("args", [("cylinder", "2", "4", "2"), ("dehw", "2", "2", "0"), ("dehw", "2", "2", "7"),
                                  ("dehw", "1", "2", "0"), ("dehw", "1", "2", "7")],
                         ids=["cylinder-musc2", "dehw-general-musc2", "dehw-rotated-musc2", "dehw-general-musc1",
                              "dehw-rotated-musc1"])
def test_general_tree_coarse_space_matches_reference(tmp_path, args):
    """Both coarse spaces on general trees -- the hanging level past maxiLeve (prolOper[maxiLeve]),
    the nodal rotations' prolongation blocks and CONT_ROTA on the interface operators -- built by the
    library's own ESTABLISH from element trees and integration points (ddpca_problem_set_subdomain_tree,
    multiscale.cpp) against the reference's own MULTISCALE_1 / MULTISCALE on the same input
    (oracle/ref_multiscale.cpp): globCoup(_1), globForc_1, globTran_1 or globTran / globTran_pena /
    globTran_D per side, globTran_D_1 and accuProl per subdomain, and the mortar operators carrying
    CONT_ROTA (systTran, systTran_pena, pemaInpo_r), each within 1e-12 of its largest entry.
    cylinder-musc2: the reference's CYLINDER example (CYLINDER_1.h, locaLeve 4, globInho 2) with
    muscSett = 2 set, run by its own SOLVE (18,336 hanging nodes, 34,323 coarse rows); dehw-*: the
    library's DEHW-synthetic general mesh (bench.py --mesh general at gl 2: contact band refined once
    more, rotated support nodes) handed to a reference MCONTACT; "rotated" also rotates every 7th node
    of every body (contact and hanging nodes among them) on both sides."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_multiscale"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_multiscale is built where the reference is (oracle/Makefile)")
    out = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=900, cwd=tmp_path)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and lines and lines[-1]["ok"], (out.stdout[-3000:], out.stderr[-2000:])
    res = lines[-1]
    assert res["hanging_nodes"] > 0 and res["coarse_rows"] > 0, res
    assert all(v <= 1e-12 for v in res["operators"].values()), res["operators"]
    names = res["operators"].keys()
    want = ["globCoup_1", "globForc_1", "globTran_1[0,0]", "globTran_D_1[0]"] if args[1] == "2" else \
        ["globCoup", "globTran[0,0]", "globTran_pena[0,0]", "globTran_D[0,0]"]
    assert all(w in names for w in want + ["accuProl[0]", "systTran[0,0]", "pemaInpo_r[0,0]"]), names
    if args[0] == "dehw":
        assert res["rotated_nodes"] > 0
