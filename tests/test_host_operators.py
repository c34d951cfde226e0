"""Host operator pipeline (MULTIGRID / MCONTACT::ESTABLISH restatement, the producer of every
GPU operand) against the reference's own operators on identical meshes.

Tolerances: coordinates 1e-15 absolute (same arithmetic), operator fingerprints (A * probe,
||A||_F) 1e-12 relative -- the Galerkin products and element stiffness are summed in a
different order than Eigen's, which moves entries at the 1e-16 level; structures (nnz, node
ordering, constrained dofs, contact-node numbering) must be identical.
"""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import CASE_PARAMS, golden, ref_csr


def probe(n):
    """Same integer-exact probe as oracle/ref_harness.cpp."""
    return ((np.arange(n) * 7919 + 13) % 2003) / 2003.0 - 0.5


def close(a, b, rtol):
    return np.abs(a - b).max() <= rtol * max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("case", ["beam_s1", "beam_s2", "beam_gl1"])
def test_single_domain_operators(ddpca, case):
    g = golden(case)
    P = ddpca.Problem(*CASE_PARAMS[case]).ESTABLISH()
    G = P.grid(0)
    assert np.abs(G.nodeCoor - g["coords"]).max() <= 1e-15
    assert np.array_equal(G.consFlag, g["consFlag"])
    assert close(G.consForc, g["consForc"], 1e-14)
    L = G.maxiLeve
    assert L + 1 == len(g["level_rows"])
    for l in range(L + 1):
        K = G.consStif(l)
        fp = g[f"K{l}_fp"]
        assert K.shape == (int(fp[0]), int(fp[1])) and K.nnz == int(fp[2])
        assert abs(np.linalg.norm(K.data) / fp[3] - 1) <= 1e-12
        assert close(K @ probe(K.shape[1]), g[f"K{l}_Kv"], 1e-12)
    for l in range(L):
        Pm = G.realProl(l)
        assert close(Pm @ probe(Pm.shape[1]), g[f"P{l}_Kv"], 1e-13)


def test_full_matrices_entrywise(ddpca):
    g = golden("beam_s1")
    G = ddpca.Problem(*CASE_PARAMS["beam_s1"]).ESTABLISH().grid(0)
    for l in range(2):
        K, Kr = G.consStif(l), ref_csr(g, f"K{l}")
        assert (abs(K - Kr)).max() <= 1e-13 * abs(Kr).max()
    Pm, Pr = G.realProl(0), ref_csr(g, "P0")
    assert (abs(Pm - Pr)).max() == 0.0


@pytest.mark.parametrize("case", ["twoblock_f0", "twoblock_f3", "beam_dd"])
def test_integration_points_match_contact_search(ddpca, case):
    """conforming_face_ips restates CSEARCH::CONTACT_SEARCH for coincident faces."""
    g = golden(case)
    P = ddpca.Problem(*CASE_PARAMS[case])
    for ts in range(P.nint):
        assert np.array_equal(P.array("ip_node", ts), g[f"if{ts}_ip_node"].ravel())
        assert np.abs(P.array("ip_shap", ts) - g[f"if{ts}_ip_shap"].ravel()).max() <= 1e-13
        assert np.abs(P.array("ip_basis", ts) - g[f"if{ts}_ip_basis"].ravel()).max() <= 1e-13
        assert close(P.array("ip_w", ts), g[f"if{ts}_ip_w"], 1e-13)
        assert close(P.array("iface_param", ts), g[f"if{ts}_param"], 1e-13)


@pytest.mark.parametrize("case", ["twoblock_f0", "twoblock_f3", "beam_dd"])
def test_interface_operators(ddpca, case):
    g = golden(case)
    P = ddpca.Problem(*CASE_PARAMS[case]).ESTABLISH()
    for tv in range(P.nsub):
        G = P.grid(tv)
        K, Kr = G.consStif(G.maxiLeve), ref_csr(g, f"sd{tv}_KL")
        assert K.nnz == Kr.nnz
        assert abs(K - Kr).max() <= 1e-13 * abs(Kr).max()
        assert close(G.consForc, g[f"sd{tv}_consForc"], 1e-13)
    names = ["systMass", "systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr", "inpoDisp",
             "inteInpo", "pemaInpo_r"]
    for ts in range(P.nint):
        # coincident faces: the reference's Newton projection leaves ~1e-18 m of gap noise
        assert np.abs(P.array("inpoNgap", ts) - g[f"if{ts}_inpoNgap"]).max() <= 1e-14
        for s in range(2):
            assert np.array_equal(P.array("nodeCont", 2 * ts + s), g[f"if{ts}_s{s}_nodeCont"])
            for n in names:
                A, B = P.csr(n, 2 * ts + s), ref_csr(g, f"if{ts}_s{s}_{n}")
                assert A.shape == B.shape, n
                assert abs(A - B).max() <= 1e-12 * abs(B).max(), n


def test_dehw_generator_shape(ddpca):
    """Synthetic DEHW-shaped chain: 2G subdomains, G contacts + 2(G-1) glued interfaces."""
    P = ddpca.Problem("dehw", 3, 2, 2, 1, 1, 0.2)
    assert P.nsub == 6 and P.nint == 3 + 4
    for ts in range(3):
        assert P.array("iface_param", ts)[0] == 0.2
        assert tuple(P.array("iface_body", ts)) == (2 * ts, 2 * ts + 1)
    for ts in range(3, 7):
        assert P.array("iface_param", ts)[0] == -1.0
    # 2x2 coarse faces refined once -> 4x4 fine faces x 16 integration points
    assert len(P.array("ip_w", 0)) == 16 * 16


def test_rank_local_establish_builds_only_owned(ddpca):
    P = ddpca.Problem("dehw", 2, 2, 2, 1, 1, 0.2)
    owner = [0, 0, 1, 1]
    P.ESTABLISH(owner, rank=1)
    assert len(P.array("consForc", 0)) == 0 and len(P.array("consForc", 2)) > 0
    full = ddpca.Problem("dehw", 2, 2, 2, 1, 1, 0.2).ESTABLISH()
    assert np.array_equal(P.array("consForc", 3), full.array("consForc", 3))


def test_bad_arguments_raise(ddpca):
    with pytest.raises(ddpca.DdpcaError):
        ddpca.Problem("nosuchkind", 1)
    with pytest.raises(ddpca.DdpcaError):
        ddpca.Problem("beam", 7, 2, 2, 1, 2, 1, 1)  # diviNumb not divisible by domaNumb
    P = ddpca.Problem("beam", 8, 2, 2, 1, 1, 1, 1)
    with pytest.raises(ddpca.DdpcaError):
        P.array("consForc", 5)


@pytest.mark.parametrize("args", [("cylinder", "2", "1"), ("cylinder", "4", "2"), ("cylinder", "2", "1", "rot"),
                                  ("beam", "2"), ("beam", "2", "rot")],
                         ids=["cylinder", "cylinder-locaLeve4", "cylinder-rotated", "beam-uniform", "beam-rotated"])
def test_general_tree_pipeline_matches_reference(tmp_path, args):
    """The host operator pipeline on general octrees (ddpca_multigrid_*: TRANSFER with the hanging
    level and coupled nodes, PATCH, STIF_MATR, CONSTRAINT(1) with nodeRota; MULTIGRID.h:722-1255)
    against the reference's own pipeline on the same element trees (oracle/ref_multigrid.cpp).
    CYLINDER_1's meshes: curved cylinders, 4-way inhomogeneous refinement, local refinement towards
    the contact lines (632 / 3136 hanging nodes per subdomain); "rot" puts nodal rotations on every
    seventh node (fine, coarse and hanging ones); BEAM is a uniform tree through the same general
    path.  Positions, level counts, consFlag, dispForc and the PATCHed coordinates must be identical,
    realProl and the hanging rows of prolOper[maxiLeve] exact, consStif within 1e-13 of the level's
    largest entry (element stiffness and Galerkin products summed in another order), consForc 1e-12."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_multigrid"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_multigrid is built where the reference is (oracle/Makefile)")
    out = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=600, cwd=tmp_path)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and lines and lines[-1]["ok"], (out.stdout[-3000:], out.stderr[-2000:])
    for sub in lines[:-1]:
        assert sub["positions_equal"] and sub["levels_equal"] and sub["consFlag_equal"] and sub["dispForc_equal"], sub
        assert sub["coords"] == 0.0 and sub["realProl"] == 0.0 and sub["hang"] == 0.0, sub
        assert sub["K_rel"] <= 1e-13 and sub["consForc_rel"] <= 1e-12, sub
    if args[0] == "cylinder":
        assert lines[-1]["hanging_nodes"] > 0
    if "rot" in args:
        assert all(sub["rotated"] > 0 for sub in lines[:-1])


@pytest.mark.parametrize("rounds", [4])
def test_local_refinement_matches_reference(tmp_path, rounds):
    """MULTIGRID::REFINE (MULTIGRID.h:375-545) through ddpca_multigrid_refine against the
    reference's REFINE on the same box, round by round (oracle/ref_multigrid.cpp "refine"): every
    pattern 0-6 mixed in one round, spliFlag chains (the children a round selects are refined in the
    next), GRLE_CHECK's level balancing (MULTIGRID.h:547-678), planSurf moving the new nodes of a
    curved face (CURVEDS::REFINE's role).  Node ids and coordinates must be bitwise equal, every
    element's corners, parent, level, pattern and children identical, the next split set equal."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_multigrid"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_multigrid is built where the reference is (oracle/Makefile)")
    out = subprocess.run([str(exe), "refine", str(rounds)], capture_output=True, text=True, timeout=600, cwd=tmp_path)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and lines and lines[-1]["ok"], (out.stdout[-3000:], out.stderr[-2000:])
    rr = [l for l in lines if "round" in l]
    assert len(rr) == rounds and all(r["nodes_equal"] and r["elements_equal"] and r["next_split_equal"] for r in rr), rr
    assert any(r["planSurf"] > 0 for r in rr) and rr[-1]["new_elements"] > 0


@pytest.mark.parametrize("args", [("1", "1", "2"), ("0", "1", "3", "rot")], ids=["cylinder-schedule", "rotated"])
def test_refined_tree_pipeline_matches_reference(tmp_path, args):
    """CYLINDER_1's refinement schedule (MESH, CYLINDER_1.h:346-443: globInho rounds of pattern 1,
    globHomo of pattern 0, locaLeve local rounds of pattern 0 along a band of the curved face) run
    through ddpca_multigrid_refine, then the operator pipeline built on the library's own refined
    tree against the reference's REFINE + TRANSFER + STIF_MATR + CONSTRAINT(1): trees identical each
    round, then positions, levels, PATCHed coordinates, consFlag and dispForc identical, realProl and
    the hanging rows exact, consStif 1e-13.  consForc (1e-12) is compared whenever the reference's
    own dispForc is intact: its MULTIGRID.h:1204 shrinks the vector onto a block of itself (an
    Eigen aliasing resize that reads the freed buffer) when consDofv holds more dofs than the fine
    level's constrained rows, so on such inputs its consForc is not defined (reported -1)."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_multigrid"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_multigrid is built where the reference is (oracle/Makefile)")
    out = subprocess.run([str(exe), "refine_pipeline", *args], capture_output=True, text=True, timeout=600, cwd=tmp_path)
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and lines and lines[-1]["ok"], (out.stdout[-3000:], out.stderr[-2000:])
    assert all(l["nodes_equal"] and l["elements_equal"] for l in lines if "round" in l)
    sub = [l for l in lines if "subdomain" in l][0]
    assert sub["positions_equal"] and sub["levels_equal"] and sub["consFlag_equal"] and sub["dispForc_equal"], sub
    assert sub["coords"] == 0.0 and sub["realProl"] == 0.0 and sub["hang"] == 0.0 and sub["K_rel"] <= 1e-13, sub
    assert sub["consForc_rel"] <= 1e-12 and (sub["consForc_rel"] >= 0 or not sub["reference_dispForc_intact"]), sub
    assert sub["hanging"] > 0 and lines[-1]["hanging_nodes"] > 0
    if "rot" in args:
        assert sub["rotated"] > 0
