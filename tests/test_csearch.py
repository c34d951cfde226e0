"""Contact search (CSEARCH::BUCKET_SORT / CONTACT_SEARCH / SEGMENT_INTERSECT, CSEARCH.h:205-230,
614-817) restated in csearch.cpp and exported as ddpca_contact_search.  CPU only.

* Conforming faces: on the two-block contact the search must reproduce, point for point, the
  conforming-face rule the host problem builder uses (and the reference's own fixture pins).
* The reference's own curved search: oracle/ref_csearch.cpp lets the reference build its CYLINDER
  example (non-matching, locally refined cylinder surfaces) and run its CONTACT_SEARCH, then feeds
  the same faces / coordinates / bucket counts to ddpca_contact_search: same point count and node
  ids, shape values / basis / weights to 1e-9 (the Newton projections and 2x2 pivoted solves round
  differently), gaps to 1e-12 (absolute; they are ~1e-7)."""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest


def test_conforming_contact_matches_face_rule(ddpca):
    P = ddpca.Problem("twoblock", 0.0, 2)
    node = P.array("ip_node", 0).reshape(-1, 2, 4)
    ref = dict(shap=P.array("ip_shap", 0).reshape(-1, 2, 4), basis=P.array("ip_basis", 0).reshape(-1, 3, 3),
               gap=P.array("ip_gap", 0), w=P.array("ip_w", 0))
    xyz = [P.array("coords", s).reshape(-1, 3) for s in range(2)]
    faces = [np.unique(node[:, s, :], axis=0) for s in range(2)]
    c2 = [xyz[s][faces[s]].mean(axis=1)[:, :2] for s in range(2)]
    out = ddpca.contact_search(xyz[0], faces[0], c2[0], xyz[1], faces[1], c2[1], [8, 8])
    assert len(out["w"]) == len(ref["w"])
    # same points, possibly in another order: key = (master face, slave face, point position)
    def key(nd, sh):
        return [tuple(nd[q].reshape(-1)) + tuple(np.round(sh[q, 0], 12)) for q in range(len(nd))]
    ka, kb = key(out["node"], out["shap"]), key(node, ref["shap"])
    ia = np.array(sorted(range(len(ka)), key=lambda q: ka[q]))
    ib = np.array(sorted(range(len(kb)), key=lambda q: kb[q]))
    assert np.array_equal(out["node"][ia], node[ib])
    for k in ("shap", "basis", "gap", "w"):
        assert np.abs(out[k][ia] - ref[k][ib]).max() <= 1e-12 * max(1.0, np.abs(ref[k]).max()), k


def test_reference_curved_contact_search(tmp_path):
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_csearch"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_csearch is built only where the reference is")
    out = subprocess.run([str(exe), "1", "4", "2", "2e-4"], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ), cwd=tmp_path)
    assert out.returncode in (0, 1), out.stderr[-2000:]
    res = json.loads(out.stderr.strip().splitlines()[-1])
    assert res["ok"], res
    for itf in res["interfaces"]:
        assert itf["ips"] == itf["ips_ref"] > 0 and itf["nodes_equal"], itf


@pytest.mark.parametrize("dist", ["1e-5", "0"])
def test_adaptive_refine_selection_matches_reference(tmp_path, dist):
    """CSEARCH::ADAPTIVE_REFINE's selection (CSEARCH.h:839-956) against the reference's own run on
    its CYLINDER example (oracle/ref_refine.cpp): of the 4096 finest leaf elements per side of the
    first curved contact pair, exactly the elements the reference refines (1024 per side, the band
    within distCrit = 1e-5 of the other surface; none at 0) are the ones ddpca_refine_select flags,
    and isnoRefi agrees.  Then the refinement itself through the library -- CURVEDS::REFINE
    (ddpca_curveds_plan on the side's cylinder surface, exported from the reference's indiPoin
    grid) and MULTIGRID::REFINE with GRLE_CHECK (ddpca_multigrid_refine) on the trees as they were
    before -- must leave each side's tree exactly as the reference's ADAPTIVE_REFINE does: node ids
    and coordinates bitwise (3332 nodes per side on the curved surface), corners, parents, levels,
    patterns, children."""
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_refine"
    if not exe.exists():
        pytest.skip("oracle/_ref/ref_refine is built where the reference is (oracle/Makefile)")
    out = subprocess.run([str(exe), dist], capture_output=True, text=True, timeout=600, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stderr.strip().splitlines()[-1])
    print(res)
    assert res["equal"] and res["trees_equal"], res
    if dist != "0":
        assert res["isnoRefi"] and min(res["refined_ref"]) > 0 and min(res["planSurf"]) > 0, res
    else:
        assert not res["isnoRefi"], res
