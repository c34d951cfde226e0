"""The C-ABI library loads, exports every entry point include/ddpca_amd.h declares, and fails
loudly (no silent CPU fallback) when no gfx950 GPU is present."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

HEADER = Path(__file__).resolve().parents[1] / "include" / "ddpca_amd.h"
PROBE_HEADER = HEADER.with_name("ddpca_probe.h")


def declared(header=HEADER):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:ddpca|mgpis|mcontact)_\w+)\s*\(", text)))


def test_exports_every_declared_symbol(ddpca):
    L = ddpca.lib()
    names = declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_probes_live_in_their_own_library(ddpca):
    """The measurement probes (include/ddpca_probe.h) are exported by libddpca_probe.so, not by the
    product library."""
    names = declared(PROBE_HEADER)
    assert names == ["ddpca_probe_grid_barrier", "ddpca_stream_ceiling"]
    P = ddpca.probe_lib()
    assert all(hasattr(P, n) for n in names)
    assert not any(hasattr(ddpca.lib(), n) for n in names)


def test_built_for_gfx950_only():
    so = Path(__file__).resolve().parents[1] / "ddpca-admm_amd" / "libddpca_amd.so"
    data = so.read_bytes()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert other not in data or other == b"sm_"  # no other GPU code objects


def test_device_entry_points_fail_loudly_without_gpu(ddpca):
    if ddpca.gpu_available():
        pytest.skip("GPU present")
    P = ddpca.Problem("beam", 8, 2, 2, 1, 1, 1, 1).ESTABLISH()
    with pytest.raises(ddpca.DdpcaError) as e:
        ddpca.MGPIS.from_problem(P, 0)
    assert e.value.code in (-3, -2)
    with pytest.raises(ddpca.DdpcaError):
        ddpca.MCONTACT(P)


def test_round5_entry_points_refuse_bad_arguments(ddpca):
    """The tree-input ESTABLISH (ddpca_problem_set_subdomain_tree / _set_contact), the timing
    transport (mcontact_gpu_comm_loopback) and the V-cycle-copy SpMV (mgpis_gpu_spmv_copy) check
    their arguments before anything changes (no GPU)."""
    L = ddpca.lib()
    assert L.mcontact_gpu_comm_loopback(None, None) == -1
    assert L.mgpis_gpu_spmv_copy(None, 0, 1, None, None) == -1
    assert L.ddpca_problem_set_contact(None, 0, 0, 1) == -1
    assert L.ddpca_problem_set_subdomain_tree(None, 0, None) == -1
    h = ctypes.c_void_p()
    assert L.ddpca_problem_empty(2, 1, ctypes.byref(h)) == 0
    try:
        assert L.ddpca_problem_set_contact(h, 1, 0, 1) == -1   # interface index
        assert L.ddpca_problem_set_contact(h, 0, 0, 0) == -1   # one body twice
        assert L.ddpca_problem_set_contact(h, 0, 0, 2) == -1   # body out of range
        assert L.ddpca_problem_set_contact(h, 0, 1, 0) == 0
        assert L.ddpca_problem_set_subdomain_tree(h, 0, None) < 0  # no tree
        assert L.ddpca_problem_set_subdomain_tree(h, 2, None) == -1  # subdomain index
    finally:
        L.ddpca_problem_destroy(h)


def test_last_error_is_thread_local_string(ddpca):
    with pytest.raises(ddpca.DdpcaError):
        ddpca.Problem("beam", 1)
    assert b"beam" in ddpca.lib().ddpca_last_error()


def test_partition_helpers():
    import importlib
    part = importlib.import_module("ddpca-admm_amd.partition")
    assert part.block_owner(8, 1) == [0] * 8
    assert part.block_owner(8, 4) == [0, 0, 1, 1, 2, 2, 3, 3]
    assert part.block_owner(8, 8) == list(range(8))
    own = part.lpt_owner([5, 4, 3, 3, 2, 1], 3)
    loads = [sum(d for d, o in zip([5, 4, 3, 3, 2, 1], own) if o == r) for r in range(3)]
    assert max(loads) - min(loads) <= 1
    # the layout rule of bench.py: blocks for equal sizes, LPT otherwise
    assert part.owner_for([7] * 8, 4) == part.block_owner(8, 4)
    assert part.owner_for([5, 4, 3, 3, 2, 1], 3) == own


def test_uneven_dehw_chain_sizes(ddpca):
    """The dehw generator's `uneven` chain (q[10]): group g is 1 + g mod 3 blocks long, so the
    subdomains come in three sizes (DEHW's uneven subdomains, DEHW.h:2238-2258), with the glued
    x planes at the groups' cumulative lengths: every interface still conforming (integration
    points on both sides)."""
    P = ddpca.Problem("dehw", 6, 2, 2, 1, 1, 0.3, 0, 0, 0, 0, 1)
    sizes = [len(P.array("coords", tv)) // 3 for tv in range(P.nsub)]
    assert len(set(sizes)) == 3 and sizes[0] < sizes[2] < sizes[4] and sizes[0] == sizes[6], sizes
    for ts in range(P.nint):
        assert len(P.array("ip_w", ts)) > 0
    P.ESTABLISH()


REF_BIND = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_bind"


@pytest.mark.skipif(not REF_BIND.exists(), reason="oracle/_ref/ref_bind is built only where the reference is")
@pytest.mark.parametrize("fric", ["0", "0.3"])
def test_reference_binding_hands_over_operators_exactly(fric):
    """oracle/ref_bind.hpp (the binding INTEGRATION.md shows) compiled against the reference's own
    classes: the reference's ESTABLISH output, read back through the C ABI, is bit-identical."""
    import json
    import subprocess
    out = subprocess.run([str(REF_BIND), fric, "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.splitlines()[0])
    assert res["ok"] and res["K_rel"] == 0 and res["iface_ops"] == 0


def _one_hex(L):
    """A one-element tree (the unit cube, corners in MULTIGRID's order) through ddpca_multigrid_create."""
    c = ctypes
    xyz = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], np.float64)
    keep = [xyz, np.arange(8, dtype=np.int64), np.array([-1], np.int64), np.zeros(1, np.int64),
            np.array([-1], np.int64), np.zeros(2, np.int64)]
    h = c.c_void_p()
    rc = L.ddpca_multigrid_create(c.c_int64(8), keep[0].ctypes.data_as(c.c_void_p), c.c_int64(1),
                                  *[k.ctypes.data_as(c.c_void_p) for k in keep[1:]], c.c_void_p(0), c.byref(h))
    assert rc == 0
    return h


def _nelem(L, h):
    c = ctypes
    data, count, dt = c.c_void_p(), c.c_int64(), c.c_int()
    assert L.ddpca_multigrid_tree(h, b"parent", c.byref(data), c.byref(count), c.byref(dt)) == 0
    return count.value


def test_multigrid_inputs_are_checked_before_the_tree_changes(ddpca):
    """negative dofs of consDofv / exteForc are refused (not truncated to node 0);
    ddpca_multigrid_refine checks plan_ptr (monotone, nodes in range) and spliFlag (element, child
    0..7) and runs REFINE on a copy, so a refused call leaves the tree and its refinement patterns
    as they were, and a valid call afterwards refines normally."""
    c = ctypes
    L = ddpca.lib()
    h = _one_hex(L)
    try:
        p = lambda a: np.ascontiguousarray(a).ctypes.data_as(c.c_void_p)  # noqa: E731
        for what in (b"consDofv", b"exteForc"):
            for bad in (-1, -2, 24):
                idx, val = np.array([bad], np.int64), np.array([1.0])
                assert L.ddpca_multigrid_set(h, what, c.c_int64(1), p(idx), p(val)) == -1, (what, bad)
        elem, patt = np.array([0], np.int64), np.array([1], np.int64)
        # reversed plan_ptr, node out of range, spliFlag child beyond pattern 1's four children
        cases = [dict(pp=[0, 2, 1], pn=[0, 1, 2], fe=[], fc=[]),
                 dict(pp=[0, 2], pn=[0, 99], fe=[], fc=[]),
                 dict(pp=[0], pn=[0], fe=[0], fc=[9]),
                 dict(pp=[0], pn=[0], fe=[0], fc=[6])]
        for cs in cases:
            npl = len(cs["pp"]) - 1
            pp, pn = np.array(cs["pp"], np.int64), np.array(cs["pn"], np.int64)
            px = np.zeros(3 * max(npl, 1))
            fe, fc = np.array(cs["fe"] or [0], np.int64), np.array(cs["fc"] or [0], np.int64)
            rc = L.ddpca_multigrid_refine(h, c.c_int64(1), p(elem), p(patt), c.c_int64(npl), p(pp), p(pn), p(px),
                                          c.c_int64(len(cs["fe"])), p(fe), p(fc))
            assert rc == -1, cs
            assert _nelem(L, h) == 1, cs
            data, count, dt = c.c_void_p(), c.c_int64(), c.c_int()
            assert L.ddpca_multigrid_tree(h, b"refiPatt", c.byref(data), c.byref(count), c.byref(dt)) == 0
            assert c.cast(data, c.POINTER(c.c_int64))[0] == -1, cs  # the pattern was not written
        z = np.zeros(3)
        rc = L.ddpca_multigrid_refine(h, c.c_int64(1), p(elem), p(np.array([0], np.int64)), c.c_int64(0), p(z), p(z),
                                      p(z), c.c_int64(0), p(z), p(z))
        assert rc == 0 and _nelem(L, h) == 9
    finally:
        L.ddpca_multigrid_destroy(h)


@pytest.mark.parametrize("band", [0, 1], ids=["uniform", "band-refined"])
def test_dehw_interfaces_cover_their_planes(ddpca, band):
    """The synthetic DEHW chain's conforming interfaces (capi_host.cpp conforming_interface(_xyz)):
    every face of the plane on both sides paired (a missing mate is an error, not a skipped face), so
    each interface's integration weights sum to its plane's area, and a contact plane carries
    faces x 16 points x 4^k (the band splits each contact face in four and integrates it one level
    coarser: the same points per area)."""
    import numpy as np
    G, nx, ny, nz, gl, kc, kg = 2, 3, 2, 2, 2, 2, 1
    P = ddpca.Problem("dehw", G, nx, ny, nz, gl, 0.2, kc, kg, band, 0)
    h = 0.01
    for ts in range(P.nint):
        w = P.array("ip_w", ts)
        area = (nx * h) * (ny * h) if ts < G else (ny * h) * (nz * h)
        assert abs(w.sum() - area) <= 1e-12 * area, (ts, w.sum(), area)
        if ts < G:
            faces = nx * ny * 4 ** (gl + band)
            ke = max(kc - 1, 0) if band else kc
            assert len(w) == faces * 16 * 4 ** ke, (ts, len(w))
