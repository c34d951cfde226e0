"""GPU parity of the MGPIS device path (SELL-BSR3 SpMV, V-cycle, PCG) against the reference.

Tolerances: SpMV vs reference K*v <= 1e-13 relative (inf-norm); converged
MGPIS solution vs the reference's CG_SOLV solution <= 1e-8 relative L2 (different smoother,
same 1e-14 recursive-residual stop rule, MGPIS.h:175, 198).
"""
import numpy as np
import scipy.sparse as sp
import pytest

from conftest import CASE_PARAMS, golden

pytestmark = pytest.mark.gpu


def _problem(ddpca, case):
    return ddpca.Problem(*CASE_PARAMS[case]).ESTABLISH()


@pytest.mark.parametrize("case", ["beam_s1", "beam_s2", "beam_gl1"])
def test_spmv_matches_reference(ddpca, gpu, case):
    g = golden(case)
    P = _problem(ddpca, case)
    L = P.grid(0).maxiLeve
    M = ddpca.MGPIS.from_problem(P, 0)
    v = ((np.arange(len(g["consForc"])) * 7919 + 13) % 2003) / 2003.0 - 0.5
    y = M.spmv(v)
    ref = g[f"K{L}_Kv"]
    # fp64 SpMV rounding bound: per row |error| <~ nnz_row * eps * (|K| |v|)_row.  Against the
    # identical host matrix the kernel must sit at that bound (1e-14 of the scale); against the
    # reference's K*v the operator-construction rounding (~1e-15 per entry, summed in another
    # order by Eigen) enters too, so 1e-12 of the scale.
    K = P.grid(0).consStif(L)
    scale = (abs(K) @ np.abs(v)).max()
    assert np.abs(y - K @ v).max() <= 1e-14 * scale
    assert np.abs(y - ref).max() <= 1e-12 * scale


@pytest.mark.parametrize("case", ["beam_s2", "beam_gl1"])
def test_table_mode_is_the_same_operator(ddpca, gpu, case):
    """Table mode keeps one copy of each distinct row's block values and groups the rows by type
    (the device numbering changes); every row's blocks stay in the canonical slot order of the
    streamed layout, so y = Kx must agree bit for bit.  The solve's dot products run over the
    other numbering, so the solves agree to solver accuracy (iterations +-1, 1e-10)."""
    P = _problem(ddpca, case)
    n = len(P.grid(0).consForc)
    v = ((np.arange(n) * 7919 + 13) % 2003) / 2003.0 - 0.5
    Ms = ddpca.MGPIS.from_problem(P, 0, table_mode=0)
    Mt = ddpca.MGPIS.from_problem(P, 0, table_mode=2)
    assert np.array_equal(Ms.spmv(v), Mt.spmv(v))
    xs, its, _ = Ms.CG_SOLV(1, P.grid(0).consForc)
    xt, itt, rr = Mt.CG_SOLV(1, P.grid(0).consForc)
    assert rr <= 1e-14 and abs(its - itt) <= 1
    assert np.linalg.norm(xt - xs) <= 1e-10 * np.linalg.norm(xs)
    assert np.linalg.norm(xt - golden(case)["x_mg"]) <= 1e-8 * np.linalg.norm(golden(case)["x_mg"])


@pytest.mark.parametrize("smoother,nu", [(0, 1), (1, 1), (1, 2), (2, 2), (3, 1), (3, 2)])
@pytest.mark.parametrize("case", ["beam_s1", "beam_s2", "beam_gl1"])
def test_cg_solution_matches_reference(ddpca, gpu, case, smoother, nu):
    g = golden(case)
    P = _problem(ddpca, case)
    M = ddpca.MGPIS.from_problem(P, 0, smoother=smoother, nu=nu)
    b = P.grid(0).consForc
    x, it, rr = M.CG_SOLV(1, b)
    xr = g["x_mg"]
    assert rr <= 1e-14
    assert np.linalg.norm(x - xr) <= 1e-8 * np.linalg.norm(xr), (it, np.linalg.norm(x - xr) / np.linalg.norm(xr))


@pytest.mark.parametrize("lowp", [1, 2])
@pytest.mark.parametrize("case", ["beam_s1", "beam_s2", "beam_gl1"])
def test_fp32_stored_preconditioner_keeps_the_solution(ddpca, gpu, case, lowp):
    """precond_fp32: the V-cycle's level operators rounded once to fp32.  The Krylov operator and
    the stop rule stay fp64, so the solution still meets ||r|| <= 1e-14 ||b|| and matches the
    reference's CG_SOLV result like the fp64 path; the preconditioner changes only slightly, so
    the iteration count stays within 2 of the fp64-preconditioned run.  lowp = 2 also stores the
    fine level's smoother copy as block-exponent fp16 (precond_fp32 = 2, 11 significant bits):
    same solution bar; the slender beams under Chebyshev(2) -- the most precision-sensitive
    smoother -- take up to 15 % more iterations (measured 71 -> 74, 76 -> 83, 26 -> 29; bf16
    storage, 8 bits, took 83 / 102 / 46 and was dropped; the DEHW bench workload with block
    Jacobi keeps its 23.6 iterations per solve)."""
    g = golden(case)
    P = _problem(ddpca, case)
    b = P.grid(0).consForc
    x64, it64, _ = ddpca.MGPIS.from_problem(P, 0, smoother=2, nu=2).CG_SOLV(1, b)
    x32, it32, rr = ddpca.MGPIS.from_problem(P, 0, smoother=2, nu=2, precond_fp32=lowp).CG_SOLV(1, b)
    assert rr <= 1e-14
    assert abs(it32 - it64) <= (2 if lowp == 1 else max(2, 0.15 * it64)), (it32, it64)
    assert np.linalg.norm(x32 - g["x_mg"]) <= 1e-8 * np.linalg.norm(g["x_mg"])


@pytest.mark.parametrize("case", ["beam_s1", "beam_gl1"])
def test_diag_pcg_matches_reference(ddpca, gpu, case):
    g = golden(case)
    P = _problem(ddpca, case)
    M = ddpca.MGPIS.from_problem(P, 0)
    x, it, rr = M.CG_SOLV(0, P.grid(0).consForc)
    xr = g["x_diag"]
    assert np.linalg.norm(x - xr) <= 1e-7 * np.linalg.norm(xr)


def test_zero_rhs_returns_zero(ddpca, gpu):
    P = _problem(ddpca, "beam_s1")
    M = ddpca.MGPIS.from_problem(P, 0)
    x, it, rr = M.CG_SOLV(1, np.zeros(len(P.grid(0).consForc)))
    assert it == 0 and not x.any()


def test_vcycle_is_symmetric_positive(ddpca, gpu):
    """The preconditioner must be SPD for CG: u^T M v == v^T M u and v^T M v > 0."""
    P = _problem(ddpca, "beam_s2")
    n = len(P.grid(0).consForc)
    rng = np.random.default_rng(20251017)
    for smoother, nu, f32 in [(0, 1, 0), (1, 1, 0), (2, 2, 0), (2, 2, 1), (1, 1, 2), (2, 2, 2), (3, 1, 0), (3, 2, 1),
                              (3, 2, 2), (1, 1, 3), (3, 2, 3), (4, 2, 3), (4, 2, 1)]:
        M = ddpca.MGPIS.from_problem(P, 0, smoother=smoother, nu=nu, precond_fp32=f32)
        u, v = rng.standard_normal(n), rng.standard_normal(n)
        Mu, Mv = M.MULT_VCYC(u), M.MULT_VCYC(v)
        assert abs(u @ Mv - v @ Mu) <= 1e-10 * abs(u @ Mv)
        assert v @ Mv > 0
    # precond_fp32 = 4: the colour sweeps gather an fp32 copy of the iterate (GsFine::x4; lattice
    # fine transfers, so on a headline subdomain), so the V-cycle is symmetric only to that rounding
    # (a few 1e-8 relative); still positive
    H = ddpca.headline_problem(gl=3).ESTABLISH()
    n = len(H.grid(1).consForc)
    M = ddpca.MGPIS.from_problem(H, 1, smoother=3, nu=2, precond_fp32=4)
    u, v = rng.standard_normal(n), rng.standard_normal(n)
    Mu, Mv = M.MULT_VCYC(u), M.MULT_VCYC(v)
    print("fp32 iterate copy: symmetry", abs(u @ Mv - v @ Mu) / abs(u @ Mv))
    assert abs(u @ Mv - v @ Mu) <= 1e-6 * abs(u @ Mv)
    assert v @ Mv > 0


@pytest.mark.parametrize("f32", [0, 2])
def test_multicolour_gauss_seidel_on_the_headline_subdomains(ddpca, gpu, f32):
    """smoother = 3: multicolour block Gauss-Seidel on the fine level (forward before, backward
    after the coarse correction; the forward sweep's residual r = -U x), block Jacobi with nu = 2
    sweeps below.  On the headline's DEHW-synthetic subdomains (gl = 3) it must reach the same stop
    rule with the same solution as block Jacobi V(1,1) in fewer PCG iterations (CPU study,
    profiles/smoother_study.py at gl = 4: 23-24 -> 18)."""
    P = ddpca.headline_problem(gl=3).ESTABLISH()
    for tv in (0, 1):
        b = P.grid(tv).consForc
        xj, ij, _ = ddpca.MGPIS.from_problem(P, tv, smoother=1, nu=1, omega=-1.7, precond_fp32=f32).CG_SOLV(1, b)
        xg, ig, rr = ddpca.MGPIS.from_problem(P, tv, smoother=3, nu=2, omega=-1.7, precond_fp32=f32).CG_SOLV(1, b)
        print(tv, "block Jacobi", ij, "multicolour GS", ig)
        assert rr <= 1e-14
        assert ig <= 0.85 * ij, (ig, ij)
        assert np.linalg.norm(xg - xj) <= 1e-10 * np.linalg.norm(xj)


def test_fp32_iterate_copy_keeps_the_solution(ddpca, gpu):
    """precond_fp32 = 4: as 3 (int8 V-cycle copies), and the fine colour sweeps gather the iterate
    from an fp32 stride-4 copy (one 16-B load per neighbour block instead of three 8-B fp64 loads;
    the forward sweep and the prolongation write only that copy, the backward sweep also the fp64
    output z).  The products, the epilogues and z stay fp64, so the preconditioner moves only by the
    fp32 rounding of the neighbours' values: PCG (the Krylov operator and vectors, the dot products and
    the stop rule in fp64) must reach the same ||r|| <= 1e-14 ||b|| within one more iteration, and the
    solution within the PCG's tolerance of the int8 run's."""
    P = ddpca.headline_problem(gl=3).ESTABLISH()
    for tv in (0, 1):
        b = P.grid(tv).consForc
        if not np.any(b):
            b = np.random.default_rng(tv).standard_normal(len(b))
        opt = dict(smoother=3, nu=2, omega=-1.7, table_mode=0)
        M3 = ddpca.MGPIS.from_problem(P, tv, precond_fp32=3, **opt)
        M4 = ddpca.MGPIS.from_problem(P, tv, precond_fp32=4, **opt)
        x3, i3, _ = M3.CG_SOLV(1, b)
        x4, i4, rr = M4.CG_SOLV(1, b)
        # the fp32 copy is on (the V-cycles differ by the rounding of the gathered iterate only)
        r = np.random.default_rng(7).standard_normal(len(b))
        z3, z4 = M3.MULT_VCYC(r), M4.MULT_VCYC(r)
        dz = np.linalg.norm(z4 - z3) / np.linalg.norm(z3)
        print(tv, "int8", i3, "int8 + fp32 iterate", i4, "V-cycle difference", dz)
        assert 0.0 < dz <= 1e-5
        assert rr <= 1e-14
        assert i4 <= i3 + 1, (i4, i3)
        assert np.linalg.norm(x4 - x3) <= 1e-10 * np.linalg.norm(x3)


@pytest.mark.parametrize("smoother,mesh", [(1, "headline"), (3, "headline"), (1, "general")])
def test_block_jacobi_fp32_iterate_copy_keeps_the_solution(ddpca, gpu, monkeypatch, smoother, mesh):
    """precond_fp32 = 4 (DDPCA_BJ_X4=0 turns this part off): every block-Jacobi level of the V-cycle (all of them
    under smoother 1 -- the fine one included --, the levels below the colour sweeps under smoother
    3) keeps its iterate in fp32 copies (LevelDev::x4a / x4b): the first sweep (k_jac0 / the fused
    restriction), the sweeps and the prolongation write the copy, the sweeps and the residual
    gather it, and only the level's last sweep writes fp64.  The products and epilogues stay fp64:
    the V-cycle moves by the fp32 rounding of the iterates only, stays symmetric to that rounding,
    and PCG reaches the same ||r|| <= 1e-14 ||b|| within one more iteration.  general: the general
    mesh's rotated support nodes (rotation block entries in the prolongation, k_prolong_rot_x4) and
    explicit transfer lists (k_prolong_x4)."""
    if mesh == "general":
        monkeypatch.setenv("DDPCA_LATTICE", "0")
        P = ddpca.headline_problem(gl=3, **ddpca.GENERAL_FEATURES).ESTABLISH()
    else:
        P = ddpca.headline_problem(gl=3).ESTABLISH()
    # (the exact solve pinned at level 1: a lone gl-3 subdomain otherwise takes it right below the
    # fine level, and under smoother 3 no block-Jacobi level would be left)
    opt = dict(smoother=smoother, nu=2, omega=-1.7, table_mode=0, precond_fp32=4, coarse_level=1)
    for tv in (0, 1):
        b = P.grid(tv).consForc
        if not np.any(b):
            b = np.random.default_rng(tv).standard_normal(len(b))
        monkeypatch.setenv("DDPCA_BJ_X4", "0")
        M = ddpca.MGPIS.from_problem(P, tv, **opt)
        monkeypatch.delenv("DDPCA_BJ_X4")
        Mx = ddpca.MGPIS.from_problem(P, tv, **opt)
        x, i, _ = M.CG_SOLV(1, b)
        xx, ix, rr = Mx.CG_SOLV(1, b)
        rng = np.random.default_rng(11)
        u, v = rng.standard_normal(len(b)), rng.standard_normal(len(b))
        zu, zux = M.MULT_VCYC(u), Mx.MULT_VCYC(u)
        zvx = Mx.MULT_VCYC(v)
        dz = np.linalg.norm(zux - zu) / np.linalg.norm(zu)
        asym = abs(u @ zvx - v @ zux) / (np.linalg.norm(u) * np.linalg.norm(zvx))
        print(tv, "smoother", smoother, "PCG", i, "->", ix, "V-cycle difference", dz, "asymmetry", asym)
        assert 0.0 < dz <= 1e-5
        assert asym <= 1e-6
        assert rr <= 1e-14
        assert ix <= i + 1, (ix, i)
        assert np.linalg.norm(xx - x) <= 1e-10 * np.linalg.norm(x)


@pytest.mark.parametrize("lowp", [3, 4])
def test_colour_ssor_keeps_the_solution(ddpca, gpu, lowp):
    """smoother = 4: multicolour block SSOR on the fine level -- a forward and a backward sweep before
    AND after the coarse correction, the reference's MULT_VCYC smoothing order (MGPIS.h:64-76,
    101-114), with its reuse of the previous sweep's partial sums (three operator passes per V-cycle
    instead of the Gauss-Seidel pair's two).  Same stop rule and solution as smoother 3, in no more
    PCG iterations (CPU study, profiles/r06_study: 18 -> 17 at gl 4 on the int8 copies)."""
    P = ddpca.headline_problem(gl=3).ESTABLISH()
    for tv in (0, 1):
        b = P.grid(tv).consForc
        if not np.any(b):
            b = np.random.default_rng(tv).standard_normal(len(b))
        opt = dict(nu=2, omega=-1.7, table_mode=0, precond_fp32=lowp)  # 4: on the fp32 iterate copy too
        x3, i3, _ = ddpca.MGPIS.from_problem(P, tv, smoother=3, **opt).CG_SOLV(1, b)
        x4, i4, rr = ddpca.MGPIS.from_problem(P, tv, smoother=4, **opt).CG_SOLV(1, b)
        print(tv, "precond_fp32", lowp, "colour GS", i3, "colour SSOR", i4)
        assert rr <= 1e-14
        assert i4 <= i3, (i4, i3)
        assert np.linalg.norm(x4 - x3) <= 1e-10 * np.linalg.norm(x3)


def test_int8_smoother_copy_keeps_the_solution(ddpca, gpu):
    """precond_fp32 = 3: the fine levels' V-cycle copies in block-scaled int8 (nine int8 and a
    scale per 3x3 block) instead of block-exponent fp16.  The Krylov operator and the stop rule stay fp64:
    the same ||r|| <= 1e-14 ||b||, the solution within the PCG's tolerance of the fp16 run's, and
    at most two more iterations on the headline's subdomains (CPU study at gl = 5 on late
    right-hand sides: 18 against 18, profiles/smoother_study.py --ibits 8 --qscale exact)."""
    P = ddpca.headline_problem(gl=3).ESTABLISH()
    for tv in (0, 1):
        b = P.grid(tv).consForc
        if not np.any(b):
            b = np.random.default_rng(tv).standard_normal(len(b))
        opt = dict(smoother=3, nu=2, omega=-1.7, table_mode=0)  # streamed rows: every level has its copy
        x2, i2, _ = ddpca.MGPIS.from_problem(P, tv, precond_fp32=2, **opt).CG_SOLV(1, b)
        x3, i3, rr = ddpca.MGPIS.from_problem(P, tv, precond_fp32=3, **opt).CG_SOLV(1, b)
        print(tv, "fp16 copy", i2, "int8 copy", i3)
        assert rr <= 1e-14
        assert i3 <= i2 + 2, (i3, i2)
        assert np.linalg.norm(x3 - x2) <= 1e-10 * np.linalg.norm(x2)


def _round_blocks(K, node, kind):
    """K with every 3x3 node block rounded as the device stores its V-cycle copy: kind 2 block-exponent
    fp16 (2^e x fp16, e = frexp exponent of the block maximum), kind 3 block-scaled int8 (scale =
    the block maximum / 127 in fp32 with its low 8 bits cleared, values rounded and clamped to +-127)"""
    Kc = K.tocoo()
    key = node[Kc.row].astype(np.int64) * (node.max() + 1) + node[Kc.col]
    _, inv = np.unique(key, return_inverse=True)
    mx = np.zeros(inv.max() + 1)
    np.maximum.at(mx, inv, np.abs(Kc.data))
    if kind == 2:
        e = np.frexp(mx)[1][inv]
        v = np.ldexp(np.ldexp(Kc.data, -e).astype(np.float16).astype(np.float64), e)
    else:
        s32 = (mx / 127.0).astype(np.float32).view(np.uint32) & np.uint32(0xFFFFFF00)
        sc = s32.view(np.float32).astype(np.float64)[inv]
        v = np.clip(np.rint(Kc.data / sc), -127, 127) * sc
    return sp.csr_matrix((v, (Kc.row, Kc.col)), shape=K.shape)


@pytest.mark.parametrize("lowp", [2, 3])
def test_reduced_precision_copy_decodes_the_host_rounding(ddpca, gpu, lowp):
    """The V-cycle's fine-level copy (precond_fp32 = 2: block-exponent fp16, 3: block-scaled int8)
    applied through the device kernels equals the restated rounding of the fp64 operator applied
    in fp64 (only the summation order differs), and differs from the fp64 product by the
    rounding's size -- the records are decoded exactly, not approximately."""
    P = ddpca.headline_problem(gl=3).ESTABLISH()
    tv = 1
    G = P.grid(tv)
    L = G.maxiLeve
    nn = [int(v) for v in P.array("leveCount", tv)]
    flag = np.asarray(P.array("consFlag", tv))
    node = np.nonzero(flag[:3 * nn[L]])[0] // 3
    K = G.consStif(L).tocsr()
    x = np.random.default_rng(7).standard_normal(K.shape[0])
    M = ddpca.MGPIS.from_problem(P, tv, smoother=3, nu=2, omega=-1.7, precond_fp32=lowp, table_mode=0)
    y = M.spmv_vcycle_copy(x)
    yq = _round_blocks(K, node, lowp) @ x
    y64 = K @ x
    rel = np.linalg.norm(y - yq) / np.linalg.norm(yq)
    off = np.linalg.norm(y - y64) / np.linalg.norm(y64)
    print("lowp", lowp, "device vs host rounding", rel, "vs fp64", off)
    assert rel <= 1e-13
    assert off >= (1e-6 if lowp == 2 else 1e-4)
    assert np.array_equal(M.spmv(x), M.spmv(x))  # the fp64 path untouched
    assert np.linalg.norm(M.spmv(x) - y64) <= 1e-13 * np.linalg.norm(y64)


def test_csr_dropin_matches_native(ddpca, gpu):
    """mgpis_gpu_create from the reference layout (condensed CSR) == the native create.  The CSR
    entry point has no coordinates, so it keeps the reference node order while the native create
    renumbers levels >= 1 for gather locality: the sums run in another order, so the two agree
    to the solver accuracy (iterations +-2, solutions 1e-10), not bit for bit."""
    g = golden("beam_s1")
    P = _problem(ddpca, "beam_s1")
    G = P.grid(0)
    L = G.maxiLeve
    import scipy.sparse as sp
    K = [G.consStif(l) for l in range(L + 1)]
    nn = [int(x) for x in P.array("leveCount", 0)]
    flag = G.consFlag
    free_dof = [np.flatnonzero(flag[: 3 * nn[l]]).astype(np.int32) for l in range(L + 1)]
    S = [sp.csr_matrix((P.array("S:w", 0, l), P.array("S:col", 0, l), P.array("S:ptr", 0, l)),
                       shape=(nn[l + 1], nn[l])) for l in range(L)]
    M1 = ddpca.MGPIS.from_csr(nn, free_dof, K, S)
    M2 = ddpca.MGPIS.from_problem(P, 0)
    b = G.consForc
    x1, i1, _ = M1.CG_SOLV(1, b)
    x2, i2, _ = M2.CG_SOLV(1, b)
    assert abs(i1 - i2) <= 2
    assert np.linalg.norm(x1 - x2) <= 1e-10 * np.linalg.norm(x2)
    assert np.linalg.norm(x1 - g["x_mg"]) <= 1e-8 * np.linalg.norm(g["x_mg"])


_CONCURRENT = r'''
import importlib, json, sys, threading
import numpy as np
import scipy.sparse as sp
sys.path.insert(0, sys.argv[1])
D = importlib.import_module("ddpca-admm_amd")
# one problem per thread (no host state shared), the whole fine level as the V-cycle's exact level:
# a dense SPD inverse of 4,455 - 165 rows by rocSOLVER potrf + potri (device_mgpis.hip
# invert_spd_device), the size class of the r04b failures (n = 3468)
probs = [D.Problem("beam", 16, 4, 2, 1, 1, 1, 1).ESTABLISH() for _ in range(5)]
n = len(probs[0].grid(0).consForc)
r = np.random.default_rng(20251017).standard_normal(n)
rounds = []
for rnd in range(2):  # the first round starts cold (rocBLAS / Tensile kernels not loaded yet)
    out, err = [None] * 4, [None] * 4
    def work(i):
        try:
            M = D.MGPIS.from_problem(probs[i], 0, coarse_level=1)
            out[i] = M.MULT_VCYC(r)
        except Exception as e:
            err[i] = repr(e)
    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts: t.start()
    for t in ts: t.join()
    rounds.append((out, err))
serial = D.MGPIS.from_problem(probs[4], 0, coarse_level=1).MULT_VCYC(r)
res = {"n": n, "errors": [e for _, err in rounds for e in err if e],
       "bit_identical": [[bool(o is not None and np.array_equal(o, serial)) for o in out] for out, _ in rounds],
       "max_abs_diff": [[float(np.abs(o - serial).max()) if o is not None else None for o in out] for out, _ in rounds]}
print(json.dumps(res))
'''


_CONCURRENT_CG = r'''
import importlib, json, sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
D = importlib.import_module("ddpca-admm_amd")
# the reference's pattern: MGPIS objects filled one after another, then CG_SOLV(1) on each from an
# omp parallel for (MCONTACT.h:2511-2531); handles alternate between the default V-cycle and the
# headline's (multicolour Gauss-Seidel fine level, int8 / fp32 copies)
opts = [{}, dict(D.HEADLINE_OPTIONS), {}, dict(D.HEADLINE_OPTIONS)]
probs = [D.Problem("beam", 16, 4, 2, 2, 1, 1, 1).ESTABLISH() for _ in range(4)]
n = len(probs[0].grid(0).consForc)
rng = np.random.default_rng(20251017)
rhs = [probs[0].grid(0).consForc] + [rng.standard_normal(n) * 1e3 for _ in range(2)]
res = {"n": n, "errors": [], "phases": {}}
def serial_ref(i):
    M = D.MGPIS.from_problem(probs[i], 0, **opts[i])
    return [M.CG_SOLV(1, b) for b in rhs]
ref = [serial_ref(i) for i in range(4)]
def compare(name, out):
    ok = []
    for i in range(4):
        if out[i] is None:
            ok.append(False)
            continue
        ok.append(all(np.array_equal(x, xr) and it == itr for (x, it, _), (xr, itr, _) in zip(out[i], ref[i])))
    res["phases"][name] = ok
# phase 1: handles created serially on this thread, four threads solving at once, three RHS each
Ms = [D.MGPIS.from_problem(probs[i], 0, **opts[i]) for i in range(4)]
out, err = [None] * 4, [None] * 4
bar = threading.Barrier(4)
def solve(i):
    try:
        bar.wait()
        out[i] = [Ms[i].CG_SOLV(1, b) for b in rhs]
    except Exception as e:
        err[i] = repr(e)
ts = [threading.Thread(target=solve, args=(i,)) for i in range(4)]
for t in ts: t.start()
for t in ts: t.join()
compare("serial_create_concurrent_solve", out)
res["errors"] += [e for e in err if e]
# phase 2: threads 0-2 create their handles (graph capture at create) while thread 3 solves on a
# handle created before -- the r05p hazard (a capture overlapping another thread's synchronous calls)
out, err = [None] * 4, [None] * 4
def create_and_solve(i):
    try:
        bar.wait()
        M = Ms[i] if i == 3 else D.MGPIS.from_problem(probs[i], 0, **opts[i])
        out[i] = [M.CG_SOLV(1, b) for b in rhs]
    except Exception as e:
        err[i] = repr(e)
ts = [threading.Thread(target=create_and_solve, args=(i,)) for i in range(4)]
for t in ts: t.start()
for t in ts: t.join()
compare("concurrent_create_and_solve", out)
res["errors"] += [e for e in err if e]
res["iters"] = [[it for _, it, _ in r] for r in ref]
print(json.dumps(res))
'''


def test_concurrent_cg_solv_bit_identical(ddpca, gpu):
    """The reference calls MGPIS::CG_SOLV(1) on different MGPIS objects from concurrent OpenMP
    threads (MCONTACT.h:2511-2531, MGPIS.h:163-225); include/ddpca_amd.h promises the same for
    handles.  In a fresh process: four host threads each solve three right-hand sides on their own
    handle at once (two handles with the default V-cycle, two with the headline's), then three
    threads create handles -- every PCG graph is captured at create, under the library's capture
    lock -- while the fourth solves.  Every solution and iteration count must equal the serial
    solve's on the same handle options, bit for bit, and no call may fail (the r05p failure was a
    lazily captured graph on a solving thread: hipStreamEndCapture ... previous error during
    capture)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    p = subprocess.run([sys.executable, "-c", _CONCURRENT_CG, root], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ))
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, (p.stdout[-2000:], p.stderr[-3000:])
    res = json.loads(lines[-1])
    print(f"concurrent CG_SOLV, n = {res['n']}: {res}")
    assert not res["errors"], res
    assert all(all(v) for v in res["phases"].values()), res


def test_concurrent_dense_factorisations_bit_identical(ddpca, gpu, tmp_path):
    """Four host threads of one fresh process factorise the same dense SPD matrix at once -- each its
    own MGPIS handle whose exact level is the whole fine level (potrf + potri by rocSOLVER on its own
    stream and rocBLAS handle, invert_spd_device), with the process-wide solver lock OFF
    (DDPCA_SOLVER_LOCK=0) -- twice (the first round with rocBLAS cold).  Every thread's A^-1 r (the
    V-cycle of that handle) must equal a serial handle's bit for bit: the r04b failures were potrf
    info 1479 / 2229 on bit-identical input under 4 in-process ranks."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    env = dict(os.environ, DDPCA_SOLVER_LOCK="0")
    p = subprocess.run([sys.executable, "-c", _CONCURRENT, root], capture_output=True, text=True, timeout=300, env=env)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, (p.stdout[-2000:], p.stderr[-3000:])
    res = json.loads(lines[-1])
    print(f"concurrent potrf/potri, n = {res['n']}: {res}")
    assert not res["errors"], res
    assert all(all(r) for r in res["bit_identical"]), res
