"""Parity of the exact option set the headline number is measured with.

bench.py runs MCONTACT on the synthetic DEHW chain with ``HEADLINE_OPTIONS`` (ddpca-admm_amd/
__init__.py: multicolour block Gauss-Seidel on the fine level, block-Jacobi with two sweeps
below, damping 1.7/lambda_max, fp32 V-cycle levels with block-scaled int8 on the three finest,
streamed rows (table_mode 0), automatic exact-solve level, 4 PCG iterations per hipGraph replay) and ``HEADLINE_MUSC`` (interface-eliminated coarse space,
muscSett = 2, doleMcsc = 1).  These tests run that same set:

* reduced chain: ``headline_problem(gl=3)`` -- the bench's workload (``HEADLINE_WORKLOAD``: 8-subdomain
  batch, 4 frictional contacts and 6 glued interfaces, contact faces integrated over 4 x 4
  polygons and glued faces over 2 x 2, i.e. the same integration points per contact node as the
  bench) at 4 MG levels (21k dof per subdomain), so the automatic exact-solve level lands on level 1
  exactly as at the bench's size, and the fine and next level run the int8 smoother copies.  A fixed-k trajectory (20 ADMM iterations) against the CPU oracle
  (oracle.admm, MCONTACT.h:2493-2845, with exact subdomain solves: the SGS-faithful oracle CG to
  1e-14) on the same host operators: resuMoni rows within 1e-7 relative,
  displacements 1e-7, contact tractions 1e-7.
* full size: the bench's own problem (8 x 1.22M dof, 6 levels, coarse space on), three device ADMM
  iterations, then the fourth's body balance and coarse correction against the oracle's started
  from the device's iterate (oracle.admm init= / body_only=; the subdomain solves by the oracle's
  CG_SOLV(1), pinned to the reference by test_oracle.py): u at 1e-8.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows_close(rows, ref, k, rtol, floor=1e-12):
    a, b = rows[:k], ref[:k]
    scale = np.abs(ref[:k]).max(axis=0, keepdims=True)
    err = np.abs(a - b)
    ok = err <= rtol * np.abs(b) + floor * scale
    return ok.all(), (err / np.maximum(np.abs(b), floor * scale)).max()


_VIEW_LOCK = __import__("threading").Lock()  # the problem's array views fill a cache: one thread at a time


def _lazy_solve(P, oracle, tv):
    """One subdomain's oracle CG_SOLV(1), its hierarchy built at the call and dropped after it (the
    full-size problem: a few 1.2M-dof hierarchies in host memory at a time), with a progress line."""
    def solve(b):
        import time
        t = time.time()
        with _VIEW_LOCK:
            G = P.grid(tv)
            L = G.maxiLeve
            K, Pr = [G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)]
        M = oracle.MgpisOracle(K, Pr)
        del K, Pr
        x, it, _ = M.CG_SOLV(1, b)
        print(f"  oracle CG_SOLV(1) subdomain {tv}: {it} iterations, {time.time() - t:.1f} s", flush=True)
        return x
    return solve


def _oracle_problem(P, oracle, lazy=False):
    """Subdomain solves by the SGS-faithful oracle PCG (1e-14, exact to the trajectory tolerance)."""
    subs = []
    for tv in range(P.nsub):
        G = P.grid(tv)
        L = G.maxiLeve
        if lazy:
            solve = _lazy_solve(P, oracle, tv)
        else:
            M = oracle.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
            solve = (lambda b, M=M: M.CG_SOLV(1, b)[0])
        subs.append(dict(consForc=G.consForc, solve=solve, consFlag=G.consFlag, presc=np.zeros(len(G.consFlag))))
    names = ["systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr", "pemaInpo_r", "inteInpo"]
    ifaces = []
    for ts in range(P.nint):
        fric, pn, pf = P.array("iface_param", ts)
        ifaces.append(dict(body=tuple(int(b) for b in P.array("iface_body", ts)), fric=float(fric),
                           comp=1 if fric == 0.0 else 3, pemaDiag=P.array("pemaDiag", ts),
                           inpoNgap=P.array("inpoNgap", ts),
                           ops=[{n: P.csr(n, 2 * ts + s) for n in names} for s in range(2)]))
    coarse = dict(globCoup_1=P.csr("globCoup_1"), globForc_1=P.array("globForc_1"), baseReco=P.array("baseReco"),
                  globTran_1=[[P.csr("globTran_1", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D_1=[P.csr("globTran_D_1", tv) for tv in range(P.nsub)],
                  accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    return subs, ifaces, coarse


@pytest.mark.parametrize("opts", ["HEADLINE_OPTIONS", "HEADLINE_OPTIONS_SMALL"])
def test_headline_options_trajectory_matches_oracle(ddpca, oracle, gpu, opts):
    """Both headline option sets (bench.py takes HEADLINE_OPTIONS_SMALL -- two-sweep block Jacobi --
    on ranks owning at most 4 subdomains, headline_options)."""
    H, M = getattr(ddpca, opts), ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem(gl=3)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    assert P.nsub == 8 and P.nint == 10
    assert len(P.array("ip_w", 0)) == 16 * 6144  # 4 x 4 polygons per contact face
    mc = ddpca.MCONTACT(P, **H)
    k = 20
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    its = mc.get("pcg_iters")
    subs, ifaces, coarse = _oracle_problem(P, oracle)
    res = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=coarse)
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-7)
    print(f"headline options, reduced chain: last PCG iterations {list(its)}, worst resuMoni rel {worst:.2e}")
    assert ok, worst
    for tv in range(P.nsub):
        u, ur = mc.get("resuDisp", tv), res["u"][tv]
        assert np.linalg.norm(u - ur) <= 1e-7 * np.linalg.norm(ur), tv
    for ts in range(P.nint):
        g, gr = mc.get("inpoGamm", ts), res["gamma"][ts]
        assert np.linalg.norm(g - gr) <= 1e-7 * max(np.linalg.norm(gr), 1e-300), ts


def test_headline_density_interface_step_matches_operators(ddpca, oracle, gpu):
    """The per-ip interface kernels at the bench's integration-point density (k_gamma_ip,
    k_traction_ip, the wave-per-node k_inpo_node with its multi-pass lane loop: a contact node
    carries 16 ips per face at ip_contact = 2) against the reference's stored operators
    (MCONTACT.h:2632-2704) on the device's own state: after iteration 1 read lambda^1, after
    iteration 2 read u^2, gamma^2, aux^2, lambda^2 and recompute
      gamma = P(1/2 (inpoLagr_0 lam_0 - inpoLagr_1 lam_1 + pemaInpo_r_0 u_0 - pemaInpo_r_1 u_1)
                - 1/2 pemaDiag inpoNgap)                                        (2632-2668)
      aux   = inteMass_pena^-1 (systTran_pena^T u + inteMass lam + inteInpo gamma) (2671-2684)
      lam'  = lam + inteMass^-1 (systTran_pena^T u - inteMass_pena aux)            (2689-2704)
    with scipy's sparse products and exact sparse LU solves."""
    import scipy.sparse.linalg as spla
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem(gl=3)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    mc = ddpca.MCONTACT(P, **H)
    assert mc.CONTACT_ANALYSIS(1, check=False) == 1
    lam1 = {k: mc.get("inteLagr", k) for k in range(2 * P.nint)}
    assert mc.CONTACT_ANALYSIS(1, check=False) == 1
    u = [mc.get("resuDisp", tv) for tv in range(P.nsub)]
    worst = dict(gamma=0.0, aux=0.0, lam=0.0)
    for ts in range(P.nint):
        fric = float(P.array("iface_param", ts)[0])
        comp = 1 if fric == 0.0 else 3
        body = [int(b) for b in P.array("iface_body", ts)]
        c = -0.5 * P.array("pemaDiag", ts) * P.array("inpoNgap", ts)
        for s, sgn in ((0, 1.0), (1, -1.0)):
            c = c + 0.5 * sgn * (P.csr("inpoLagr", 2 * ts + s) @ lam1[2 * ts + s]
                                 + P.csr("pemaInpo_r", 2 * ts + s) @ u[body[s]])
        gr, _ = oracle._project(c, comp, fric)
        g = mc.get("inpoGamm", ts)
        assert g.shape == gr.shape
        eg = np.linalg.norm(g - gr) / max(np.linalg.norm(gr), 1e-300)
        worst["gamma"] = max(worst["gamma"], eg)
        assert eg <= 1e-12, (ts, eg)
        for s in range(2):
            k = 2 * ts + s
            St, Mm, Mp = P.csr("systTran_pena", k), P.csr("inteMass", k), P.csr("inteMass_pena", k)
            rhs = St.T @ u[body[s]] + Mm @ lam1[k] + P.csr("inteInpo", k) @ g
            ar = spla.spsolve(Mp.tocsc(), rhs)
            a = mc.get("inteAuxi", k)
            ea = np.linalg.norm(a - ar) / max(np.linalg.norm(ar), 1e-300)
            lr = lam1[k] + spla.spsolve(Mm.tocsc(), St.T @ u[body[s]] - Mp @ a)
            el = np.linalg.norm(mc.get("inteLagr", k) - lr) / max(np.linalg.norm(lr), 1e-300)
            worst["aux"], worst["lam"] = max(worst["aux"], ea), max(worst["lam"], el)
            assert ea <= 1e-10, (k, ea)
            assert el <= 1e-8, (k, el)
    print(f"headline density ({len(P.array('ip_w', 0))} ips on contact 0): worst rel. gamma {worst['gamma']:.2e}, "
          f"aux {worst['aux']:.2e}, lambda {worst['lam']:.2e}")


def test_headline_fullsize_step_matches_oracle(ddpca, oracle, gpu):
    """The timed problem itself (8 x 1.22M dof, 6 levels, the interface-eliminated coarse space as
    bench.py runs it) past iteration 0: the device runs 3 ADMM iterations, its aux and lambda of
    every side start the body balance and coarse correction of one oracle iteration (oracle.admm
    init= / body_only=, MCONTACT.h:2511-2612: the SGS-faithful oracle CG_SOLV(1) to 1e-14 per
    subdomain, the dense coarse solve), and the device's u after its 4th iteration must match at
    1e-8.  At iteration 3 every subdomain carries interface tractions, so all eight
    MGPIS solves and the coarse correction enter.  (The interface step's kernels are checked at the
    bench's integration-point density by test_headline_density_interface_step_matches_operators;
    its ip-sized operators at full size -- ~10^9 stored entries -- would not fit this test's time.)"""
    import time
    t0 = time.time()
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem()
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    assert P.nsub == 8 and len(P.grid(0).consFlag) > 1_000_000
    mc = ddpca.MCONTACT(P, **H)
    assert mc.CONTACT_ANALYSIS(3, check=False) == 3
    init = dict(u=[mc.get("resuDisp", tv).copy() for tv in range(P.nsub)],
                aux=[[mc.get("inteAuxi", 2 * ts + s).copy() for s in range(2)] for ts in range(P.nint)],
                lam=[[mc.get("inteLagr", 2 * ts + s).copy() for s in range(2)] for ts in range(P.nint)])
    assert mc.CONTACT_ANALYSIS(1, check=False) == 1
    its = list(mc.get("pcg_iters"))
    ud = [mc.get("resuDisp", tv) for tv in range(P.nsub)]
    del mc
    print(f"device iterations 1-4 done ({time.time() - t0:.0f} s); oracle body balance + coarse correction "
          "of iteration 4 from the device's iterate 3", flush=True)
    subs = [dict(consForc=P.grid(tv).consForc, solve=_lazy_solve(P, oracle, tv), consFlag=P.grid(tv).consFlag,
                 presc=np.zeros(len(P.grid(tv).consFlag))) for tv in range(P.nsub)]
    ifaces = [dict(body=tuple(int(b) for b in P.array("iface_body", ts)),
                   ops=[{n: P.csr(n, 2 * ts + s) for n in ("systTran", "systTran_pena", "inteMass")} for s in range(2)])
              for ts in range(P.nint)]
    print(f"  interface systTran operators ({time.time() - t0:.0f} s)", flush=True)
    coarse = dict(globCoup_1=P.csr("globCoup_1"), globForc_1=P.array("globForc_1"), baseReco=P.array("baseReco"),
                  globTran_1=[[P.csr("globTran_1", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D_1=[], accuProl=[])
    for tv in range(P.nsub):
        coarse["globTran_D_1"].append(P.csr("globTran_D_1", tv))
        coarse["accuProl"].append(P.csr("accuProl", tv))
        print(f"  coarse operators of subdomain {tv}: globTran_D_1 {coarse['globTran_D_1'][-1].nnz} entries "
              f"({time.time() - t0:.0f} s)", flush=True)
    res = oracle.admm(subs, ifaces, maxit=1, check=False, coarse=coarse, init=init, body_only=True, workers=8)
    eu = [np.linalg.norm(ud[tv] - res["u"][tv]) / np.linalg.norm(res["u"][tv]) for tv in range(P.nsub)]
    assert all(np.linalg.norm(res["u"][tv]) > 0 for tv in range(P.nsub))
    print(f"full size, ADMM iteration 4 from the device's iterate 3 ({time.time() - t0:.0f} s): device PCG its {its}; "
          f"rel u per subdomain {['%.1e' % e for e in eu]}")
    assert max(eu) <= 1e-8, eu


@pytest.mark.parametrize("env,opts", [(("DDPCA_STREAMS", "1"), "HEADLINE_OPTIONS"),
                                      (("DDPCA_STREAMS", "1"), "HEADLINE_OPTIONS_SMALL"),
                                      (("DDPCA_TAIL_PACING", "0"), "HEADLINE_OPTIONS"),
                                      (("DDPCA_MCG_PAIR", "0"), "HEADLINE_OPTIONS"),
                                      (("DDPCA_PCG_STREAMS", "4"), "HEADLINE_OPTIONS")],
                         ids=["one-stream", "one-stream-small", "whole-replay-pacing", "unpaired-mass-spmv",
                              "four-part-split"])
def test_schedule_variants_are_bit_identical(ddpca, gpu, monkeypatch, env, opts):
    """Schedule-only variants of the headline path must not change a bit: the two-stream split of
    the body-balance batch and of the mass CG (MgpisDevice / MassBatch ::set_split, default on)
    against one stream, on both option sets; whole-replay pacing to the end of every solve
    against the one-iteration tail graphs; and the fused interface update's mass SpMV reading each
    shared inteMass once for both its systems (k_mcg_spmv2) against one read per system.  ADMM trajectory, displacements and PCG iteration
    counts equal bit for bit (8 ADMM iterations, reduced chain).  (The variants measured slower
    and kept opt-in in round 3 -- stencil-coded copies, XCD-slab placement, four-wave colour
    workgroups, inverses by row, fused first sweeps -- were deleted in round 4)"""
    H, M = getattr(ddpca, opts), ddpca.HEADLINE_MUSC
    out = {}
    for variant in ("default", "alt"):
        if variant == "alt":
            monkeypatch.setenv(*env)
        else:
            monkeypatch.delenv(env[0], raising=False)
        P = ddpca.headline_problem(gl=3)
        P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
        P.ESTABLISH()
        mc = ddpca.MCONTACT(P, **H)
        assert mc.CONTACT_ANALYSIS(8, check=False) == 8
        out[variant] = (mc.monitor().copy(), [mc.get("resuDisp", tv).copy() for tv in range(P.nsub)],
                        np.array(mc.get("pcg_iters")).copy())
        del mc
    assert np.array_equal(out["default"][0], out["alt"][0])
    for a, b in zip(out["default"][1], out["alt"][1]):
        assert np.array_equal(a, b)
    assert np.array_equal(out["default"][2], out["alt"][2])


def test_coarse_correction_kx_from_recursive_residual(ddpca, gpu, monkeypatch):
    """The coarse-space correction takes consStif[L] x as b - r from PCG's recursive residual
    (device_mcontact.hip coarse_correct) instead of the reference's explicit product
    (MCONTACT.h:2585-2587).  On the headline option set (int8 / fp32 V-cycle copies) the two
    schedules must agree: resuMoni rows within 1e-8 relative and displacements within 1e-9 after
    10 ADMM iterations (DDPCA_CS_SPMV=1 forces the explicit fp64 SpMV)."""
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("DDPCA_CS_SPMV", v)
        P = ddpca.headline_problem(gl=3)
        P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
        P.ESTABLISH()
        mc = ddpca.MCONTACT(P, **H)
        assert mc.CONTACT_ANALYSIS(10, check=False) == 10
        out[v] = (mc.monitor().copy(), [mc.get("resuDisp", tv).copy() for tv in range(P.nsub)])
        del mc
    ok, worst = _rows_close(out["0"][0], out["1"][0], k=10, rtol=1e-8)
    du = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(out["0"][1], out["1"][1]) if np.any(b))
    print(f"b - r vs explicit K x: worst resuMoni rel {worst:.2e}, displacements {du:.2e}")
    assert ok, worst
    assert du <= 1e-9, du


def _oracle_problem_no_coarse(P, oracle):
    """_oracle_problem without a coarse space, plus each subdomain's hanging rows (oracle.admm's
    `hang`: OUTP_SUB1's prolOper[maxiLeve] rows, MULTIGRID.h:1279, and their fold into the body
    balance, 1257-1261)."""
    subs = []
    for tv in range(P.nsub):
        G = P.grid(tv)
        L = G.maxiLeve
        M = oracle.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
        n3 = 3 * int(P.array("leveCount", tv)[-1])  # the MGPIS fine level (consFlag also covers the hanging level)
        s = dict(consForc=G.consForc, solve=(lambda b, M=M: M.CG_SOLV(1, b)[0]), consFlag=G.consFlag[:n3],
                 presc=np.zeros(n3))
        H = G.hangRows()
        if H.shape[0]:
            s["hang"] = H
        subs.append(s)
    names = ["systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr", "pemaInpo_r", "inteInpo"]
    ifaces = []
    for ts in range(P.nint):
        fric, pn, pf = P.array("iface_param", ts)
        ifaces.append(dict(body=tuple(int(b) for b in P.array("iface_body", ts)), fric=float(fric),
                           comp=1 if fric == 0.0 else 3, pemaDiag=P.array("pemaDiag", ts),
                           inpoNgap=P.array("inpoNgap", ts),
                           ops=[{n: P.csr(n, 2 * ts + s) for n in names} for s in range(2)]))
    return subs, ifaces


def test_band_sweeps_match_full_sweeps(ddpca, gpu, monkeypatch):
    """Band mode of the multicolour fine level (GsFine::band): on the general mesh the
    colours cover only the nodes the band level adds and their neighbours (the rest is level L-1's),
    and the ADMM trajectory with it matches the full-level sweeps' to the PCG tolerance -- the
    preconditioner changes, the 1e-14 stop on the same fp64 operator does not: resuMoni rows 1e-7
    (SURVEY §8 c4), displacements 1e-9.  The headline's uniform fine level has no band."""
    monkeypatch.setenv("DDPCA_LATTICE", "0")
    H, M = ddpca.HEADLINE_OPTIONS, ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem(gl=3, **ddpca.GENERAL_FEATURES)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    k = 8
    runs = {}
    for band in ("1", "0"):
        monkeypatch.setenv("DDPCA_GS_BAND", band)
        mc = ddpca.MCONTACT(P, **H)
        assert mc.CONTACT_ANALYSIS(k, check=False) == k
        runs[band] = (mc.get("gs_rows"), mc.monitor(), [mc.get("resuDisp", tv) for tv in range(P.nsub)])
        del mc
    (rb, mb, ub), (rf, mf, uf) = runs["1"], runs["0"]
    print("gs rows band / ring / far", list(rb), "full", list(rf))
    assert rb[1] > 0 and rb[2] > 0 and rb[0] < 0.6 * rf[0] and rf[1] == rf[2] == 0
    ok, worst = _rows_close(mb, mf, k=k, rtol=1e-7)
    assert ok, worst
    for a, b in zip(ub, uf):
        assert np.linalg.norm(a - b) <= 1e-9 * np.linalg.norm(b)
    monkeypatch.delenv("DDPCA_GS_BAND")
    Q = ddpca.headline_problem(gl=3).ESTABLISH()
    mq = ddpca.MCONTACT(Q, **H)
    rows = mq.get("gs_rows")
    assert rows[1] == rows[2] == 0 and rows[0] > 0


@pytest.mark.parametrize("opts", ["HEADLINE_OPTIONS"])
def test_general_mesh_trajectory_matches_oracle(ddpca, oracle, gpu, monkeypatch, opts):
    """bench.py's general-mesh line at reduced size: the DEHW chain with its contact band refined
    once more (DEHW.h:1562 -- a general tree: TRANSFER renumbers it, hanging nodes on the level past
    the MGPIS hierarchy, contact and glued faces in the band refined) and rotated support nodes
    (DEHW.h:197 -- prolongation blocks off w I, R^T K R), the interface-eliminated coarse space DEHW
    runs (muscSett = 2, doleMcsc = 1: DEHW.h:2222, 2239), built by the host MULTISCALE_1 on this
    general tree (the hanging level's rows and the rotation blocks in Q / H / Rc, multiscale.cpp;
    pinned to the reference's own by tests/test_coarse_space.py::test_general_tree_coarse_space_matches_reference)
    and prolonged on the device by the scalar stencil plus CSR rows for the nodes whose chain meets
    a rotation block; the lattice transfers switched off (DDPCA_LATTICE=0: explicit index lists),
    the bench's option set at 8 subdomains per GPU.  A fixed-k trajectory (8 ADMM iterations)
    against the CPU oracle on the same host operators, with the hanging rows and the coarse space:
    resuMoni rows 1e-7 relative, displacements (incl. the hanging level) 1e-7, contact
    tractions 1e-7."""
    monkeypatch.setenv("DDPCA_LATTICE", "0")
    H, M = getattr(ddpca, opts), ddpca.HEADLINE_MUSC
    P = ddpca.headline_problem(gl=3, **ddpca.GENERAL_FEATURES)
    P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    Pu = ddpca.headline_problem(gl=3, band=1, rot=0).ESTABLISH()
    G, Gu = P.grid(0), Pu.grid(0)
    L = G.maxiLeve
    assert L == 4 and G.hangRows().shape[0] > 0  # gl 3 + the band level, hanging nodes past it
    # the rotated support nodes change the transfer blocks below the band level (a new node above
    # the bottom face takes w R_par from its rotated parents; same positions, same sparsity)
    assert abs(G.realProl(L - 2) - Gu.realProl(L - 2)).max() > 1e-3
    mc = ddpca.MCONTACT(P, **H)
    k = 8
    assert mc.CONTACT_ANALYSIS(k, check=False) == k
    subs, ifaces = _oracle_problem_no_coarse(P, oracle)
    coarse = dict(globCoup_1=P.csr("globCoup_1"), globForc_1=P.array("globForc_1"), baseReco=P.array("baseReco"),
                  globTran_1=[[P.csr("globTran_1", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
                  globTran_D_1=[P.csr("globTran_D_1", tv) for tv in range(P.nsub)],
                  accuProl=[P.csr("accuProl", tv) for tv in range(P.nsub)])
    res = oracle.admm(subs, ifaces, maxit=k, check=False, coarse=coarse)
    ok, worst = _rows_close(mc.monitor(), res["rows"], k=k, rtol=1e-7)
    print(f"general mesh ({opts}): last PCG iterations {list(mc.get('pcg_iters'))}, worst resuMoni rel {worst:.2e}")
    assert ok, worst
    for tv in range(P.nsub):
        u, ur = mc.get("resuDisp", tv), res["u"][tv]
        assert len(u) == len(ur) == 3 * len(P.grid(tv).nodeCoor), tv
        assert np.linalg.norm(u - ur) <= 1e-7 * np.linalg.norm(ur), tv
    for ts in range(P.nint):
        g, gr = mc.get("inpoGamm", ts), res["gamma"][ts]
        assert np.linalg.norm(g - gr) <= 1e-7 * max(np.linalg.norm(gr), 1e-300), ts
