"""The multi-rank device path on one GPU: two mcontact_gpu handles (ranks 0 and 1 of 2) in one
process, connected by the in-process test transport (mcontact_gpu_comm_local) instead of RCCL.

Everything but the wire is the production code: rank-local ESTABLISH(owner, rank), each rank's
batch of owned subdomains, the gamma offsets and the halves exchanged for cross-rank interfaces,
the MONITOR all-reduce, and with a coarse space the rank-local coarse operators, the setup
all-reduce of the dense coarse matrix (coarse_invert after comm init) and the per-iteration
coarse right-hand side all-reduce.  The two-rank run must reproduce the single-rank run: same
iteration count and stopping decision, resuMoni rows and displacements to the PCG accuracy (each
rank's batch holds different members, so the V-cycle's exact-solve level and the rounding of the
batched launches differ; 1e-8 is far below any bookkeeping error, which would be O(1)).  The CPU
counterpart over gloo is tests/test_distributed_cpu.py."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ARGS = ("dehw", 2, 2, 2, 1, 2, 0.3)  # 4 subdomains (2 worm/wheel groups), 3 levels, mu = 0.3


def _problem(ddpca, musc, owner=None, rank=0):
    P = ddpca.Problem(*ARGS)
    if musc:
        P.set_coarse(musc, [1] * P.nsub)
    return P.ESTABLISH(owner, rank) if owner is not None else P.ESTABLISH()


CASES = [(0, False), (2, False), (1, False), (2, True), (1, True)]


@pytest.mark.parametrize("musc,double_m", CASES, ids=[f"musc{m}{'-double_m' if d else ''}" for m, d in CASES])
@pytest.mark.parametrize("owner", [[0, 1, 0, 1], [0, 0, 1, 1]])
def test_two_ranks_in_one_process_match_single_rank(ddpca, gpu, owner, musc, double_m, monkeypatch):
    """owner [0,1,0,1] puts every worm/wheel contact across the ranks (gamma halves exchanged),
    [0,0,1,1] the glued chain links; musc 2 / 1: interface-eliminated / LATIN coarse space built
    rank-locally.  double_m: the coarse problem forced onto DOUBLE_M_1 / DOUBLE_M's MGPIS
    (DDPCA_COARSE_MG_MIN = 1; MCONTACT.h:1857-1866, 1229-1237) -- the rank-local build then gathers
    the whole coarse operator at setup (two all-reduces of (row, col, value) triplets, duplicates
    summed) and every rank builds the same hierarchy.

    The V-cycle's exact-solve level is pinned (its automatic choice depends on the members per
    rank), so the ranks do the single-rank run's arithmetic: per-subdomain kernels, the MONITOR
    norms and the coarse right-hand side in per-source slots (build_coarse), the coarse operator's
    entries each from one side.  Required: resuMoni rows, displacements and gamma within 1e-12 of the
    single-rank run (measured: identical bits), far inside SURVEY c4's 1e-7."""
    if double_m:
        monkeypatch.setenv("DDPCA_COARSE_MG_MIN", "1")
    maxit = 300
    opts = dict(coarse_level=1)
    ref = ddpca.MCONTACT(_problem(ddpca, musc), **opts)
    n_ref = ref.CONTACT_ANALYSIS(maxit)
    rows_ref = ref.monitor()
    if double_m:
        cs = ref.get("coarse_solve", 0)
        assert cs[1] == 1, cs  # the multigrid coarse solve
    probs = [_problem(ddpca, musc, owner, r) for r in range(2)]
    ranks = [ddpca.MCONTACT(probs[r], rank=r, nranks=2, owner=owner, **opts) for r in range(2)]
    ddpca.MCONTACT.comm_local(ranks)
    out, err = [None, None], [None, None]

    def run(r):
        try:
            out[r] = ranks[r].CONTACT_ANALYSIS(maxit)
        except Exception as e:  # noqa: BLE001 -- reported below
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank hung"
    assert err == [None, None], err
    assert out[0] == out[1] == n_ref, (out, n_ref)
    worst = {"moni": 0.0, "u": 0.0, "gamma": 0.0}
    for r in range(2):
        rows = ranks[r].monitor()
        assert rows.shape == rows_ref.shape
        scale = np.abs(rows_ref).max(axis=0, keepdims=True)
        rel = np.abs(rows - rows_ref) / (np.abs(rows_ref) + 1e-12 * scale + 1e-300)
        worst["moni"] = max(worst["moni"], float(rel.max()))
        for tv in range(4):
            if owner[tv] != r:
                continue
            u, ur = ranks[r].get("resuDisp", tv), ref.get("resuDisp", tv)
            worst["u"] = max(worst["u"], float(np.linalg.norm(u - ur) / np.linalg.norm(ur)))
        for ts in range(probs[r].nint):
            body = [int(b) for b in probs[r].array("iface_body", ts)]
            if r in (owner[body[0]], owner[body[1]]):
                g, gr = ranks[r].get("inpoGamm", ts), ref.get("inpoGamm", ts)
                worst["gamma"] = max(worst["gamma"], float(np.abs(g - gr).max() / np.abs(gr).max()))
    print(f"owner {owner} musc {musc} double_m {double_m}: {n_ref} iterations, worst relative differences {worst}")
    assert worst["moni"] <= 1e-12 and worst["u"] <= 1e-12 and worst["gamma"] <= 1e-12, worst


@pytest.mark.parametrize("musc", [0, 2])
def test_lpt_packed_uneven_subdomains_match_single_rank(ddpca, gpu, musc):
    """DEHW's subdomains differ in size (52 of them, DEHW.h:2238-2258) and SURVEY §8 e1 packs them
    onto the GPUs by LPT.  Twelve subdomains of three sizes (the dehw generator's `uneven` chain:
    group g is 1 + g mod 3 blocks long) packed by partition.owner_for (LPT by node count: uneven
    batches, every rank holding subdomains of different sizes, interfaces crossing ranks in every
    direction) on four in-process ranks, against the single-rank run of the same options: the same
    iteration count on every rank, resuMoni rows, displacements and gamma equal to 1e-12 (the rank
    layout does not enter the arithmetic)."""
    from importlib import import_module
    part = import_module("ddpca-admm_amd.partition")
    args = ("dehw", 6, 2, 2, 1, 2, 0.3, 0, 0, 0, 0, 1)

    def problem(owner=None, rank=0):
        P = ddpca.Problem(*args)
        if musc:
            P.set_coarse(musc, [1] * P.nsub)
        return P.ESTABLISH(owner, rank) if owner is not None else P.ESTABLISH()

    P0 = problem()
    sizes = [len(P0.array("coords", tv)) // 3 for tv in range(P0.nsub)]
    assert len(set(sizes)) == 3, sizes
    nr = 4
    owner = part.owner_for(sizes, nr)
    assert owner == part.lpt_owner(sizes, nr)
    loads = [sum(s for s, o in zip(sizes, owner) if o == r) for r in range(nr)]
    print("sizes", sizes, "owner", owner, "loads", loads)
    maxit = 300
    opts = dict(coarse_level=1)
    ref = ddpca.MCONTACT(P0, **opts)
    n_ref = ref.CONTACT_ANALYSIS(maxit)
    rows_ref = ref.monitor()
    probs = [problem(owner, r) for r in range(nr)]
    ranks = [ddpca.MCONTACT(probs[r], rank=r, nranks=nr, owner=owner, **opts) for r in range(nr)]
    ddpca.MCONTACT.comm_local(ranks)
    out, err = [None] * nr, [None] * nr

    def run(r):
        try:
            out[r] = ranks[r].CONTACT_ANALYSIS(maxit)
        except Exception as e:  # noqa: BLE001 -- reported below
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(nr)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank hung"
    assert err == [None] * nr, err
    assert out == [n_ref] * nr, (out, n_ref)
    worst = {"moni": 0.0, "u": 0.0, "gamma": 0.0}
    for r in range(nr):
        rows = ranks[r].monitor()
        assert rows.shape == rows_ref.shape
        scale = np.abs(rows_ref).max(axis=0, keepdims=True)
        worst["moni"] = max(worst["moni"], float((np.abs(rows - rows_ref) / (np.abs(rows_ref) + 1e-12 * scale + 1e-300)).max()))
        for tv in range(P0.nsub):
            if owner[tv] == r:
                u, ur = ranks[r].get("resuDisp", tv), ref.get("resuDisp", tv)
                worst["u"] = max(worst["u"], float(np.linalg.norm(u - ur) / np.linalg.norm(ur)))
        for ts in range(P0.nint):
            body = [int(b) for b in P0.array("iface_body", ts)]
            if owner[body[0]] == r:
                g, gr = ranks[r].get("inpoGamm", ts), ref.get("inpoGamm", ts)
                worst["gamma"] = max(worst["gamma"], float(np.abs(g - gr).max() / np.abs(gr).max()))
    print(f"musc {musc}: {n_ref} iterations, worst relative differences {worst}")
    assert worst["moni"] <= 1e-12 and worst["u"] <= 1e-12 and worst["gamma"] <= 1e-12, worst
