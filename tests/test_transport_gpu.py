"""The exchanges of a multi-rank run (SURVEY §8 e) on the one GPU of a test box.

* RCCL itself: a ONE-rank communicator (mcontact_gpu_unique_id -> comm_init) carries the grouped
  send / receive of the gamma halves (to itself) and the all-reduce, element for element
  (mcontact_gpu_comm_check), and an ADMM run whose MONITOR and coarse right-hand-side all-reduces go
  through it is bit-identical to the run without a communicator.  Two ranks cannot share one GPU
  through RCCL ("Duplicate GPU detected"), so this is as far as the wire goes on one card.
* The in-process transport (mcontact_gpu_comm_local) that carries every multi-rank device test
  matches grouped sends and receives per peer in issue order, as RCCL does (an ordering bug fails
  there as it would on the wire): its exchange and all-reduce on 2, 4 and 8 ranks, then the
  headline chain's N = 8 layout -- one subdomain per rank, every contact and glued link across
  ranks -- against a single-rank run of the same options.

The reference shares gamma, aux and lambda in memory between its OpenMP subdomain threads
(MCONTACT.h:2511-2537, 2629-2704) and sums the MONITOR norms in one process (2725-2845)."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SMALL = ("dehw", 2, 2, 2, 1, 2, 0.3)  # 4 subdomains, 3 levels, mu = 0.3


def _run_threads(fns, timeout=300):
    out, err = [None] * len(fns), [None] * len(fns)

    def run(i):
        try:
            out[i] = fns[i]()
        except Exception as e:  # noqa: BLE001 -- reported below
            err[i] = e

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=timeout)
    assert not any(t.is_alive() for t in th), "a rank hung"
    assert all(e is None for e in err), err
    return out


def test_rccl_one_rank_comm_check(ddpca, gpu):
    P = ddpca.Problem(*SMALL).ESTABLISH()
    mc = ddpca.MCONTACT(P)
    mc.comm_init(ddpca.MCONTACT.unique_id())
    mc.comm_check(1 << 16)
    mc.comm_check(3)


@pytest.mark.parametrize("musc", [0, 2])
def test_rccl_one_rank_run_is_bit_identical(ddpca, gpu, musc):
    """The per-iteration all-reduces through a one-rank RCCL communicator on the solve stream (ncclAllReduce
    of the MONITOR norms and, with the coarse space, of its right-hand side) leave every bit as it was."""
    out = {}
    for comm in (False, True):
        P = ddpca.Problem(*SMALL)
        if musc:
            P.set_coarse(musc, [1] * P.nsub)
        P.ESTABLISH()
        mc = ddpca.MCONTACT(P)
        if comm:
            mc.comm_init(ddpca.MCONTACT.unique_id())
        assert mc.CONTACT_ANALYSIS(12, check=False) == 12
        out[comm] = (mc.monitor().copy(), [mc.get("resuDisp", tv).copy() for tv in range(P.nsub)])
        del mc
    assert np.array_equal(out[False][0], out[True][0])
    for a, b in zip(out[False][1], out[True][1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_local_transport_comm_check(ddpca, gpu, nranks):
    P = ddpca.headline_problem(gl=1).ESTABLISH()  # 8 subdomains, tiny
    owner = [tv % nranks for tv in range(P.nsub)]
    ranks = [ddpca.MCONTACT(P, rank=r, nranks=nranks, owner=owner) for r in range(nranks)]
    ddpca.MCONTACT.comm_local(ranks)
    _run_threads([lambda m=m: m.comm_check(5000) for m in ranks])


def test_headline_chain_eight_ranks_one_subdomain_each(ddpca, gpu):
    """BASELINE config 5's N = 8 layout on the reduced chain (headline_problem(gl=3), interface-
    eliminated coarse space): rank r owns subdomain r (what bench.py --gpus 8 does), builds only its
    own operators (ESTABLISH(owner, rank): rank-local coarse rows, summed by the setup all-reduce),
    runs bench.py's option set for one subdomain per rank (headline_options(1)), exchanges the gamma
    halves of all 10 interfaces -- every contact and every glued link crosses ranks -- and
    all-reduces the MONITOR norms and the coarse right-hand side.  Against one rank holding all
    eight with the same options (exact-solve level pinned: its automatic choice depends on the
    batch): the same iterations to convergence, resuMoni rows 1e-7, displacements
    1e-8, contact tractions 1e-7 of the largest."""
    M = ddpca.HEADLINE_MUSC
    H = dict(ddpca.headline_options(1), coarse_level=1)

    def problem(owner=None, rank=0):
        P = ddpca.headline_problem(gl=3)
        P.set_coarse(M["muscSett"], [M["doleMcsc"]] * P.nsub)
        return P.ESTABLISH(owner, rank) if owner is not None else P.ESTABLISH()

    ref = ddpca.MCONTACT(problem(), **H)
    n_ref = ref.CONTACT_ANALYSIS(200)
    rows_ref = ref.monitor()
    owner = list(range(8))
    probs = [problem(owner, r) for r in range(8)]
    ranks = [ddpca.MCONTACT(probs[r], rank=r, nranks=8, owner=owner, **H) for r in range(8)]
    ddpca.MCONTACT.comm_local(ranks)
    n = _run_threads([lambda m=m: m.CONTACT_ANALYSIS(200) for m in ranks], timeout=600)
    assert n == [n_ref] * 8, (n, n_ref)
    scale = np.abs(rows_ref).max(axis=0, keepdims=True)
    worst = 0.0
    for r in range(8):
        rows = ranks[r].monitor()
        assert rows.shape == rows_ref.shape
        rel = np.abs(rows - rows_ref) / (np.abs(rows_ref) + 1e-12 * scale + 1e-300)
        worst = max(worst, float(rel.max()))
        u, ur = ranks[r].get("resuDisp", r), ref.get("resuDisp", r)
        assert np.linalg.norm(u - ur) <= 1e-8 * max(np.linalg.norm(ur), 1e-300), r
    for ts in range(probs[0].nint):
        body = [int(b) for b in probs[0].array("iface_body", ts)]
        g, gr = ranks[body[0]].get("inpoGamm", ts), ref.get("inpoGamm", ts)
        assert np.abs(g - gr).max() <= 1e-7 * np.abs(gr).max(), ts
    print(f"8 ranks x 1 subdomain: {n_ref} ADMM iterations, worst resuMoni rel {worst:.2e}")
    assert worst <= 1e-7, worst
