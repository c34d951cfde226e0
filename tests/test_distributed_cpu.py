"""Multi-rank decomposition of the ADMM loop on CPU (gloo, world_size 2).

The GPU path assigns subdomains to ranks (partition.block_owner), gives each rank the interface
sides of its subdomains, sums the two halves of every gamma (RCCL send/recv of the halves, or a
sum) and all-reduces the MONITOR norms.  This test runs the same decomposition with the CPU
oracle over gloo and requires the rank-split run to reproduce the single-process trajectory to
rounding (1e-12 relative), including the stopping decision."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ARGS = ("dehw", 2, 2, 2, 1, 1, 0.3)
ARGS_COARSE = ("dehw", 2, 2, 2, 1, 2, 0.3)  # 3 levels, coarse space on level 1


def _problem(args=ARGS, coarse=False, owner=None, rank=0):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    D = importlib.import_module("ddpca-admm_amd")
    from test_mcontact_gpu import _oracle_coarse, _oracle_problem
    P = D.Problem(*args)
    if coarse:
        P.set_coarse(2, [1] * P.nsub)
    P.ESTABLISH()
    if not coarse:
        return P, _oracle_problem(P), None
    if owner is None:
        return P, _oracle_problem(P), _oracle_coarse(P)
    # this rank's own share of the coarse operators, built rank-locally as on the GPU path
    Q = D.Problem(*args)
    Q.set_coarse(2, [1] * Q.nsub)
    Q.ESTABLISH(owner, rank)
    body = [tuple(int(b) for b in Q.array("iface_body", ts)) for ts in range(Q.nint)]
    loc = dict(globCoup_1=Q.csr("globCoup_1"), globForc_1=Q.array("globForc_1"), baseReco=Q.array("baseReco"),
               globTran_1=[[Q.csr("globTran_1", 2 * ts + s) if owner[body[ts][s]] == rank else None
                            for s in range(2)] for ts in range(Q.nint)],
               globTran_D_1=[Q.csr("globTran_D_1", tv) if owner[tv] == rank else None for tv in range(Q.nsub)],
               accuProl=[Q.csr("accuProl", tv) if owner[tv] == rank else None for tv in range(Q.nsub)])
    return P, _oracle_problem(P), loc


def _worker(rank, world, port, out, coarse=False, owner_override=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    part = importlib.import_module("ddpca-admm_amd.partition")
    owner = owner_override or part.block_owner(4, world)
    P, (subs, ifaces), cs = _problem(ARGS_COARSE if coarse else ARGS, coarse, owner, rank)

    def allreduce(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        dist.all_reduce(t)
        return t.numpy()

    res = O.admm(subs, ifaces, maxit=60, check=True, rank=rank, owner=owner, allreduce=allreduce, coarse=cs)
    out[rank] = (res["rows"], [res["u"][tv] for tv in range(len(subs)) if owner[tv] == rank], res["iters"])
    dist.destroy_process_group()


@pytest.mark.parametrize("coarse,owner", [(False, None), (True, None), (True, [0, 1, 0, 1])])
def test_two_rank_admm_matches_single_rank(oracle, coarse, owner):
    """coarse: the interface-eliminated coarse space with rank-local operators (each rank's
    ESTABLISH(owner, rank) share), the dense coarse matrix and the per-iteration right-hand side
    summed across ranks -- the device path's decomposition; owner [0,1,0,1] puts every
    interface across the two ranks."""
    P, (subs, ifaces), cs = _problem(ARGS_COARSE if coarse else ARGS, coarse)
    ref = oracle.admm(subs, ifaces, maxit=60, check=True, coarse=cs)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, out, coarse, owner), nprocs=2, join=True)
    part = importlib.import_module("ddpca-admm_amd.partition")
    owner = owner or part.block_owner(len(subs), 2)
    for rank in range(2):
        rows, us, iters = out[rank]
        assert iters == ref["iters"]
        scale = np.abs(ref["rows"]).max(axis=0, keepdims=True)
        assert np.all(np.abs(rows - ref["rows"]) <= 1e-12 * np.abs(ref["rows"]) + 1e-14 * scale)
        mine = [tv for tv in range(len(subs)) if owner[tv] == rank]
        for u, tv in zip(us, mine):
            assert np.linalg.norm(u - ref["u"][tv]) <= 1e-12 * np.linalg.norm(ref["u"][tv])
