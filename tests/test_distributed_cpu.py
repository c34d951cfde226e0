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


def _problem():
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    D = importlib.import_module("ddpca-admm_amd")
    from test_mcontact_gpu import _oracle_problem
    P = D.Problem("dehw", 2, 2, 2, 1, 1, 0.3).ESTABLISH()
    return P, _oracle_problem(P)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from oracle import oracle as O
    part = importlib.import_module("ddpca-admm_amd.partition")
    P, (subs, ifaces) = _problem()
    owner = part.block_owner(len(subs), world)

    def allreduce(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        dist.all_reduce(t)
        return t.numpy()

    res = O.admm(subs, ifaces, maxit=60, check=True, rank=rank, owner=owner, allreduce=allreduce)
    out[rank] = (res["rows"], [res["u"][tv] for tv in range(len(subs)) if owner[tv] == rank], res["iters"])
    dist.destroy_process_group()


def test_two_rank_admm_matches_single_rank(oracle):
    P, (subs, ifaces) = _problem()
    ref = oracle.admm(subs, ifaces, maxit=60, check=True)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    part = importlib.import_module("ddpca-admm_amd.partition")
    owner = part.block_owner(len(subs), 2)
    for rank in range(2):
        rows, us, iters = out[rank]
        assert iters == ref["iters"]
        scale = np.abs(ref["rows"]).max(axis=0, keepdims=True)
        assert np.all(np.abs(rows - ref["rows"]) <= 1e-12 * np.abs(ref["rows"]) + 1e-14 * scale)
        mine = [tv for tv in range(len(subs)) if owner[tv] == rank]
        for u, tv in zip(us, mine):
            assert np.linalg.norm(u - ref["u"][tv]) <= 1e-12 * np.linalg.norm(ref["u"][tv])
