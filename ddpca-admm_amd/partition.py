"""Subdomain -> rank assignment for one-process-per-GPU runs.

The reference runs every subdomain in one OpenMP process (MCONTACT.h:2511).  Here each rank
(GPU) owns a set of subdomains; ranks are balanced by fine-level dofs with the LPT rule
(largest first onto the least-loaded rank), keeping a worm/wheel contact pair on one rank when
the pair count divides evenly (no exchange for that interface).
"""
from __future__ import annotations

import heapq
from typing import Sequence


def lpt_owner(dofs: Sequence[int], nranks: int) -> list[int]:
    """Longest-processing-time-first packing; ties broken by subdomain index (deterministic)."""
    if nranks < 1:
        raise ValueError("nranks must be >= 1")
    owner = [0] * len(dofs)
    heap = [(0, r) for r in range(nranks)]
    heapq.heapify(heap)
    for tv in sorted(range(len(dofs)), key=lambda i: (-dofs[i], i)):
        load, r = heapq.heappop(heap)
        owner[tv] = r
        heapq.heappush(heap, (load + dofs[tv], r))
    return owner


def block_owner(nsub: int, nranks: int) -> list[int]:
    """Contiguous blocks of subdomains per rank (keeps neighbouring subdomains together)."""
    if nranks < 1:
        raise ValueError("nranks must be >= 1")
    return [min(nranks - 1, tv * nranks // nsub) for tv in range(nsub)]


def owner_for(sizes: Sequence[int], nranks: int) -> list[int]:
    """The bench's and the tests' layout rule: contiguous blocks (block_owner, which keeps DEHW's
    worm/wheel contact pairs on one rank) when every subdomain has the same size, LPT packing by
    size (lpt_owner) when they differ -- DEHW's 52 subdomains of different sizes (DEHW.h:2238-2258)."""
    if len(set(int(s) for s in sizes)) <= 1:
        return block_owner(len(sizes), nranks)
    return lpt_owner(sizes, nranks)
