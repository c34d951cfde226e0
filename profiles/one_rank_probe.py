"""One rank of an N-rank bench layout, alone on one GPU: the headline problem is
established in full, rank r's handle of the N-rank layout (bench.py's block owners and option set)
is connected to the timing transport mcontact_gpu_comm_loopback -- every gamma half it sends comes
back to itself, the all-reduces keep its own values -- and its ADMM iterations are timed as bench.py
times them.  What is measured is one rank's whole share of the iteration (its subdomains' PCG
solves with the coarse-space correction, its interface sides, the mass solves, MONITOR) without
the RCCL traffic; the numbers themselves are not the N-rank answer.  A rank whose subdomains are
all worms never sees the loaded wheels here: its right-hand sides stay zero and its PCG solves exit
at once, so the wheel ranks (odd ranks at N = 8) are the ones that time the solves -- in the real
run a worm's PCG takes the same iteration count as a wheel's (cpu_baseline: 15 and 15).

    python profiles/one_rank_probe.py OUT.json [--layouts 8:0,8:1,4:0,2:0] [--steps 10] [--warmup 2] [--precond-fp32 P]

(world:rank pairs; bench.py's N-rank run is as slow as its slowest rank plus its RCCL traffic.)
"""
import argparse
import importlib
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")
part = importlib.import_module("ddpca-admm_amd.partition")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--layouts", default="8:0,8:1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precond-fp32", type=int, default=None, help="override the option set's precond_fp32")
    ap.add_argument("--nu", type=int, default=None, help="override the option set's sweeps per level")
    ap.add_argument("--smoother", type=int, default=None, help="override the option set's smoother")
    ap.add_argument("--options", choices=["auto", "headline", "small"], default="auto",
                    help="the option set: bench.py's choice by subdomains per rank, or force one")
    a = ap.parse_args()
    import torch
    t0 = time.perf_counter()
    P = D.headline_problem()
    nsub = P.nsub
    P.set_coarse(D.HEADLINE_MUSC["muscSett"], [D.HEADLINE_MUSC["doleMcsc"]] * nsub)
    P.ESTABLISH()
    print(f"[probe] setup {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    rows = []
    for lay in a.layouts.split(","):
        world, r = (int(x) for x in lay.split(":"))
        owner = part.block_owner(nsub, world)
        H = D.headline_options(max(list(owner).count(q) for q in range(world))) if a.options == "auto" else \
            dict(D.HEADLINE_OPTIONS if a.options == "headline" else D.HEADLINE_OPTIONS_SMALL)
        if a.precond_fp32 is not None:
            H["precond_fp32"] = a.precond_fp32
        if a.nu is not None:
            H["nu"] = a.nu
        if a.smoother is not None:
            H["smoother"] = a.smoother
        mc = D.MCONTACT(P, device=0, rank=r, nranks=world, owner=owner, **H)
        mc.comm_loopback()
        mc.CONTACT_ANALYSIS(a.warmup, check=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = mc.CONTACT_ANALYSIS(a.steps, check=False)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        tm = mc.timing()
        owned = [tv for tv in range(nsub) if owner[tv] == r]
        row = {"world": world, "rank": r, "subdomains": owned,
               "dof": int(sum(int(P.array("freeCount", tv)[-1]) for tv in owned)),
               "options": H, "steps": n, "ms_per_iter": 1e3 * el / n,
               "solve_ms_per_iter": tm["solve_ms"] / n, "iface_ms_per_iter": tm["iface_ms"] / n,
               "pcg_iters_per_solve": tm["pcg_iterations"] / max(n * len(owned), 1),
               "mass_cg_iters_per_iter": int(mc.get("mass_iters")[0]) / n}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del mc
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
