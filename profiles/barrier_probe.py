"""Persistent grid barrier vs graph kernel boundary on one MI355X (ddpca_probe_grid_barrier): the
measurement behind DESIGN §8's persistent below-fine V-cycle decision.  Per pass, n doubles are
rewritten from what other workgroups (other XCDs) wrote in the previous pass -- the data flow of a
V-cycle level sweep -- at the below-fine level sizes of the headline batch and at 64 / 256
workgroups (one per CU at most), and (r05) with the persistent workgroups pinned to one XCD --
8 x blocks launched, only id % 8 == 0 working, 8 / 32 of them -- so the barrier's arrivals and
polls stay in one L2 (the agent-scope release / acquire stay: co-location gives no visibility).

    python profiles/barrier_probe.py OUT.json
"""
import importlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")


def main():
    rows = []
    for n in (4096, 32768, 262144, 1228800):  # ~ levels L-4 .. L-1 of the 8-subdomain batch (dof)
        for blocks, pin in ((64, False), (256, False), (8, True), (32, True)):
            r = D.probe_grid_barrier(n, phases=64, blocks=blocks, pin=pin)
            r.update(n=n, blocks=blocks, pin=pin, phases=64)
            rows.append(r)
            print(json.dumps(r), flush=True)
            if r["timed_out"]:
                raise SystemExit("a persistent workgroup timed out: stop")
    with open(sys.argv[1], "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
