"""HBM bytes per launch of the V-cycle's fine-level kernels from rocprofv3 PMC passes.

    python profiles/pmc_kernels.py FETCH_CSV WRITE_CSV [--out FILE]

FETCH_CSV / WRITE_CSV: run_counter_collection.csv of two separate passes
(`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`, `--kernel-include-regex
"k_prolong|k_restrict|k_sell<1|k_sell<2"`) over `bench.py --steps 1 --warmup 1` at the default
bench configuration (profiles/round_profile.sh).  Per kernel and grid size: the median over the
launches in which every subdomain runs (>= 0.9 of the largest value), FETCH_SIZE x 2 + WRITE_SIZE
(the gfx950 correction of make_traffic.py), next to the algorithmic bytes of the fine-level
launches at that configuration:

  nodes  n_f = 3,278,600 real fine nodes (8 x 97 x 65 x 65), n_c = 426,888 on level L-1,
  blocks nnzb = 86,119,688 stored 3x3 blocks on the fine level (from the roofline kernel's
         6,766,288,912 B = 74 nnzb + 120 n_f),
  k_sell<1> (residual, block-exponent fp16)  22 nnzb + 72 n_f   (20 B values + 2 B offset per
            block; x gathered once, b read, r written)
  k_sell<2> (Jacobi sweep, fp16, fp32 3x3 inverse)  22 nnzb + 108 n_f
  k_prolong (lattice)  53 n_f + 24 n_c   (4-B code, mask, x_f read + written, e_c read once)
  k_prolong<true> (explicit lists)  the same + 4 B per streamed parent-index slot
  k_restrict (lattice, fused first sweep, fp32 inverse)  24 n_f + 93 n_c
  k_restrict (explicit)  the same + 12 B per (coarse node, child) slot
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re
import statistics
from pathlib import Path

N_F, N_C, NNZB = 3_278_600, 426_888, 86_119_688
ALGO = {  # (kernel prefix, grid) -> algorithmic bytes per launch at the bench configuration
    ("k_sell<1,", 3278848): 22 * NNZB + 72 * N_F,
    ("k_sell<2,", 3278848): 22 * NNZB + 108 * N_F,
    # precond_fp32 = 4 (round 6): the fine prolongation into the colour sweeps' fp32 iterate copy
    # (4-B code, mask, 16 B read + written per fine node), the restriction from their fp32 residual
    # (16 B per fine node): checked before the fp64 forms below (prefix match)
    ("k_prolong_lat_x4", 3278848): 37 * N_F + 24 * N_C,
    ("k_restrict_lat<true, true, false, float, HIP_vector_type", 427008): 16 * N_F + 93 * N_C,
    ("k_prolong_lat", 3278848): 53 * N_F + 24 * N_C,
    ("k_prolong<true>", 3278848): 53 * N_F + 24 * N_C,
    ("k_restrict_lat", 427008): 24 * N_F + 93 * N_C,
    ("k_restrict<true", 427008): 24 * N_F + 93 * N_C,
}


def rows(path: str, counter: str) -> dict[tuple[str, int], list[float]]:
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+)(<[^()]*>)?\(", r["Kernel_Name"])
        name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
        out[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def full(vals: list[float]) -> float:
    top = max(vals)
    return statistics.median([v for v in vals if v >= 0.9 * top])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch, write = rows(a.fetch_csv, "FETCH_SIZE"), rows(a.write_csv, "WRITE_SIZE")
    res = []
    for key in sorted(set(fetch) & set(write), key=lambda k: -k[1]):
        name, grid = key
        hbm = 2.0 * full(fetch[key]) * 1024.0 + full(write[key]) * 1024.0
        algo = next((v for (p, g), v in ALGO.items() if name.startswith(p) and g == grid), None)
        res.append({"kernel": name, "grid": grid, "launches": len(fetch[key]), "hbm_bytes": hbm,
                    "algorithmic_bytes": algo, "ratio": (hbm / algo) if algo else None})
        print(f"{name:55s} grid={grid:8d} n={len(fetch[key]):4d} hbm={hbm / 1e6:9.1f} MB"
              + (f"  algorithmic={algo / 1e6:9.1f} MB  ratio={hbm / algo:5.2f}" if algo else ""))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
