"""HBM bytes per launch of the roofline kernel from rocprofv3 PMC passes -> profiles/traffic.json.

    python profiles/make_traffic.py FETCH_CSV WRITE_CSV --smoother 1 --nu 1 --precond-fp32 1 [...]

FETCH_CSV / WRITE_CSV are the run_counter_collection.csv files of two separate passes
(`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`, each `--kernel-include-regex "k_sell<3"`)
over `bench.py --steps 1 --warmup 1`.  Only the fine-level launches (largest grid) in which every
subdomain iterates are used (the first ADMM iteration's worm subdomains have a zero right-hand
side and skip the kernel; those launches show about half the bytes and are dropped).

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section, checked here with profiles/calib_stream.hip
(`hipcc --offload-arch=gfx950 -O3`, run under `rocprofv3 --pmc FETCH_SIZE`; r01_pmc_calibration.txt):
1 GiB streamed with 8-B and 16-B lanes reads back FETCH_SIZE = 524,29x KB): FETCH_SIZE counts
half of the bytes of coalesced streaming reads on gfx950 -> x2; WRITE_SIZE is taken as bytes.
FETCH_SIZE counts L2 misses served by the Infinity Cache too, so it bounds HBM reads from above.
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
from pathlib import Path


def per_launch(path: str, counter: str) -> list[tuple[int, float]]:
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and "k_sell<3," in r["Kernel_Name"]:
            out.append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return out


def full_launches(rows: list[tuple[int, float]]) -> list[float]:
    g = max(n for n, _ in rows)
    vals = [v for n, v in rows if n == g]
    top = max(vals)
    return [v for v in vals if v >= 0.9 * top]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    # defaults: bench.py's (the package's HEADLINE_WORKLOAD / HEADLINE_OPTIONS)
    import importlib
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    pkg = importlib.import_module("ddpca-admm_amd")
    W, H = pkg.HEADLINE_WORKLOAD, pkg.HEADLINE_OPTIONS
    for k, d in [("groups", W["groups"]), ("nx", W["nx"]), ("ny", W["ny"]), ("nz", W["nz"]), ("gl", W["gl"]),
                 ("smoother", H["smoother"]), ("nu", H["nu"]), ("precond-fp32", H["precond_fp32"]),
                 ("table-mode", H["table_mode"])]:
        ap.add_argument(f"--{k}", type=int, default=d)
    ap.add_argument("--value-layout", default="fp64-pairs, col16")
    ap.add_argument("--mesh", default="headline", help="general: bench.py --mesh general's line (profiles/traffic_general.json)")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parent / "traffic.json"))
    a = ap.parse_args()
    fetch = full_launches(per_launch(a.fetch_csv, "FETCH_SIZE"))
    write = full_launches(per_launch(a.write_csv, "WRITE_SIZE"))
    fkb, wkb = statistics.median(fetch), statistics.median(write)
    res = {
        "kernel": "k_sell<kPcg> fine level",
        "config": dict(groups=a.groups, nx=a.nx, ny=a.ny, nz=a.nz, gl=a.gl, smoother=a.smoother, nu=a.nu,
                       precond_fp32=a.precond_fp32, table_mode=a.table_mode, value_layout=a.value_layout,
                       **({} if a.mesh == "headline" else {"mesh": a.mesh})),
        "fetch_size_kb_median": fkb,
        "write_size_kb_median": wkb,
        "launches_used": [len(fetch), len(write)],
        "fetch_correction": 2.0,
        "hbm_bytes_per_launch": 2.0 * fkb * 1024.0 + wkb * 1024.0,
    }
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
