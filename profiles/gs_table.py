"""Per-launch table of the multicolour fine-level sweeps (k_gs<0|1|2>): the library's byte model,
rocprof durations, PMC HBM bytes, achieved GB/s and the fraction of 8 TB/s.

    python profiles/gs_table.py DIR

DIR holds gs_model.json (profiles/gs_probe.py) and the outputs of three runs of gs_probe.py:
trace/ (`rocprofv3 --kernel-trace --stats`), pmc_fetch/ and pmc_write/ (`rocprofv3 --pmc
FETCH_SIZE` / `--pmc WRITE_SIZE`, `--kernel-include-regex k_gs`).  The launches of every V-cycle
come in the order forward colours 0..K-1, residual, backward colours K-1..0; per slot the launches
in which every subdomain runs (>= 0.9 of the slot's largest PMC value; for durations the
launches of the same V-cycles) give the median.  HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE, in KiB
(the gfx950 correction of profiles/make_traffic.py).  Writes DIR/gs_table.txt and gs_table.json.
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys
from pathlib import Path

PEAK = 8000.0


def phase(name: str):
    m = re.search(r"k_gs<(\d),", name)
    return int(m.group(1)) if m else None


def load_counter(d: Path, counter: str) -> list[tuple[int, int, float]]:
    f = next(d.rglob("*counter_collection.csv"))
    out = []
    for r in csv.DictReader(open(f)):
        ph = phase(r["Kernel_Name"])
        if ph is None or r["Counter_Name"] != counter:
            continue
        out.append((int(r["Dispatch_Id"]), ph, float(r["Counter_Value"])))
    out.sort()
    return out


def load_trace(d: Path) -> list[tuple[int, int, float]]:
    f = next(d.rglob("*kernel_trace.csv"))
    out = []
    for r in csv.DictReader(open(f)):
        ph = phase(r["Kernel_Name"])
        if ph is None:
            continue
        out.append((int(r["Dispatch_Id"]), ph, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    out.sort()
    return out


def slots(seq: list[tuple[int, int, float]], K: int) -> list[list[float]]:
    """Split the launch sequence into V-cycles (K forward, 1 residual, K backward) -> per slot values."""
    pattern = [0] * K + [1] + [2] * K
    per = [[] for _ in pattern]
    i = 0
    while i + len(pattern) <= len(seq):
        if [p for _, p, _ in seq[i:i + len(pattern)]] == pattern:
            for s in range(len(pattern)):
                per[s].append(seq[i + s][2])
            i += len(pattern)
        else:
            i += 1
    return per


def main():
    d = Path(sys.argv[1])
    model = json.loads((d / "gs_model.json").read_text())
    K, mb, names = model["colours"], model["launch_bytes"], model["order"]
    fetch = slots(load_counter(d / "pmc_fetch", "FETCH_SIZE"), K)
    write = slots(load_counter(d / "pmc_write", "WRITE_SIZE"), K)
    dur = slots(load_trace(d / "trace"), K)
    rows = []
    for s in range(2 * K + 1):
        def full(v):
            top = max(v)
            return statistics.median([x for x in v if x >= 0.9 * top])
        hbm = (2.0 * full(fetch[s]) + full(write[s])) * 1024.0 if fetch[s] and write[s] else None
        t = statistics.median(sorted(dur[s])[len(dur[s]) // 4:]) if dur[s] else None  # drop the short tail launches
        rows.append({"launch": names[s], "model_bytes": mb[s], "pmc_bytes": hbm, "pmc_over_model": hbm / mb[s] if hbm else None,
                     "ms": t * 1e3 if t else None, "achieved_gbs": mb[s] / t / 1e9 if t else None,
                     "frac_of_8tbs": mb[s] / t / 1e9 / PEAK if t else None, "vcycles": len(dur[s])})
    fam = {}
    for key, sel in (("forward", range(K)), ("residual", [K]), ("backward", range(K + 1, 2 * K + 1)), ("all", range(2 * K + 1))):
        m = sum(rows[s]["model_bytes"] for s in sel)
        h = sum(rows[s]["pmc_bytes"] or 0.0 for s in sel)
        t = sum(rows[s]["ms"] or 0.0 for s in sel) * 1e-3
        fam[key] = {"model_bytes": m, "pmc_bytes": h, "pmc_over_model": h / m, "ms": t * 1e3,
                    "achieved_gbs": m / t / 1e9, "frac_of_8tbs": m / t / 1e9 / PEAK}
    res = {"colours": K, "launches": rows, "families": fam, "source": str(d)}
    (d / "gs_table.json").write_text(json.dumps(res, indent=1) + "\n")
    lines = [f"{'launch':8s} {'model MB':>9s} {'PMC MB':>9s} {'PMC/model':>9s} {'ms':>8s} {'GB/s':>7s} {'of 8TB/s':>8s}"]
    for r in rows:
        lines.append(f"{r['launch']:8s} {r['model_bytes'] / 1e6:9.1f} {(r['pmc_bytes'] or 0) / 1e6:9.1f} {r['pmc_over_model'] or 0:9.3f} "
                     f"{r['ms'] or 0:8.4f} {r['achieved_gbs'] or 0:7.0f} {r['frac_of_8tbs'] or 0:8.3f}")
    for k, f in fam.items():
        lines.append(f"{k:8s} {f['model_bytes'] / 1e6:9.1f} {f['pmc_bytes'] / 1e6:9.1f} {f['pmc_over_model']:9.3f} "
                     f"{f['ms']:8.4f} {f['achieved_gbs']:7.0f} {f['frac_of_8tbs']:8.3f}")
    (d / "gs_table.txt").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
