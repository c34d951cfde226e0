"""Per-kernel time per ADMM iteration from a rocprofv3 CSV kernel trace of bench.py (one stream):
the window from the second k_pcg_init to the end, grouped by kernel name and grid.
    python profiles/breakdown_csv.py RUN_KERNEL_TRACE_CSV [TOP]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
inits = [i for i, r in enumerate(rows) if "k_pcg_init" in r["Kernel_Name"]]
sel = rows[inits[1]:]
nit = len(inits) - 1
t0 = int(sel[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in sel)
g = collections.defaultdict(list)
for r in sel:
    m = re.search(r"(k_\w+|__amd\w+)(<[^()]*>)?", r["Kernel_Name"])
    key = ((m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:50], int(r["Grid_Size_X"]))
    g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in g.values())
print(f"window {(t1 - t0) / 1e6 / nit:.2f} ms per ADMM iteration; kernel sum {tot / 1e6 / nit:.2f} ms; "
      f"{sum(len(v) for v in g.values()) / nit:.0f} launches")
for (n, gx), ds in sorted(g.items(), key=lambda kv: -sum(kv[1]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{sum(ds) / 1e6 / nit:7.2f} ms/it n/it={len(ds) / nit:6.1f} grid={gx:8d} avg={sum(ds) / len(ds) / 1e3:7.1f}us {n}")
