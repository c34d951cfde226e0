"""Idle time between consecutive kernels of the ADMM window of a rocprofv3 kernel trace: the total,
its histogram, and the largest gaps with the kernels either side (what the host round trips cost).
Usage: python profiles/kernel_gaps.py <trace .db | kernel_trace.csv>"""
import collections
import re
import sqlite3
import sys

import numpy as np


def rows_of(path):
    if path.endswith(".csv"):
        import csv
        out = []
        with open(path) as f:
            for r in csv.DictReader(f):
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                out.append((r["Kernel_Name"], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), e - s, s))
        return sorted(out, key=lambda r: r[3])
    c = sqlite3.connect(path)
    return c.execute("select name, grid_x, duration, start from kernels order by start").fetchall()


def short(n):
    m = re.search(r"(k_\w+)(<[^()]*>)?\(", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


rows = rows_of(sys.argv[1])
inits = [s for n, gx, d, s in rows if "k_pcg_init" in n]
t0 = inits[1]
nit = len(inits) - 1
sel = [r for r in rows if r[3] >= t0]
gaps = []
end = sel[0][3] + sel[0][2]
for i in range(1, len(sel)):
    n, gx, d, s = sel[i]
    gaps.append((s - end, short(sel[i - 1][0]), short(n)))
    end = max(end, s + d)
g = np.array([x[0] for x in gaps], dtype=float)
print(f"{nit} ADMM iterations, {len(sel)} kernels; idle {g[g > 0].sum() / 1e6 / nit:.2f} ms/it")
for lo, hi in [(0, 2e3), (2e3, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e9)]:
    m = (g >= lo) & (g < hi)
    print(f"  gaps {lo / 1e3:6.0f}-{hi / 1e3:6.0f} us: {m.sum() / nit:7.1f}/it  {g[m].sum() / 1e6 / nit:6.3f} ms/it")
pairs = collections.defaultdict(float)
cnt = collections.Counter()
for x in gaps:
    if x[0] >= 5e3:
        pairs[(x[1], x[2])] += x[0]
        cnt[(x[1], x[2])] += 1
print("gaps >= 5 us by (before -> after):")
for k, v in sorted(pairs.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {v / 1e6 / nit:6.3f} ms/it  {cnt[k] / nit:5.1f}/it  {k[0]} -> {k[1]}")
