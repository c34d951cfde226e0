"""Per-kernel summary (calls, total, average) of a rocprofv3 --kernel-trace database
(rocpd sqlite, rocprofv3 >= 1.0 default output), as the --stats CSV would give it.

    python profiles/kernel_stats.py gpurun_out/prof/run_results.db [--csv out.csv]
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    for r in rows[:a.top]:
        print(f"{r[2] / 1e6:9.2f} ms {r[1]:6d} {r[3] / 1e3:9.1f} us {100 * r[2] / tot:5.1f}%  {r[0][:120]}")
    print(f"total kernel time {tot / 1e6:.2f} ms")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_ALL)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], f"{r[3]:.6f}", f"{100 * r[2] / tot:.2f}", r[4], r[5]])


if __name__ == "__main__":
    main()
