"""roofline_check.py on a CSV kernel trace (rocprofv3 --output-format csv): the sampled launches
(the first fine k_sell<kPcg> after each k_pcg_init) vs the bench's HIP-event average.

    python profiles/roofline_check_csv.py KERNEL_TRACE_CSV BENCH_JSON
"""
import csv
import json
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gmax = max(int(r["Grid_Size_X"]) for r in rows if "k_sell<3," in r["Kernel_Name"])
armed, durs = False, []
for r in rows:
    n = r["Kernel_Name"]
    if "k_pcg_init" in n:
        armed = True
    elif armed and "k_sell<3," in n and int(r["Grid_Size_X"]) == gmax:
        durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        armed = False
b = None
for line in open(sys.argv[2]):
    if line.startswith("{"):
        b = json.loads(line)
ev = b["roofline"]["avg_launch_ms"]
# the bench samples the timed steps' solves: the last `samples` of them
samp = durs[-b["roofline"]["samples"]:]
print(json.dumps({"rocprof_sampled_ms": [round(d, 4) for d in samp], "rocprof_mean_ms": statistics.mean(samp),
                  "hip_event_mean_ms": ev, "ratio": statistics.mean(samp) / ev,
                  "algorithmic_bytes_per_launch": b["roofline"]["algorithmic_bytes_per_launch"],
                  "rocprof_TBs": b["roofline"]["algorithmic_bytes_per_launch"] / statistics.mean(samp) / 1e9}, indent=1))
