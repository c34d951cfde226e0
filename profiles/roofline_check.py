"""Cross-check of bench.py's live roofline timing against rocprof: the durations rocprofv3 recorded
for the sampled launches (the first fine k_sell<kPcg> after each k_pcg_init, i.e. the eager first
PCG iteration of every batched solve) vs the HIP-event average the bench printed in the same run.

    python profiles/roofline_check.py TRACE_DB TRACE_LOG
"""
import json
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, grid_x, duration, start from kernels order by start").fetchall()
    gmax = max(g for n, g, d, s in rows if "k_sell<3," in n)
    durs, armed = [], False
    for n, g, d, s in rows:
        if "k_pcg_init" in n:
            armed = True
        elif armed and "k_sell<3," in n and g == gmax:
            durs.append(d / 1e6)
            armed = False
    line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
    j = json.loads(line)["roofline"]
    timed = durs[-j["samples"]:]
    print(f"bench HIP-event avg of the sampled k_sell<kPcg> launches: {j['avg_launch_ms']:.4f} ms over {j['samples']} samples")
    print("rocprof durations of the first fine PCG SpMV after each k_pcg_init (ms):", [round(x, 4) for x in durs])
    print(f"rocprof mean over the {len(timed)} timed ones: {sum(timed) / len(timed):.4f} ms")


if __name__ == "__main__":
    main()
