"""Cross-check of bench.py's whole-step roofline (roofline.step_*) against a one-stream rocprofv3
kernel trace and PMC passes over every kernel of the same configuration.

    python profiles/step_check.py TRACE_DB BENCH_JSON [--fetch FETCH_CSV --write WRITE_CSV] [--out out.json]

TRACE_DB: rocpd database of `DDPCA_STREAMS=1 rocprofv3 --kernel-trace --stats -- python3 bench.py
--steps K --warmup 1 --no-cpu-baseline` (one stream, so kernel durations do not include waiting for
the other half's waves); BENCH_JSON: that run's JSON line (its byte model of the same iterations).
FETCH/WRITE: run_counter_collection.csv of `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
passes (all kernels) over `bench.py --steps 1 --warmup 1`: HBM bytes per phase of one ADMM
iteration (FETCH_SIZE x 2 KB, WRITE_SIZE KB: MI355X_MICROARCH.md's gfx950 corrections, checked in
profiles/r01_pmc_calibration.txt).

Every launch of an ADMM iteration (which ends with its MONITOR reductions, k_reduce_pairs) is put
in one of bench.py's phases by name, grid and position:
  fine_level_pcg            k_sell<3> and the V-cycle's launches on the fine level (grid = fine
                            nodes; the multicolour sweeps k_gs), k_axpy, the restriction out of
                            the fine level
  coarse_levels_and_scalars every other launch of the PCG (coarser levels, k_coarse, k_fin)
  coarse_space              launches between k_outp and the interface's first launch
  mass_cg                   k_mcg_*, k_mcheb_* (the Chebyshev start), k_scal_*
  interface_rhs_monitor     the rest (copies, k_cpl, k_outp, gamma, projection, traction, norms)
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re
import sqlite3
import statistics

PHASES = ["fine_level_pcg", "coarse_levels_and_scalars", "coarse_space", "mass_cg", "interface_rhs_monitor"]
PCG = ("k_sell", "k_jac0", "k_restrict", "k_prolong", "k_axpy", "k_fin", "k_coarse", "k_dot", "k_pcg_init",
       "k_split_sc", "k_merge_sc", "k_diag", "k_gs")
IFACE_START = ("k_gamma_ip", "k_sell_w", "k_project", "k_pair_norms")


def short(name: str) -> str:
    m = re.search(r"(k_\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def split_iterations(seq):
    """seq: [(name, grid, dur, start)] in time order -> list of iterations (lists of launches);
    an iteration ends with its MONITOR reduction (the last k_reduce_pairs before the next copy)."""
    its, cur, seen_red = [], [], False
    for r in seq:
        n = short(r[0])
        if seen_red and not n.startswith("k_reduce_pairs") and not n.startswith("k_pair_norms"):
            its.append(cur)
            cur, seen_red = [], False
        cur.append(r)
        if n.startswith("k_reduce_pairs"):
            seen_red = True
    if cur:
        its.append(cur)
    # ADMM iterations only (trailing read-backs and setup launches carry no PCG)
    return [it for it in its if any(short(r[0]).startswith("k_pcg_init") for r in it)]


def classify(it):
    """phase of every launch of one ADMM iteration"""
    names = [short(r[0]) for r in it]
    fine_grid = max((r[1] for r, n in zip(it, names) if n.startswith("k_sell<3")), default=0)
    rgrid = max((r[1] for r, n in zip(it, names) if n.startswith("k_restrict")), default=0)
    out = []
    stage = "pre"
    for r, n in zip(it, names):
        if n.startswith("k_pcg_init"):
            stage = "pcg"
        elif n.startswith("k_outp"):
            stage = "cs"
            out.append("interface_rhs_monitor")
            continue
        elif stage == "cs" and n.startswith(IFACE_START):
            stage = "iface"
        if n.startswith(("k_mcg", "k_mcheb", "k_scal")):
            out.append("mass_cg")
        elif stage == "pcg" and n.startswith(PCG):
            fine = (n.startswith(("k_sell", "k_jac0", "k_prolong", "k_axpy", "k_pcg_init")) and r[1] >= 0.5 * fine_grid) or \
                   (n.startswith("k_restrict") and r[1] == rgrid) or n.startswith("k_gs")
            out.append("fine_level_pcg" if fine else "coarse_levels_and_scalars")
        elif stage == "cs":
            out.append("coarse_space")
        else:
            out.append("interface_rhs_monitor")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("bench_json")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pmc-bench", help="the FETCH pass's own JSON line: the byte model of exactly that iteration")
    ap.add_argument("--out")
    a = ap.parse_args()
    def last_json(path):
        out = None
        for line in open(path):
            line = line.strip()
            if line.startswith("{"):
                out = json.loads(line)
        return out
    bench = last_json(a.bench_json)
    roof = bench["roofline"]
    model = roof["step_split_bytes"]
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, duration, start from kernels order by start").fetchall()
    its = split_iterations(rows)
    # the timed iterations: the last `steps` complete ones
    steps = bench["steps"]
    its = its[-steps:]
    per = {p: [] for p in PHASES}
    wall = []
    for it in its:
        ph = classify(it)
        acc = collections.Counter()
        for r, p in zip(it, ph):
            acc[p] += r[2]
        for p in PHASES:
            per[p].append(acc[p] / 1e6)
        wall.append((it[-1][3] + it[-1][2] - it[0][3]) / 1e6)
    res = {"iterations_used": len(its), "bench_ms_per_step": bench["ms_per_step"],
           "trace_window_ms_per_iter": statistics.median(wall), "phases": {}}
    tot_ms = 0.0
    for p in PHASES:
        ms = statistics.median(per[p])
        tot_ms += ms
        b = model[p]
        res["phases"][p] = {"kernel_ms_per_iter": ms, "model_bytes_per_iter": b,
                            "achieved_GBs": b / (ms * 1e-3) / 1e9 if ms > 0 else None,
                            "frac_of_8TBs": b / (ms * 1e-3) / 8e12 if ms > 0 else None}
    res["kernel_ms_per_iter"] = tot_ms
    res["model_step_bytes"] = roof["step_bytes"]
    res["bench_step_frac"] = roof["step_frac"]
    res["kernel_time_step_frac"] = roof["step_bytes"] / (tot_ms * 1e-3) / 8e12
    res["trace_window_step_frac"] = roof["step_bytes"] / (res["trace_window_ms_per_iter"] * 1e-3) / 8e12
    if a.fetch and a.write:
        # PMC passes (--steps 1 --warmup 1): the last complete iteration of each pass
        def pmc(path, counter, scale):
            recs = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
                          for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter)
            seq = [(n, g, 0, s, v) for s, n, g, v in recs]
            it = split_iterations(seq)[-1]
            ph = classify(it)
            acc = collections.Counter()
            for r, p in zip(it, ph):
                acc[p] += r[4] * scale
            return acc
        fetch = pmc(a.fetch, "FETCH_SIZE", 2.0 * 1024)
        write = pmc(a.write, "WRITE_SIZE", 1024.0)
        pm = last_json(a.pmc_bench)["roofline"] if a.pmc_bench else roof
        tot_t = 0.0
        for p in PHASES:
            t = fetch[p] + write[p]
            tot_t += t
            res["phases"][p]["pmc_hbm_bytes_per_iter"] = t
            res["phases"][p]["pmc_model_bytes_per_iter"] = pm["step_split_bytes"][p]
            res["phases"][p]["pmc_over_model"] = t / pm["step_split_bytes"][p] if pm["step_split_bytes"][p] else None
        res["pmc_step_bytes"] = tot_t
        res["pmc_over_model"] = tot_t / pm["step_bytes"]
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
