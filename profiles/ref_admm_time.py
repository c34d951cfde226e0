"""The reference's OWN ADMM iteration on the bench workload (VERDICT r05 missing #2).

ORACLE / MEASUREMENT INFRASTRUCTURE -- not part of the product.  Builds the headline problem (or a
smaller one), runs the device ADMM loop to a late state (bench.py's option set), writes every
operator the reference's CONTACT_ANALYSIS reads plus that state as raw files (dump()), and runs
oracle/_ref/ref_admm_time (compiled from /root/reference's headers by oracle/Makefile): the
reference's unmodified MCONTACT::CONTACT_ANALYSIS on those operators -- all subdomains'
MGPIS::CG_SOLV(1) in its omp parallel for, the interface-eliminated coarse correction, the
interface step with its LDLT mass solves, MONITOR and its per-iteration text output -- timed per
iteration from its own "The <tc>-th iteration" lines (run()).

    python profiles/ref_admm_time.py OUT.json [--gl G] [--steps K] [--stop S] [--no-device] [--threads T]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
IFACE = ("systTran", "systTran_pena", "inteMass", "inteMass_pena", "inpoLagr", "pemaInpo_r", "inteInpo")


def _log(msg):
    print(f"[ref_admm_time] {msg}", file=sys.stderr, flush=True)


class Dump:
    def __init__(self, d: str):
        self.d = d
        self.meta = []

    def csr(self, name, P, base, index=0, level=0):
        shape = P.array(f"{base}:shape", index, level)
        ptr = np.ascontiguousarray(P.array(f"{base}:ptr", index, level), dtype=np.int64)
        ptr.tofile(f"{self.d}/{name}.ptr")
        np.ascontiguousarray(P.array(f"{base}:col", index, level), dtype=np.int32).tofile(f"{self.d}/{name}.col")
        np.ascontiguousarray(P.array(f"{base}:val", index, level), dtype=np.float64).tofile(f"{self.d}/{name}.val")
        self.meta.append(f"csr {name} {int(shape[0])} {int(shape[1])} {int(ptr[-1])}")

    def vec(self, name, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        v.tofile(f"{self.d}/{name}.f64")
        self.meta.append(f"vec {name} {len(v)}")

    def ivec(self, name, v):
        v = np.ascontiguousarray(v, dtype=np.int64)
        v.tofile(f"{self.d}/{name}.i64")
        self.meta.append(f"ivec {name} {len(v)}")

    def close(self):
        with open(f"{self.d}/meta.txt", "w") as f:
            f.write("\n".join(self.meta) + "\n")


def dump(P, d: str, state=None) -> None:
    """Every operand of the reference's ADMM loop for problem P (uniform subdomains: no hanging
    level) and the state {u[tv], aux[ts][s], lam[ts][s]} (None: zeros) into directory d."""
    nsub, nint = P.nsub, P.nint
    D = Dump(d)
    try:
        musc = 2 if P.csr("globCoup_1").shape[0] > 0 else 0
    except Exception:  # noqa: BLE001 -- no coarse space
        musc = 0
    D.meta += [f"nsub {nsub}", f"nint {nint}", f"muscSett {musc}"]
    for tv in range(nsub):
        _log(f"dumping subdomain {tv}")
        flag = np.asarray(P.array("consFlag", tv))
        N = len(flag) // 3
        nlev = int(P.array("maxiLeve", tv)[0]) + 1
        nfree = int(P.array("freeCount", tv)[-1])
        if len(P.csr("K", tv, nlev - 1).indptr) - 1 != nfree:
            raise ValueError("subdomain with a hanging level: the dump covers uniform subdomains only")
        D.meta.append(f"sub {tv} {N} {nlev} {nfree}")
        for l in range(nlev):
            D.csr(f"K{tv}_{l}", P, "K", tv, l)
        for l in range(nlev - 1):
            D.csr(f"P{tv}_{l}", P, "P", tv, l)
        D.ivec(f"consFlag{tv}", flag)
        D.vec(f"consForc{tv}", P.array("consForc", tv))
        cd = P.array("consDofv", tv)
        if len(cd):
            D.ivec(f"cdof{tv}", cd)
            D.vec(f"cval{tv}", P.array("consDofv_val", tv))
        D.vec(f"u{tv}", state["u"][tv] if state else np.zeros(3 * N))
    for ts in range(nint):
        _log(f"dumping interface {ts}")
        body = [int(b) for b in P.array("iface_body", ts)]
        fric = float(P.array("iface_param", ts)[0])
        nip = len(P.array("ip_w", ts))
        D.meta.append(f"iface {ts} {body[0]} {body[1]} {fric!r} {nip}")
        D.vec(f"basis{ts}", P.array("ip_basis", ts))
        D.vec(f"pemaDiag{ts}", P.array("pemaDiag", ts))
        D.vec(f"inpoNgap{ts}", P.array("inpoNgap", ts))
        for s in range(2):
            for n in IFACE:
                D.csr(f"{n}{ts}_{s}", P, n, 2 * ts + s)
            m = P.csr("inteMass", 2 * ts + s).shape[0]
            D.vec(f"aux{ts}_{s}", state["aux"][ts][s] if state else np.zeros(m))
            D.vec(f"lam{ts}_{s}", state["lam"][ts][s] if state else np.zeros(m))
    if musc:
        D.csr("globCoup_1", P, "globCoup_1")
        D.vec("globForc_1", P.array("globForc_1"))
        for ts in range(nint):
            for s in range(2):
                D.csr(f"globTran_1{ts}_{s}", P, "globTran_1", 2 * ts + s)
        for tv in range(nsub):
            D.csr(f"globTran_D_1{tv}", P, "globTran_D_1", tv)
            D.csr(f"accuProl{tv}", P, "accuProl", tv)
        D.ivec("baseReco", P.array("baseReco"))
        D.ivec("doleMcsc", P.array("doleMcsc"))
    D.close()


def run(exe, d: str, stop: int = 2, threads: int | None = None, timeout_s: float = 1500.0) -> dict:
    """ref_admm_time on dump d: the wall time of each of the first `stop` iterations of the
    reference's CONTACT_ANALYSIS (its text output into a scratch directory) and its resuMoni rows."""
    out = tempfile.mkdtemp(prefix="ddpca_refadmm_out_")
    env = dict(os.environ)
    if threads:
        env["OMP_NUM_THREADS"] = str(threads)
    try:
        # stderr forwarded line by line (progress of a run of minutes), stdout (the reference's own
        # prints) goes to the harness's pipe
        p = subprocess.Popen([str(exe), d, out, str(stop)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                             env=env)
        t0, err = time.perf_counter(), []
        for line in p.stderr:
            err.append(line)
            if line.startswith("[ref_admm_time]"):
                _log(line.strip()[len("[ref_admm_time] "):])
            if time.perf_counter() - t0 > timeout_s:
                p.kill()
                break
        rc = p.wait()
        lines = [l for l in err if l.startswith("{")]
        if rc != 0 or not lines:
            raise RuntimeError(f"{exe}: exit {rc}: {''.join(err)[-800:]}")
        res = json.loads(lines[-1])
        if "error" in res:
            raise RuntimeError(res["error"])
        mon = Path(out) / "resuMoni.txt"
        res["resuMoni"] = np.loadtxt(mon, ndmin=2).tolist() if mon.exists() and mon.stat().st_size else []
        return res
    finally:
        shutil.rmtree(out, ignore_errors=True)


def device_state(P, mc) -> dict:
    return {"u": [mc.get("resuDisp", tv) for tv in range(P.nsub)],
            "aux": [[mc.get("inteAuxi", 2 * ts + s) for s in range(2)] for ts in range(P.nint)],
            "lam": [[mc.get("inteLagr", 2 * ts + s) for s in range(2)] for ts in range(P.nint)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--gl", type=int, default=None)
    ap.add_argument("--steps", type=int, default=12, help="device ADMM iterations before the state is taken")
    ap.add_argument("--stop", type=int, default=2, help="reference iterations timed")
    ap.add_argument("--no-device", action="store_true", help="zero state (no GPU)")
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--dir", default=None, help="dump directory (default: a temporary one, removed after)")
    a = ap.parse_args()
    D = importlib.import_module("ddpca-admm_amd")
    t0 = time.perf_counter()
    P = D.headline_problem(gl=a.gl)
    P.set_coarse(D.HEADLINE_MUSC["muscSett"], [D.HEADLINE_MUSC["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    _log(f"problem built in {time.perf_counter() - t0:.0f} s")
    state, dev = None, {}
    if not a.no_device:
        mc = D.MCONTACT(P, **D.headline_options(P.nsub))
        n = mc.CONTACT_ANALYSIS(a.steps, check=False)
        state = device_state(P, mc)
        dev = {"device_iterations": n, "pcg_iters_last": [int(v) for v in mc.get("pcg_iters")]}
        del mc
    d = a.dir or tempfile.mkdtemp(prefix="ddpca_refadmm_")
    os.makedirs(d, exist_ok=True)
    try:
        t = time.perf_counter()
        dump(P, d, state)
        sz = sum(f.stat().st_size for f in Path(d).iterdir())
        _log(f"dumped {sz / 1e9:.1f} GB in {time.perf_counter() - t:.0f} s")
        nsub, ndof = P.nsub, sum(int(P.array("freeCount", tv)[-1]) for tv in range(P.nsub))
        nip = sum(len(P.array("ip_w", ts)) for ts in range(P.nint))
        del P
        exe = ROOT / "oracle" / "_ref" / "ref_admm_time"
        res = run(exe, d, a.stop, a.threads)
    finally:
        if not a.dir:
            shutil.rmtree(d, ignore_errors=True)
    its = res["iteration_s"]
    res.update(dev)
    res.update({"dof": ndof, "subdomains": nsub, "integration_points": nip, "dump_bytes": sz,
                "cpu": _cpu(), "value": 1.0 / (sum(its) / len(its)), "unit": "ADMM it/s"})
    sys.path.insert(0, str(ROOT))
    import bench  # noqa: E402 -- the same host description as the bench line's
    res["host_cores"] = bench.host_cpu()
    Path(a.out).write_text(json.dumps(res))
    _log(f"reference ADMM iterations: {[round(x, 2) for x in its]} s ({res['threads']} threads) -> {res['value']:.4f} it/s")


def _cpu():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
