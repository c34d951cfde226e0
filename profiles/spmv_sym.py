"""SpMV storage experiment on one fine level (a 1.22M-dof wheel block of the bench workload):
full SELL-BSR3 vs SYM-SELL (upper blocks streamed, lower blocks re-read in place), with and
without the XCD-aware wave order.  Each configuration runs in its own process (the storage is
chosen at create from DDPCA_SYM_LEVELS / DDPCA_XCDMAP); y = Kx on a fixed vector is checked
against the full-storage result.

    python profiles/spmv_sym.py OUT
"""
import json
import os
import subprocess
import sys

CONFIGS = [("full", {"DDPCA_SYM_LEVELS": "0"}), ("sym", {"DDPCA_SYM_LEVELS": "1", "DDPCA_XCDMAP": "0"}),
           ("sym+xcd", {"DDPCA_SYM_LEVELS": "1", "DDPCA_XCDMAP": "1"})]
VARIANTS = [("f64 spmv L0", 0), ("f64 spmv L1", 1), ("f64 pcg L0", 4), ("f64 pcg L1", 5),
            ("f32 resid L0", 16 + 8), ("f32 resid L1", 16 + 9), ("f32 cheb L1", 16 + 13)]


def child():
    import importlib
    import numpy as np
    sys.path.insert(0, os.getcwd())
    D = importlib.import_module("ddpca-admm_amd")
    P = D.Problem("dehw", 1, 3, 2, 2, 5, 0.2).ESTABLISH()
    M = D.MGPIS.from_problem(P, 1, device=0, precond_fp32=1, smoother=1, table_mode=0)
    n = len(P.grid(1).consForc)
    x = np.sin(np.arange(n) * 0.37)
    y = M.spmv(x)
    out = {"y": [float(np.linalg.norm(y)), float(y[::997].sum())], "ms": {}}
    np.save("/tmp/spmv_y.npy", y)
    for name, v in VARIANTS:
        if "L0" in name and os.environ.get("DDPCA_SYM_LEVELS", "0") != "0" and "f32" in name:
            continue
        ms, nb = M.bench_spmv(v, 50)
        out["ms"][name] = ms
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    out = sys.argv[1]
    res = {}
    for tag, env in CONFIGS:
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, __file__, "--child"], env=e, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            res[tag] = {"error": r.stderr[-500:]}
            print(tag, "FAILED", r.stderr[-500:], flush=True)
            break
        res[tag] = json.loads(line[-1])
        print(tag, res[tag], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
