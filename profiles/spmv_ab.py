"""A/B of fine-level SpMV kernels on one 1.22M-dof wheel block of the bench workload
(mgpis_gpu_bench_spmv): each configuration runs in its own process with its own environment,
e.g. a second library built with other -D switches (DDPCA_AMD_LIB) -- y = Kx on a fixed vector
is printed for the cross-check.  r01_spmv_sym.json was made by this script when it compared the
full SELL-BSR3 storage with a symmetric (upper-block) storage, since removed (commit 99c5bfc).

    python profiles/spmv_ab.py OUT tag1:NAME=VAL,NAME=VAL tag2:...
"""
import json
import os
import subprocess
import sys

VARIANTS = [("f64 spmv L1", 1), ("f64 spmv L2", 2), ("f64 spmv L3", 3), ("f64 pcg L1", 5), ("f64 pcg L2", 6),
            ("f32 resid L1", 16 + 9), ("f32 resid L2", 16 + 10), ("f32 resid L3", 16 + 11), ("f32 cheb L1", 16 + 13)]


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
    for name, v in VARIANTS:
        ms, nb = M.bench_spmv(v, 50)
        out["ms"][name] = round(ms * 1e3, 2)  # us
        out.setdefault("GBs", {})[name] = round(nb / ms / 1e6)
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    out = sys.argv[1]
    res = {}
    for spec in sys.argv[2:]:
        tag, _, kv = spec.partition(":")
        env = dict(p.split("=", 1) for p in kv.split(",") if p)
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
