"""Container-only CPU calibration (needs /root/reference and oracle/_ref built): the reference's
own MGPIS::CG_SOLV(1) (oracle/_ref/ref_harness time_cg, compiled with the reference's flags) and
the SGS-faithful oracle port (oracle/oracle.cpp, the bench's cpu_baseline) on the SAME BEAM mesh
(BEAM.h NODD, diviNumb 64x4x2, globLeve gl), same thread count.  The ratio t_reference / t_port
lets the GPU host's port timing (bench.py cpu_baseline) stand for the reference, which never
travels to the GPU box.

    python profiles/cpu_calibration.py [gl] [reps] [binary] > profiles/r02_cpu_calibration.json

`binary` (default ref_harness) names the build under oracle/_ref: on the GPU host run it with
ref_harness_portable (compiled without -march=native in this container, oracle/Makefile), which
travels to the box with the snapshot -- the ratio is then measured on the host the bench's
cpu_baseline runs on, at that host's thread count.
"""
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return os.uname().machine


def main():
    gl = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    binary = sys.argv[3] if len(sys.argv) > 3 else "ref_harness"
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([str(ROOT / "oracle" / "_ref" / binary), "time_cg", "64", "4", "2", str(gl), str(reps)],
                         capture_output=True, text=True, env=env, check=True, cwd="/tmp")
    ref = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    import importlib
    D = importlib.import_module("ddpca-admm_amd")
    from oracle import oracle as O
    P = D.Problem("beam", 64, 4, 2, gl, 1, 1, 1).ESTABLISH()
    G = P.grid(0)
    L = G.maxiLeve
    M = O.MgpisOracle([G.consStif(l) for l in range(L + 1)], [G.realProl(l) for l in range(L)])
    port = []
    for _ in range(reps):
        t = time.perf_counter()
        x, it, rr = M.CG_SOLV(1, G.consForc)
        port.append(dict(cg_s=time.perf_counter() - t, iters=int(it)))
    t_ref = statistics.median(r["cg_s"] for r in ref)
    t_port = statistics.median(p["cg_s"] for p in port)
    print(json.dumps(dict(
        mesh=f"BEAM NODD 64x4x2 globLeve {gl}", n=ref[0]["n"], threads=threads, cpu=_cpu_model(), binary=binary,
        host=os.uname().nodename,
        reference=dict(cg_s=[r["cg_s"] for r in ref], iters=[r["iters"] for r in ref], median_s=t_ref),
        port=dict(cg_s=[p["cg_s"] for p in port], iters=[p["iters"] for p in port], median_s=t_port),
        ref_over_port=t_ref / t_port), indent=1))


if __name__ == "__main__":
    main()
