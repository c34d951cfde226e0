"""The multicolour fine-level sweeps (k_gs<0|1|2>) at the bench configuration, for a per-launch
rocprof / PMC table (profiles/gs_table.py).

    python profiles/gs_probe.py --out DIR [--steps 2]

One stream per batch (DDPCA_STREAMS=1: every launch covers the whole batch, so its duration and its
PMC bytes are one full colour launch) and the bench's headline problem and option set; writes
DIR/gs_model.json: the library's per-launch byte model (mcontact_gpu_get "gs_launch_bytes": forward
colours 0..K-1, the residual, backward colours K-1..0) and the chunk count of each launch.  Run it
under `rocprofv3 --kernel-trace --stats` and under two `--pmc` passes (FETCH_SIZE, WRITE_SIZE) with
`--kernel-include-regex k_gs`.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gl", type=int, default=None)
    a = ap.parse_args()
    os.environ.setdefault("DDPCA_STREAMS", "1")
    D = importlib.import_module("ddpca-admm_amd")
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    t0 = time.perf_counter()
    P = D.headline_problem(a.gl)
    P.set_coarse(D.HEADLINE_MUSC["muscSett"], [D.HEADLINE_MUSC["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    mc = D.MCONTACT(P, device=0, **D.headline_options(P.nsub))
    print(f"[gs_probe] setup {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    mc.CONTACT_ANALYSIS(a.steps, check=False)
    model = mc.get("gs_launch_bytes")
    K = (len(model) - 1) // 2
    tm = mc.timing()
    res = {"colours": K, "launch_bytes": [float(v) for v in model],
           "order": [f"fwd{k}" for k in range(K)] + ["resid"] + [f"bwd{k}" for k in range(K - 1, -1, -1)],
           "admm_iterations": a.steps, "pcg_iterations": tm["pcg_iterations"],
           "streams": os.environ.get("DDPCA_STREAMS")}
    (out / "gs_model.json").write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: res[k] for k in ("colours", "pcg_iterations")}), flush=True)


if __name__ == "__main__":
    main()
