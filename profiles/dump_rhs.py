"""The right-hand side a subdomain's body balance sees late in the headline run (what bench.py's
cpu_baseline prices: the device state after warmup + timed iterations), saved for the CPU smoother
study (profiles/smoother_study.py --rhs FILE): the device takes 18 PCG iterations on it where the
reference's SGS takes 15.

    python profiles/dump_rhs.py OUT_DIR [subdomain ...]
"""
import importlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
D = importlib.import_module("ddpca-admm_amd")


def main():
    out = Path(sys.argv[1])
    out.mkdir(parents=True, exist_ok=True)
    subs = [int(v) for v in sys.argv[2:]] or [1]
    P = D.headline_problem()
    P.set_coarse(D.HEADLINE_MUSC["muscSett"], [D.HEADLINE_MUSC["doleMcsc"]] * P.nsub)
    P.ESTABLISH()
    mc = D.MCONTACT(P, **D.headline_options(P.nsub))
    mc.CONTACT_ANALYSIS(12, check=False)
    print("device PCG iterations of the last iteration", list(mc.get("pcg_iters")), flush=True)
    body = [tuple(int(v) for v in P.array("iface_body", ts)) for ts in range(P.nint)]
    for tv in subs:
        # consForc + consOper (systTran_pena aux - systTran lambda) on the free dofs (MCONTACT.h:2520-2524)
        G = P.grid(tv)
        flag = G.consFlag == 1
        f = np.zeros(len(flag))
        for ts in range(P.nint):
            for s in range(2):
                if body[ts][s] == tv:
                    f += P.csr("systTran_pena", 2 * ts + s) @ mc.get("inteAuxi", 2 * ts + s)
                    f -= P.csr("systTran", 2 * ts + s) @ mc.get("inteLagr", 2 * ts + s)
        b = G.consForc + f[flag]
        np.save(out / f"rhs_sd{tv}.npy", b)
        print("saved", tv, len(b), float(np.linalg.norm(b)), flush=True)


if __name__ == "__main__":
    main()
