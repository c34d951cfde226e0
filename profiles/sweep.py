"""Configuration sweep of bench.py on one GPU: each configuration runs in its own process
(under a time limit) and one summary line per run is appended to the output file.

    python profiles/sweep.py OUT "--smoother 1 --nu 1" "DDPCA_SYM_LEVELS=1 --omega-scale 1.6" ...

Tokens of the form NAME=VALUE (upper-case NAME) are environment variables of that run.
"""
import os
import json
import subprocess
import sys
import time


def main():
    out = sys.argv[1]
    base = ["python3", "bench.py", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--no-general"]
    for cfg in sys.argv[2:]:
        t0 = time.time()
        toks = cfg.split()
        env = dict(os.environ)
        args = []
        for t in toks:
            k, eq, v = t.partition("=")
            if eq and k.isupper():
                env[k] = v
            else:
                args.append(t)
        try:
            r = subprocess.run(base + args, capture_output=True, text=True, timeout=240, env=env)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not line:
                msg = f"{cfg} | FAILED rc={r.returncode} {r.stderr[-300:]!r}"
            else:
                j = json.loads(line[-1])
                msg = (f"{cfg} | {j['value']:.3f} it/s | {j['ms_per_step']:.1f} ms | pcg/solve "
                       f"{j['pcg_iters_per_solve']:.2f} | spmv {j['roofline']['avg_launch_ms']:.3f} ms "
                       f"{j['roofline']['achieved']:.0f} GB/s")
        except subprocess.TimeoutExpired:
            msg = f"{cfg} | TIMEOUT"
        with open(out, "a") as f:
            f.write(msg + f" | wall {time.time() - t0:.0f}s\n")
        print(msg, flush=True)
        if "TIMEOUT" in msg or "rc=-" in msg:
            break  # a hang or a crash ends the sweep


if __name__ == "__main__":
    main()
