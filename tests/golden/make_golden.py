"""Regenerate the golden fixtures of tests/golden/ from the reference itself.

Container-only (needs /root/reference): builds oracle/_ref/ref_harness with the reference's
own flags (oracle/Makefile), runs it on each case in a scratch directory and packs the .npy
outputs of every case into one compressed <case>.npz.  The fixtures are data (inputs and
expected outputs of the reference), never reference source.

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py beam_s1    # one case
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"

# case -> harness argv (outdir appended where the mode expects it)
CASES = {
    # single-domain BEAM (BEAM.h:251-311, 403-422), full operator dumps on the smallest one
    "beam_s1": ["beam_nodd", "8", "2", "2", "1", "{out}", "1"],
    "beam_s2": ["beam_nodd", "8", "2", "2", "2", "{out}", "0"],
    "beam_gl1": ["beam_nodd", "64", "4", "2", "1", "{out}", "0"],
    # the other MGPIS drivers (MULT_SOLV, BiCGSTAB_SOLV, GMRES_SOLV) on the beam_s2 mesh
    "beam_s2_solv": ["beam_solv", "8", "2", "2", "2", "{out}"],
    # DD BEAM, 2 subdomains glued (fricCoef = -1), muscSett = 0: 3000 ADMM iterations
    "beam_dd": ["beam_dd", "8", "2", "2", "1", "2", "1", "1", "{out}"],
    # two stacked blocks: frictionless patch test and Coulomb friction (mu = 0.3)
    "twoblock_f0": ["twoblock", "0", "2", "{out}"],
    "twoblock_f3": ["twoblock", "0.3", "2", "{out}"],
    # the same with the interface-eliminated coarse space (muscSett = 2, doleMcsc = 1,
    # MCONTACT.h:1672-2301 / 2578-2612): converged runs, coarse operators dumped
    "beam_dd_m2": ["beam_dd", "4", "2", "2", "2", "2", "1", "1", "{out}", "2"],
    "twoblock_f0_m2": ["twoblock", "0", "2", "{out}", "2"],
    "twoblock_f3_m2": ["twoblock", "0.3", "2", "{out}", "2"],
    # LATIN-type coarse space (muscSett = 1, MULTISCALE, MCONTACT.h:898-1536 / 2540-2576)
    "twoblock_f0_m1": ["twoblock", "0", "2", "{out}", "1"],
    "twoblock_f3_m1": ["twoblock", "0.3", "2", "{out}", "1"],
}


def run_case(name: str) -> Path:
    argv = CASES[name]
    with tempfile.TemporaryDirectory() as work:
        out = Path(work) / "npy"
        out.mkdir()
        cmd = [str(HARNESS)] + [a.format(out=out) for a in argv]
        env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
        subprocess.run(cmd, cwd=work, check=True, env=env)
        arrays = {Path(f).stem: np.load(f) for f in sorted(glob.glob(str(out / "*.npy")))}
    dest = Path(__file__).resolve().parent / f"{name}.npz"
    np.savez_compressed(dest, **arrays)
    return dest


def main() -> None:
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
    names = sys.argv[1:] or list(CASES)
    for n in names:
        print("wrote", run_case(n))


if __name__ == "__main__":
    main()
