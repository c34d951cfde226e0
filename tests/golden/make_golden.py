"""Regenerate the golden fixtures of tests/golden/ from the reference itself.

Container-only (needs /root/reference): builds oracle/_ref/ref_harness with the reference's
own flags (oracle/Makefile), runs it on each case in a scratch directory and packs the .npy
outputs of every case into one compressed <case>.npz.  The fixtures are data (inputs and
expected outputs of the reference), never reference source.

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py beam_s1    # one case
    python tests/golden/make_golden.py --text     # the text-file fixtures (TEXT) only
"""
from __future__ import annotations

import glob
import gzip
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


# text-file fixtures: the reference's own result files (MULTIGRID::OUTP_SUB2, MCONTACT::
# OUTPUT_PRTR, resuMoni.txt) of a case, kept gzip'd under text/<case>/ -- data, for the writers'
# format tests (tests/test_writers.py).  `make_golden.py --text <case>` writes only these.
TEXT = {
    "twoblock_f0_m2": ["resuMoni.txt", "resuDisp_0.txt", "resuDisp_1.txt", "resuCont_0.txt"],
    "twoblock_f3_m2": ["resuMoni.txt", "resuCont_0.txt"],
}


def run_case(name: str, text_only: bool = False) -> Path:
    argv = CASES[name]
    here = Path(__file__).resolve().parent
    with tempfile.TemporaryDirectory() as work:
        out = Path(work) / "npy"
        out.mkdir()
        cmd = [str(HARNESS)] + [a.format(out=out) for a in argv]
        env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
        subprocess.run(cmd, cwd=work, check=True, env=env)
        arrays = {Path(f).stem: np.load(f) for f in sorted(glob.glob(str(out / "*.npy")))}
        for fname in TEXT.get(name, []):
            tdir = here / "text" / name
            tdir.mkdir(parents=True, exist_ok=True)
            with open(Path(work) / fname, "rb") as src, gzip.GzipFile(tdir / (fname + ".gz"), "wb", mtime=0) as dst:
                dst.write(src.read())
    if text_only:
        return here / "text" / name
    dest = here / f"{name}.npz"
    np.savez_compressed(dest, **arrays)
    return dest


def main() -> None:
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
    args = sys.argv[1:]
    text_only = "--text" in args
    names = [a for a in args if a != "--text"] or (list(TEXT) if text_only else list(CASES))
    for n in names:
        print("wrote", run_case(n, text_only))


if __name__ == "__main__":
    main()
