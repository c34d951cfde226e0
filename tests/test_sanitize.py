"""ASan + UBSan run of the host C++ (SURVEY §5 "race detection / sanitizers").

tests/sanitize/Makefile compiles every host translation unit of libddpca_amd (the setup code that
produces every GPU operand: generators, MCONTACT::ESTABLISH's mortar operators, the MULTIGRID
pipeline on any octree, both coarse spaces, CSEARCH, CURVEDS/REFINE, the writers; no device code)
with -fsanitize=address,undefined and links tests/sanitize/host_driver.cpp, which drives them through
the C ABI (problems of every generator incl. rank-local builds, a refined curved octree, a contact
search, the refused-argument paths).  A sanitizer report aborts the driver (halt_on_error).  The
reference-comparison harnesses of the CPU tests linked to the same objects (`make ref run`:
ref_multigrid, ref_csearch, ref_refine, ref_lagrange_host, about 5 minutes) ran clean too:
profiles/r04_sanitize.log."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent / "sanitize"


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_host_code_is_clean_under_asan_and_ubsan(tmp_path):
    b = subprocess.run(["make", "-C", str(HERE), "-j8", "all"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    exe = HERE.parents[1] / "ddpca-admm_amd" / "build" / "san" / "host_driver"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", OMP_NUM_THREADS="4", TMPDIR=str(tmp_path),
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, cwd=tmp_path, env=env)
    report = r.stdout[-2000:] + r.stderr[-4000:]
    assert r.returncode == 0, report
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, report
    assert r.stdout.strip().splitlines()[-1] == '{"ok": true, "failures": 0}', report
