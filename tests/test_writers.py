"""The reference's result files written by the library's host writers (include/ddpca_amd.h:
ddpca_write_resuDisp / _resuCont / _resuMoni) against the reference's OWN text files
(tests/golden/text/<case>/*.gz, copied verbatim from the reference's runs by make_golden.py).

CPU: fed the values the reference printed (parsed back from its files into the golden npz), the
writers must reproduce its files byte for byte -- 20 significant digits round-trip a double
exactly, so this pins the format (std::scientific, precision 20, setw(30); setw(10) for the
friction state).  The frictional resuCont prints gamma_1 t1 + gamma_2 t2, whose inputs the
reference does not print: it is checked numerically (1e-12 of the row scale) with the other
columns and the layout exact.  GPU: the device ADMM run's files against the reference's at the
contact-pressure tolerance (1e-5) -- tests/test_mcontact_gpu.py runs it.
"""
import gzip
import re

import numpy as np
import pytest

from conftest import GOLDEN, golden

TEXT = GOLDEN / "text"


def ref_text(case, name):
    with gzip.open(TEXT / case / (name + ".gz"), "rt") as f:
        return f.read()


def test_resuMoni_byte_exact(ddpca, tmp_path):
    g = golden("twoblock_f0_m2")
    out = tmp_path / "resuMoni.txt"
    ddpca.write_resuMoni(out, g["resuMoni"])
    assert out.read_text() == ref_text("twoblock_f0_m2", "resuMoni.txt")


@pytest.mark.parametrize("tv", [0, 1])
def test_resuDisp_byte_exact(ddpca, tmp_path, tv):
    g = golden("twoblock_f0_m2")
    out = tmp_path / f"resuDisp_{tv}.txt"
    ddpca.write_resuDisp(out, g[f"sd{tv}_resuDisp"])
    assert out.read_text() == ref_text("twoblock_f0_m2", f"resuDisp_{tv}.txt")


def test_resuDisp_rotated_nodes(ddpca, tmp_path):
    """MULTIGRID::nodeRota: listed nodes are printed as R u."""
    u = np.arange(12, dtype=float)
    R = np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    out = tmp_path / "d.txt"
    ddpca.write_resuDisp(out, u, rot_node=[2], rot=R.reshape(1, 9))
    got = np.loadtxt(out)
    ref = u.reshape(-1, 3).copy()
    ref[2] = R @ ref[2]
    assert np.array_equal(got, ref)


def test_resuCont_frictionless_byte_exact(ddpca, tmp_path):
    g = golden("twoblock_f0_m2")
    out = tmp_path / "resuCont_0.txt"
    ddpca.write_resuCont(out, 0.0, g["if0_resuCont"])
    assert out.read_text() == ref_text("twoblock_f0_m2", "resuCont_0.txt")


def test_resuCont_frictional_format(ddpca, tmp_path):
    g = golden("twoblock_f3_m2")
    text = ref_text("twoblock_f3_m2", "resuCont_0.txt")
    ref = g["if0_resuCont"].reshape(-1, 5)
    basis = g["if0_ip_basis"].reshape(-1, 3, 3)
    t1, t2 = basis[:, 1, :], basis[:, 2, :]
    # the tangential components behind the printed traction (t1, t2 orthonormal)
    trac = ref[:, 1:4]
    gam = np.stack([ref[:, 0], (trac * t1).sum(1), (trac * t2).sum(1)], axis=1).reshape(-1)
    stat = ref[:, 4].astype(np.int32)
    assert set(np.unique(stat)) <= {0, 1, 2} and (stat == 1).any()
    out = tmp_path / "resuCont_0.txt"
    ddpca.write_resuCont(out, 0.3, gam, stat, basis.reshape(-1))
    mine, theirs = out.read_text().splitlines(), text.splitlines()
    assert len(mine) == len(theirs)
    line = re.compile(r"^(?:[ -][ 0-9.e+-]{29}){4}[ 0-9]{9}[0-2]$")
    for a, b in zip(mine, theirs):
        assert line.match(a) and line.match(b) and len(a) == len(b) == 130
        assert a[:30] == b[:30] and a[120:] == b[120:]  # gamma_n and the state: exact
    got = np.loadtxt(out)
    scale = np.abs(ref[:, 1:4]).max(axis=1)
    assert np.all(np.abs(got[:, 1:4] - ref[:, 1:4]).max(axis=1) <= 1e-12 * scale + 1e-300)


def test_writers_reject_bad_arguments(ddpca, tmp_path):
    with pytest.raises(ddpca.DdpcaError):
        ddpca.write_resuMoni(tmp_path / "no" / "such" / "dir.txt", np.zeros((1, 2)))
    gam = np.zeros(3)
    with pytest.raises(ddpca.DdpcaError):  # frictional output needs the state and the basis
        ddpca._check(ddpca.lib().ddpca_write_resuCont(str(tmp_path / "c.txt").encode(), 0.3, 1,
                                                      gam.ctypes.data, None, None))
