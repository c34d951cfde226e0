"""Shared fixtures.  `-m gpu` tests need a gfx950 device and the built libddpca_amd.so; the
rest run on CPU (oracle vs golden vectors, host operator pipeline, C-ABI exports)."""
import importlib
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def ddpca():
    return importlib.import_module("ddpca-admm_amd")


@pytest.fixture(scope="session")
def oracle():
    return importlib.import_module("oracle.oracle")


def golden(name: str):
    return np.load(GOLDEN / f"{name}.npz")


def ref_csr(g, name):
    import scipy.sparse as sp
    return sp.csr_matrix((g[name + "_val"], g[name + "_col"], g[name + "_ptr"]), shape=tuple(g[name + "_shape"]))


# problem parameters that reproduce each golden case's meshes
CASE_PARAMS = {
    "beam_s1": ("beam", 8, 2, 2, 1, 1, 1, 1),
    "beam_s2": ("beam", 8, 2, 2, 2, 1, 1, 1),
    "beam_gl1": ("beam", 64, 4, 2, 1, 1, 1, 1),
    "beam_dd": ("beam", 8, 2, 2, 1, 2, 1, 1),
    "twoblock_f0": ("twoblock", 0.0, 2),
    "twoblock_f3": ("twoblock", 0.3, 2),
    "beam_dd_m2": ("beam", 4, 2, 2, 2, 2, 1, 1),
    "twoblock_f0_m2": ("twoblock", 0.0, 2),
    "twoblock_f3_m2": ("twoblock", 0.3, 2),
    "twoblock_f0_m1": ("twoblock", 0.0, 2),
    "twoblock_f3_m1": ("twoblock", 0.3, 2),
}


@pytest.fixture(scope="session")
def gpu(ddpca):
    if not ddpca.gpu_available():
        pytest.skip("no gfx950 GPU visible")
    return True
