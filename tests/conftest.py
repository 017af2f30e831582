"""Shared pytest setup: markers, import paths, golden-fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "tetraear-bladerf_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG_ROOT, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def iq_to_c64(iq):
    return (iq[:, 0].astype(np.float32) / 32768 + 1j * (iq[:, 1].astype(np.float32) / 32768)).astype(np.complex64)


@pytest.fixture(scope="session")
def g1():
    z = np.load(os.path.join(GOLDEN, "g1_demod.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
    return z, meta["g1"]


@pytest.fixture(scope="session")
def g2():
    z = np.load(os.path.join(GOLDEN, "g2_decode.npz"))
    meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
    return z, meta["g2"]


@pytest.fixture(scope="session")
def g3():
    return np.load(os.path.join(GOLDEN, "g3_burst.npz"))
