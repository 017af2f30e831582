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


# What the build's decode() frames do NOT carry (the reference's upper MAC, decoder.py:1055-1117,
# out of scope per SURVEY.md §2; TetraDecoder.upper_mac is the hook): frame keys recorded in the
# golden g2 records as 'upper_keys', and additional_info entries beyond the MAC PDU stage's.
UPPER_MAC_KEYS = {"call_metadata", "sds_message", "decoded_text", "is_reassembled"}
UPPER_MAC_INFO = {"talkgroup", "source_ssi", "sds_text", "mcc", "mnc"}   # call metadata: decoder.py:1062-1080


def decoded_view(frame):
    """The fields of one decode() frame dict the golden g2 'decoded' records compare on: the
    lower-MAC fields and the MAC PDU stage (decoder.py:960-1053).  The upper-MAC keys
    (UPPER_MAC_KEYS, UPPER_MAC_INFO) are excluded by declaration: test_g2_upper_mac_gap_declared
    checks the recorded reference frames hold no other keys."""
    info = frame.get("additional_info", {})
    mp = frame.get("mac_pdu")
    if mp is not None and not isinstance(mp.get("data"), str):
        mp = dict(type=mp["type"], encrypted=bool(mp["encrypted"]),
                  address=None if mp["address"] is None else int(mp["address"]),
                  length=int(mp["length"]), data=bytes(mp["data"]).hex())
    return dict(number=frame["number"], header=frame["header"], burst_crc=frame.get("burst_crc"),
                encrypted=bool(frame["encrypted"]), encryption_algorithm=frame["encryption_algorithm"],
                encryption_mode=frame.get("encryption_mode", info.get("encryption_mode")), mac_pdu=mp)
