"""The Python drop-in (INTEGRATION.md option A): this build's package ahead of the reference's on
sys.path, the reference's callers unchanged (tetraear/_overlay.py).

With the reference present (this container only; skipped elsewhere -- nothing of the reference
travels), tests/overlay_probe.py runs twice in fresh processes: once on the reference alone, once on
the overlay.  Checked:
  * every non-Qt module /root/reference/tetraear/ui/modern.py:193-201 imports resolves -- the hot-path
    modules to this build's files, the others (capture, crypto, mcc_mnc, validator, location, audio)
    to the reference's; the package-level lazy names of tetraear/__init__.py:24-36 resolve;
  * the hot-path methods (process, decode, parse_burst, _check_crc, _calculate_crc16, parse_mac_pdu,
    ...) are this build's functions; FrequencyScanner is the reference's sweep over this build's detector;
  * TetraDecoder.set_keys and TetraProtocolParser.parse_sds_data give the reference's results;
  * the 59 g2 golden streams through this build's MAC PDU stage and upper_mac give the reference's
    own decode() frame dicts key for key -- call_metadata, sds_message, decoded_text, is_reassembled,
    additional_info -- and, with auto_decrypt, the decryption fields; 153 frames each way.
Without a reference the build stands alone: the upper-MAC members raise ReferenceUnavailable."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("TETRA_REFERENCE", "/root/reference")
PKG = os.path.realpath(os.path.join(REPO, "tetraear-bladerf_amd", "tetraear"))


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "TETRAEAR_REFERENCE_ROOT")}
    env.update(extra)
    return env


@pytest.fixture(scope="module")
def probes(tmp_path_factory):
    if not os.path.isfile(os.path.join(REF, "tetraear", "core", "protocol.py")):
        pytest.skip("the reference is not present (it exists in the build container only)")
    d = tmp_path_factory.mktemp("overlay")
    out = {}
    for mode in ("reference", "overlay"):
        path = str(d / f"{mode}.json")
        r = subprocess.run([sys.executable, os.path.join(HERE, "overlay_probe.py"), mode, path], cwd=str(d),
                           env=_clean_env(TETRA_REFERENCE=REF), capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        out[mode] = json.load(open(path))
    return out


def test_modules_resolve_through_the_overlay(probes):
    o = probes["overlay"]
    ref = os.path.realpath(os.path.join(REF, "tetraear"))
    for m, f in o["modules"].items():
        mine = m in ("tetraear.signal.processor", "tetraear.signal.scanner", "tetraear.core.decoder",
                     "tetraear.core.protocol")
        assert f.startswith(PKG if mine else ref), (m, f)
    assert set(o["top_level"]) == {"TetraDecoder", "TEADecryptor", "TetraKeyManager", "TetraProtocolParser",
                                   "SignalProcessor", "BladeRFCapture", "TetraSignalDetector", "VoiceProcessor"}


def test_hot_path_never_delegates(probes):
    o = probes["overlay"]
    for name, f in o["hot"].items():
        assert f.startswith(PKG), (name, f)
    assert o["scanner_detector"]          # FrequencyScanner(...).detector is the GPU TetraSignalDetector
    assert o["common_keys"] == ["TEA1", "TEA2", "TEA3", "TEA4"]
    assert o["bound"] == ["method", "_tetraear_reference.core.decoder"]


def test_set_keys_and_sds_equal_the_reference(probes):
    r, o = probes["reference"], probes["overlay"]
    assert o["user_keys"] == r["user_keys"] and len(r["user_keys"]) == 8
    assert o["sds"] == r["sds"] and any(s for s in r["sds"])
    assert o["sds_stats"] == r["sds_stats"]


@pytest.mark.parametrize("auto_decrypt", [False, True])
def test_upper_mac_frames_equal_the_reference(probes, auto_decrypt):
    r, o = probes["reference"][f"frames_{auto_decrypt}"], probes["overlay"][f"frames_{auto_decrypt}"]
    assert len(r) == len(o) == 59
    upper = set()
    for i, (a, b) in enumerate(zip(r, o)):
        assert len(a) == len(b), i
        for fa, fb in zip(a, b):
            assert fa == fb, (i, {k: (fa.get(k), fb.get(k)) for k in set(fa) | set(fb) if fa.get(k) != fb.get(k)})
            upper |= set(fa) & {"call_metadata", "sds_message", "decoded_text", "is_reassembled", "decrypted"}
    assert sum(len(a) for a in r) == 153
    assert {"call_metadata", "sds_message", "is_reassembled"} <= upper   # the streams exercise the upper MAC
    if auto_decrypt:
        assert "decrypted" in upper


def test_standalone_build_names_the_missing_reference():
    """No reference on the path: the hot path imports and constructs as before, the upper MAC and the
    reference-only modules raise ImportError subclasses naming the overlay."""
    code = r"""
import sys
sys.path.insert(0, sys.argv[1])
import tetraear
from tetraear import _overlay
assert not _overlay.active() and len(tetraear.__path__) == 1, tetraear.__path__
from tetraear.core import TetraDecoder, TetraProtocolParser
d = TetraDecoder(auto_decrypt=False)
d.set_keys(["00112233445566778899"])
assert d.user_keys == [("TEA1", bytes.fromhex("00112233445566778899"))]
frame = {"additional_info": {}, "encrypted": True}
assert d.upper_mac(frame, None, None) is frame
for call in (lambda: TetraProtocolParser().parse_sds_data(b"x"), lambda: __import__("tetraear.signal.capture"),
             lambda: __import__("tetraear.signal.scanner", fromlist=["FrequencyScanner"]).FrequencyScanner,
             lambda: tetraear.core.TEADecryptor):
    try:
        call()
        raise SystemExit("no error")
    except ImportError as e:
        pass
try:
    d.common_keys
    raise SystemExit("common_keys without the reference")
except AttributeError:
    pass
print("ok")
"""
    r = subprocess.run([sys.executable, "-c", code, os.path.join(REPO, "tetraear-bladerf_amd")], cwd="/",
                       env=_clean_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-3000:] + r.stdout


def test_second_copy_of_the_build_is_not_the_reference(tmp_path):
    """a second copy of this build on sys.path (an installed wheel beside the source tree)
    must not be taken for the reference -- its parser would delegate back to the overlay and recurse.
    TETRAEAR_OVERLAY=0 turns the path scan off (only TETRAEAR_REFERENCE_ROOT is then consulted)."""
    import shutil
    copy = tmp_path / "site"
    shutil.copytree(os.path.join(REPO, "tetraear-bladerf_amd", "tetraear"), copy / "tetraear",
                    ignore=shutil.ignore_patterns("__pycache__", "*.so"))
    fake = tmp_path / "ref"
    (fake / "tetraear").mkdir(parents=True)
    (fake / "tetraear" / "__init__.py").write_text("")
    code = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
sys.path.append(sys.argv[2])
from tetraear import _overlay
pk = _overlay.reference_packages()
assert not any(os.path.isfile(os.path.join(p, "_overlay.py")) for p in pk), pk
if sys.argv[3] == "scan":
    assert pk == [os.path.realpath(os.path.join(sys.argv[4], "tetraear"))], pk
else:
    assert pk == [], pk
print("ok")
"""
    pkg = os.path.join(REPO, "tetraear-bladerf_amd")
    for mode, env in (("scan", _clean_env()), ("off", _clean_env(TETRAEAR_OVERLAY="0"))):
        r = subprocess.run([sys.executable, "-c", code, pkg, str(copy), mode, str(fake)], cwd="/",
                           env=env, capture_output=True, text=True, timeout=120)
        # the fake reference sits after the copy on the path in "scan" mode
        if mode == "scan":
            r = subprocess.run([sys.executable, "-c", code.replace("sys.path.append(sys.argv[2])",
                                                                   "sys.path.append(sys.argv[2]); sys.path.append(sys.argv[4])"),
                                pkg, str(copy), mode, str(fake)], cwd="/", env=env, capture_output=True, text=True,
                               timeout=120)
        assert r.returncode == 0 and r.stdout.strip() == "ok", (mode, r.stderr[-3000:] + r.stdout)
