"""CPU-only checks: the C ABI library loads and exports every declared symbol; host logic."""
import os
import re

import numpy as np
import pytest

import compat as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = []
    for h in os.listdir(os.path.join(REPO, "include")):
        if h.endswith(".h"):
            txt = open(os.path.join(REPO, "include", h)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            names += re.findall(r"\b(tetra_\w+)\s*\(", txt)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    from tetraear import _hip
    lib = _hip.lib()
    names = declared_functions()
    assert len(names) > 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.tetra_abi_version() == 2


def test_binding_covers_header():
    from tetraear import _hip
    lib = _hip.lib()
    for n in declared_functions():
        assert getattr(lib, n).argtypes is not None, f"{n} has no ctypes signature"


def test_no_device_fails_loudly():
    """Without a GPU the product path raises; it never computes on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from tetraear import _hip
    from tetraear.signal import SignalProcessor
    with pytest.raises(_hip.TetraHipError):
        SignalProcessor().process(np.ones(1000, np.complex64))


def test_cascade_table_matches_oracle_cascade():
    """decode()'s threshold cascade tabulated by best count == oracle cascade on real streams."""
    from tetraear.core.decoder import cascade_table
    tab = cascade_table()
    rng = np.random.default_rng(5)
    for best in range(10, 23):
        bits = rng.integers(0, 2, 3000)
        bits = np.where(rng.random(3000) < 0.5, bits, 0)
        # plant one window with exactly `best` matches, avoid accidental better windows
        w = O.SYNC_CONT.astype(int).copy()
        w[:22 - best] ^= 1
        bits[1000:1022] = w
        c1 = np.empty(len(bits) - 21, np.uint8)
        c2 = np.empty_like(c1)
        O.lib().orc_sync_counts(np.ascontiguousarray(bits, np.uint8), len(bits), c1, c2)
        m = int(np.maximum(c1, c2).max())
        got = O.decode_syncs(bits)
        k = tab[m]
        want = []
        if k >= 0:
            last = -10 ** 9
            for i in np.nonzero(np.maximum(c1, c2) >= k)[0]:
                if i >= last + 250:
                    want.append(int(i))
                    last = int(i)
        assert got == want, (best, m)


def test_compat_plan_decisions(g1):
    """Host plan reproduces the reference's control decisions for every golden case."""
    from tetraear.signal.processor import compat_plan
    from tetraear import _hip
    z, meta = g1
    for i, m in enumerate(meta):
        if m["n"] == 0:
            continue
        p, M, rate = compat_plan(m["fs"], m["n"], _hip.TETRA_CF32)
        assert (p.q > 1) == bool(m["dec_ok"]), (i, m)
        if m["dec_ok"]:
            assert p.q == m["q"]
        assert M == len(z[f"c{i}_decimated"])
        # filter applied <=> filtered dtype is complex128 for an unshifted chunk
        if f"c{i}_filtered" in z.files and not m["freq_offset"]:
            assert bool(p.filt) == (z[f"c{i}_filtered"].dtype == np.complex128), (i, m)


def test_compat_plan_real_input_state_and_private_plans():
    """decimate casts its sos to the input's dtype, so a real chunk's initial state comes from the
    real dtype (at q = 7 float32 and complex64 differ in a last bit; the plan carries the one scipy
    would use, as the oracle's decimate does).  filter_signal rewrites its plan's taps, so it gets a
    private plan: the cached one process() reuses for the same chunk shape keeps its own taps."""
    import scipy.signal as ss
    from tetraear.signal.processor import compat_plan
    from tetraear import _hip
    sos = ss.cheby1(8, 0.05, 0.8 / 7, output="sos")
    for real, t in ((False, np.complex64), (True, np.float32)):
        p, _, _ = compat_plan(1.8e6, 22849, _hip.TETRA_CF32, real=real)
        want = ss.sosfilt_zi(np.asarray(sos, t)).real.astype(np.float32).ravel()
        assert np.array_equal(np.ctypeslib.as_array(p.zi_f32)[:8], want), real
    a, _, _ = compat_plan(2.4e6, 5000, _hip.TETRA_CF32)
    b, _, _ = compat_plan(2.4e6, 5000, _hip.TETRA_CF32, cache=False)
    assert a is compat_plan(2.4e6, 5000, _hip.TETRA_CF32)[0] and b is not a
    taps = np.ctypeslib.as_array(a.b)[:5].copy()
    b.b[0] = 123.0
    assert np.array_equal(np.ctypeslib.as_array(compat_plan(2.4e6, 5000, _hip.TETRA_CF32)[0].b)[:5], taps)


def test_mode_selection_from_environment(monkeypatch):
    """TETRAEAR_DEMOD picks the chain for callers that construct SignalProcessor / TetraDecoder as
    the reference's GUI and scanner do (modern.py:1886-1887, scanner.py:164-172); an explicit mode=
    wins; TETRAEAR_BACKEND other than hip is refused (no CPU path in this build)."""
    from tetraear import _hip
    from tetraear.signal import SignalProcessor
    from tetraear.core import TetraDecoder
    monkeypatch.delenv("TETRAEAR_DEMOD", raising=False)
    assert SignalProcessor(sample_rate=2.4e6).mode == "compat"
    assert TetraDecoder(auto_decrypt=False).mode == "compat"
    monkeypatch.setenv("TETRAEAR_DEMOD", "etsi")
    assert SignalProcessor(sample_rate=2.4e6).mode == "etsi"
    assert TetraDecoder(auto_decrypt=False).mode == "etsi"
    assert SignalProcessor(2.4e6, mode="compat").mode == "compat"
    monkeypatch.setenv("TETRAEAR_DEMOD", "fast")
    with pytest.raises(ValueError):
        SignalProcessor()
    monkeypatch.setenv("TETRAEAR_DEMOD", "compat")
    monkeypatch.setenv("TETRAEAR_BACKEND", "cpu")
    with pytest.raises(_hip.TetraHipError):
        TetraDecoder()


def test_mac_batch_rejects_bad_frames_after_applying_earlier_ones(monkeypatch):
    """parse_mac_pdu_batch: a frame that is not integer 0/1 (bool arrays included, which the
    reference's int(..., 2) rejects) raises ValueError after the frames before it were applied."""
    from tetraear.core.protocol import TetraProtocolParser
    p = TetraProtocolParser()
    seen = []
    monkeypatch.setattr(TetraProtocolParser, "_mac_batch", lambda self, rows: seen.append(len(rows)) or [])
    good = np.zeros(40, np.int64)
    with pytest.raises(ValueError):
        p.parse_mac_pdu_batch([good, good, np.zeros(40, bool), good])
    with pytest.raises(ValueError):
        p.parse_mac_pdu_batch([good, np.full(40, 2)])
    assert seen == [2, 1]
    assert p.parse_mac_pdu_batch([np.zeros(5, bool)]) == []   # < 8 bits: None without a check
