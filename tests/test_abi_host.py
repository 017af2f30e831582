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
    assert lib.tetra_abi_version() == 1


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
