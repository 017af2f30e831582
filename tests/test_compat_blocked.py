"""The compat chain's time-blocked decimator (latency mode; compat_demod.hip k_sosb_*, oracle/compat.py:
decimate_blocked) against the reference's own fixtures, on the CPU.

The blocked form is not scipy's operation order, so it cannot be bit-exact with the reference; the
bar it was held to in round 5 is: on every G1 case it would serve, .symbols within
1e-5 of the reference's and no hard decision different outside a 1e-6 rad band around the decision
thresholds.  The G1 fixtures meet it; a wider sweep does not (1.45e-5 and 3 flips in 1.61 M
symbols, tests/test_compat_default_form.py), so since round 6 the latency form is opt-in only
(decimator="blocked", TETRA_COMPAT_BLOCKED) and these tests pin what it computes, not a default.
The one G1 case at q = 83 (20 MSps), where the cheby1 band is narrow enough for the noise to reach
5.7e-5, is outside its limits (the product refuses it there) -- checked here too, so the limit is
measured, not assumed."""
import numpy as np
import pytest

import compat as O
from conftest import iq_to_c64

DELTA = 1e-6
THR = np.array([-5, -3, 3, 5]) * np.pi / 8


def band(symbols):
    """Positions whose differential phase (processor.py:124-161, normalised) is within DELTA of a
    threshold or of +-pi."""
    if len(symbols) < 2:
        return np.zeros(0, bool)
    s = np.asarray(symbols, np.complex128)
    s = s / np.max(np.abs(s))
    ph = np.angle(s[1:] * np.conj(s[:-1]))
    return (np.min(np.abs(ph[:, None] - THR[None, :]), axis=1) < DELTA) | (np.abs(np.abs(ph) - np.pi) < DELTA)


def test_blocked_oracle_within_the_fp32_noise_of_the_reference(g1):
    z, meta = g1
    served = ties = 0
    worst = 0.0
    outside = []
    for i, m in enumerate(meta):
        x = iq_to_c64(z[f"c{i}_iq"])
        q = int(m["q"])
        if not m["dec_ok"] or q < 2:
            continue
        if "sweep" in m:   # round 6: the reference's outputs on the sweep chunks the bar fails on
            p = O.SignalProcessor(m["fs"], decimator="blocked")
            hard = p.process(x, m["freq_offset"])
            err = float(np.max(np.abs(p.symbols - z[f"c{i}_symbols"])))
            flips = int(np.sum(hard != z[f"c{i}_hard"]))
            if err > 1e-5 or flips:
                outside.append((tuple(m["sweep"]), err, flips))
            continue
        p = O.SignalProcessor(m["fs"], decimator="blocked")
        hard = p.process(x, m["freq_offset"])
        want, wh = z[f"c{i}_symbols"], z[f"c{i}_hard"]
        assert p.symbols.dtype == want.dtype and p.symbols.shape == want.shape, (i, m)
        err = np.max(np.abs(p.symbols - want)) if len(want) else 0.0
        nb = band(want)
        bad = (hard != wh) & ~nb[:len(hard)]
        if O.blocked_fits(1, len(x), q):
            served += 1
            worst = max(worst, err)
            assert err <= 1e-5, (i, m, err)
            assert not bad.any(), (i, m, int(bad.sum()))
            ties += int(nb.sum())
        else:
            assert q > O.SB_MAXQ and err > 1e-5, (i, m, err)   # the measured reason for the limit
    print(f"blocked decimator: {served} G1 cases served, worst |d symbols| {worst:.2e}, {ties} tie-band positions; "
          f"outside the bar on the reference's sweep chunks: {outside}")
    assert served >= 20 and worst < 5e-6
    # why the latency form is opt-in only: against the reference itself it leaves the bar on three
    # GUI chunks of the round-6 sweep (a flip at symbol 817 / 867, 1.008e-5 on .symbols)
    assert {o[0] for o in outside} >= {(0, 2), (28, 15), (33, 13)}, outside


def test_library_table_equals_the_oracle_table():
    """tetra_compat_blocked_table (host code of the product, no GPU needed) equals the oracle's
    restatement bit for bit, complex64 and complex128 designs, the CLI decimation factors."""
    from tetraear import _hip
    from tetraear.signal.processor import compat_plan
    lib = _hip.lib()
    for fs in (1.0e6, 1.8e6, 2.0e6, 2.4e6, 3.2e6):
        for fmt in (_hip.TETRA_CF32, _hip.TETRA_CF64):
            plan, _, _ = compat_plan(fs, 131072, fmt)
            got = np.zeros(O.SB_NPOW * 64)
            assert lib.tetra_compat_blocked_table(plan, int(fmt == _hip.TETRA_CF64), _hip.ptr(got)) == 0
            coef = np.array(plan.sos_f64[:] if fmt == _hip.TETRA_CF64 else plan.sos_f32[:],
                            np.float64 if fmt == _hip.TETRA_CF64 else np.float32)
            want = O.blocked_table(coef).ravel()
            assert np.array_equal(got, want), (fs, fmt)
            assert np.all(np.isfinite(got)) and np.max(np.abs(want[-64:])) < 1.0   # Phi^512: decayed


@pytest.mark.parametrize("n", [28, 255, 256, 257, 4096 + 17])
def test_blocked_edges_against_sequential(n):
    """Short rows (one tile, a tile plus one sample, the odd-pad minimum N = 28): blocked equals
    sequential exactly on a single tile (tile 0 starts from scipy's own state), and stays within the
    fp32 noise across tiles."""
    rng = np.random.default_rng(n)
    x = (0.3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    a, b = O.decimate(x, 10), O.decimate_blocked(x, 10)
    assert a.dtype == b.dtype and a.shape == b.shape
    if n + 54 <= O.SB_B:
        assert np.array_equal(a, b)
    else:
        assert np.max(np.abs(a - b)) <= 1e-5 * np.max(np.abs(a))


def test_blocked_chain_within_float64_rounding_of_filtfilt(g1):
    """The latency mode's whole chain (oracle, decimator="blocked" within its limits as the product
    runs it): time-blocked decimate where it fits and time-blocked filtfilt, against the reference fixtures --
    the filtfilt part is float64, so with a sequential decimator (the 20 MSps case) it stays within
    1e-12 of the reference; every served case within 1e-5 and no decision off outside the band."""
    z, meta = g1
    n = 0
    for i, m in enumerate(meta):
        if "sweep" in m:
            continue   # outside the bar by construction (previous test)
        x = iq_to_c64(z[f"c{i}_iq"])
        fits = m["dec_ok"] and m["q"] >= 2 and O.blocked_fits(1, len(x), m["q"])
        p = O.SignalProcessor(m["fs"], decimator="blocked" if fits or not m["dec_ok"] or m["q"] < 2 else "sequential")
        hard = p.process(x, m["freq_offset"])
        want, wh = z[f"c{i}_symbols"], z[f"c{i}_hard"]
        assert p.symbols.dtype == want.dtype and p.symbols.shape == want.shape, (i, m)
        if not len(want):
            continue
        err = np.max(np.abs(p.symbols - want))
        dec_blocked = m["dec_ok"] and m["q"] >= 2 and O.blocked_fits(1, len(x), m["q"])
        assert err <= (1e-5 if dec_blocked else 1e-12 * max(1.0, np.max(np.abs(want)))), (i, m, err)
        bad = (hard != wh) & ~band(want)[:len(hard)]
        assert not bad.any(), (i, m)
        n += 1
    assert n >= 25


def test_library_lfilter_table_equals_the_oracle_table():
    from tetraear import _hip
    from tetraear.signal.processor import compat_plan
    for fs in (1.8e6, 2.4e6, 240000.0, 1.0e6):
        plan, _, _ = compat_plan(fs, 131072, _hip.TETRA_CF32)
        want = O.lfilter_table(np.array(plan.b[:5]), np.array(plan.a[:5]))
        got = np.zeros(O.SB_NPOW * 16)
        assert _hip.lib().tetra_compat_blocked_table(plan, 2, _hip.ptr(got)) == 0
        assert np.array_equal(got, want.ravel()), fs
        assert np.all(np.isfinite(want)) and np.max(np.abs(want[-1])) < 1.0
