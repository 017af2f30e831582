"""CPU: pin the ETSI oracle (no reference counterpart exists -- parity unpinned vs reference).

Known answers + encoder->decoder round trips + full IQ round trips through the oracle receiver."""
import numpy as np
import pytest

import etsi as E


def test_crc16_known_answers():
    kat = np.array([(x >> (7 - k)) & 1 for x in b"123456789" for k in range(8)], np.uint8)
    assert E.crc16_reg(kat) == 0x29B1                 # CCITT-FALSE register
    assert E.crc16_reg(kat) ^ 0xFFFF == 0xD64E        # ones' complement (CRC-16/GENIBUS check value)
    c = E.crc16_reg(kat) ^ 0xFFFF
    full = np.concatenate([kat, [(c >> (15 - k)) & 1 for k in range(16)]]).astype(np.uint8)
    assert E.crc16_reg(full) == 0x1D0F                # residue of a valid codeword


def test_scrambler_properties():
    assert E.scramble_init(0, 0, 0) == 3               # BSCH: colour code 0 with the two leading 1s
    s = E.scramble_seq(E.scramble_init(262, 1, 5), 4096)
    assert 0.45 < s.mean() < 0.55
    assert not np.array_equal(s[:432], E.scramble_seq(E.scramble_init(262, 1, 6), 432))


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_block_round_trip_with_errors(kind):
    rng = np.random.default_rng(kind)
    K, a, n2, n1 = E.KIND_PARAMS[kind]
    scr = E.scramble_seq(E.scramble_init(901, 77, 12) if kind != 2 else 3, K)
    good = 0
    for trial in range(30):
        t1 = rng.integers(0, 2, n1).astype(np.uint8)
        t5 = E.encode_block(t1, kind, scr)
        soft = np.where(t5 == 0, 40, -40).astype(np.int8)
        dec, ok = E.Receiver.decode_block(soft, kind, scr)
        assert ok and np.array_equal(dec, t1)          # error-free codeword decodes exactly
        flip = rng.choice(K, int(0.01 * K), replace=False)
        soft[flip] = -soft[flip]
        dec, ok = E.Receiver.decode_block(soft, kind, scr)
        good += ok and np.array_equal(dec, t1)
    assert good >= 27                                   # ~1 % hard errors: nearly always corrected
    fails = 0
    for trial in range(30):   # noise must (almost always) fail the CRC
        garbage = rng.integers(-60, 61, K).astype(np.int8)
        fails += not E.Receiver.decode_block(garbage, kind, scr)[1]
    assert fails >= 29


@pytest.mark.parametrize("snr", [None, 15.0])
def test_iq_round_trip(snr):
    rng = np.random.default_rng(11)
    cell = E.scramble_init(262, 1, 5)
    bits, jobs = E.burst_stream(rng, 6, E.scramble_seq(cell))
    rx = E.Receiver()
    for t0 in (3.0, 3.41, 5.9):
        x = E.modulate(bits, 131072, t0=t0, phase0=rng.uniform(0, 6.28), cfo=rng.uniform(-600, 600),
                       snr_db=snr, rng=rng)
        sym, soft, hard, diag = rx.demod(x)
        assert 960 < len(sym) < 990
        res = rx.lower_mac(soft, hard, cell)
        assert len(res) >= 2
        sent = [tuple(t) for _, jj in jobs for _, t in jj]
        for _, _, dec in res:
            for kind, t1, ok in dec:
                assert ok and tuple(t1) in sent


# the reference CLI's rates: -s in MHz, the GUI slider 1.8-2.4 MHz in 0.1 MHz steps
# (/root/reference/tetraear/ui/modern.py:5518-5519, 5630-5638)
CLI_RATES = [1.8e6, 1.9e6, 2.0e6, 2.1e6, 2.2e6, 2.3e6, 2.4e6]


@pytest.mark.parametrize("fs", CLI_RATES)
def test_iq_round_trip_every_cli_rate(fs):
    """The oracle receiver at each rate the reference's callers use: a 54.6 ms chunk (131072 samples
    at 2.4 MSps, the same air time at the other rates) decodes every burst it holds, each block
    CRC-good and a transmitted payload, with ~983 symbols out."""
    rng = np.random.default_rng(int(fs) // 1000)
    cell = E.scramble_init(262, 1, 5)
    bits, jobs = E.burst_stream(rng, 6, E.scramble_seq(cell))
    rx = E.Receiver(fs)
    n = int(round(131072 * fs / 2.4e6))
    x = E.modulate(bits, n, fs=fs, t0=3.37, phase0=rng.uniform(0, 6.28), cfo=rng.uniform(-600, 600), snr_db=20.0,
                   rng=rng)
    sym, soft, hard, diag = rx.demod(x)
    assert 960 < len(sym) < 990, len(sym)
    res = rx.lower_mac(soft, hard, cell)
    assert len(res) >= 2
    sent = [tuple(t) for _, jj in jobs for _, t in jj]
    for _, _, dec in res:
        for kind, t1, ok in dec:
            assert ok and tuple(t1) in sent


def test_rate_plans_match_host_design():
    """The host planner (tetraear.signal.etsi.rate_design / etsi_plan) equals the oracle's design at
    every CLI rate and a few others: the same q1, L1, up / down, Lp and bit-identical taps; 2.4 MSps
    is the canonical plan; 20 MSps (the wideband capture) has no single-channel plan."""
    from tetraear.signal.etsi import etsi_plan, rate_design
    for fs in CLI_RATES + [1.0e6, 240e3, 300e3]:
        d = E.design(fs)
        p = etsi_plan(fs)
        assert (p.q1, p.L1, p.up, p.down, p.Lp) == (d["q1"], d["L1"], d["up"], d["down"], d["Lp"]), fs
        assert np.array_equal(np.ctypeslib.as_array(p.h1)[:p.L1], d["h1"]), fs
        assert np.array_equal(np.ctypeslib.as_array(p.hp)[:p.Lp], d["hp"]), fs
        assert 72000 * p.q1 * p.down == int(fs) * p.up   # exactly 72 kHz out
    assert rate_design(2.4e6) == (10, 48, 3, 10, 321)
    with pytest.raises(ValueError):
        rate_design(20e6)
    with pytest.raises(ValueError):
        E.design(20e6)


def test_rate_design_invariants():
    """Every rate from 0.1 to 5 MSps in 0.1 MHz steps either gets a plan inside the generic kernel's
    limits (q1 <= 13, L1 <= 64, Lp <= 4096, < 254 taps per stage-2 output, 72 kHz out exactly,
    fs1 >= 180 kHz unless q1 = 1) or raises ValueError -- never a plan the library would refuse."""
    from tetraear.signal.etsi import rate_design
    served = 0
    for k in range(1, 51):
        fs = k * 100e3
        try:
            q1, L1, up, down, Lp = rate_design(fs)
        except ValueError:
            continue
        served += 1
        assert 1 <= q1 <= 13 and 1 <= L1 <= 64 and Lp == 32 * down + 1 <= 4096 and (Lp - 1) // up + 2 < 254, fs
        assert 72000 * q1 * down == int(fs) * up, fs
        assert q1 == 1 or fs / q1 >= 180e3, fs
    assert served >= 40


@pytest.mark.parametrize("fs", [1.0e6, 500e3])
def test_iq_round_trip_other_rates(fs):
    """The oracle receiver at rates outside the GUI slider (1.0 MSps: q1 = 5, 9/25; 500 kSps: q1 = 2)."""
    rng = np.random.default_rng(int(fs) // 1000 + 7)
    cell = E.scramble_init(901, 77, 12)
    bits, jobs = E.burst_stream(rng, 6, E.scramble_seq(cell))
    rx = E.Receiver(fs)
    n = int(round(131072 * fs / 2.4e6))
    x = E.modulate(bits, n, fs=fs, t0=4.1, phase0=rng.uniform(0, 6.28), cfo=rng.uniform(-600, 600), snr_db=20.0,
                   rng=rng)
    sym, soft, hard, diag = rx.demod(x)
    res = rx.lower_mac(soft, hard, cell)
    sent = [tuple(t) for _, jj in jobs for _, t in jj]
    assert len(res) >= 2 and all(ok and tuple(t1) in sent for _, _, dec in res for _, t1, ok in dec)


def test_timing_with_given_class_sums_equals_quarter_order():
    """eo_timing_om with the quarter-order class sums handed in is eo_timing (the O-M split is a pure
    refactor), and the wideband grouped order gives the same class sums to float rounding."""
    rng = np.random.default_rng(7)
    ora = E.Receiver()
    bits = rng.integers(0, 2, 2 * 1200).astype(np.uint8)
    y = E.modulate(bits, 4 * 1100, fs=72000.0, t0=0.37, cfo=40.0, snr_db=15.0, rng=rng)
    a = ora.timing(y)
    b = ora.timing(y, om=ora.om_quarters(y))
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    p = np.abs(y.astype(np.complex128)) ** 2
    exact = np.array([p[c::4].sum() for c in range(4)])
    for U in (4, 36, 64):
        A = ora.om_grouped(y, 0, len(y), U)
        assert np.allclose(A, exact, rtol=2e-6), U
    assert np.allclose(ora.om_quarters(y), exact, rtol=2e-6)


@pytest.mark.parametrize("s,M2,U", [(0, 3932, 36), (3932, 3932, 36), (7864, 3932, 36), (36, 1000, 36),
                                    (8, 24, 36), (4, 60, 36), (40, 8000, 36), (0, 512, 4), (12, 4096, 64)])
def test_grouped_class_sums_cover_each_sample_once(s, M2, U):
    """The grouped order (head, whole groups, tail) counts every sample of row[s, s + M2) exactly
    once in its class: with integer-valued powers the sums are exact in float32."""
    rng = np.random.default_rng(s + M2 + U)
    n = s + M2 + 2 * U
    row = (rng.integers(0, 8, n) + 1j * rng.integers(0, 8, n)).astype(np.complex64)
    A = E.Receiver.om_grouped(row, s, M2, U)
    p = np.abs(row[s:s + M2].astype(np.complex128)) ** 2
    assert np.array_equal(A, np.array([p[c::4].sum() for c in range(4)], np.float32))
