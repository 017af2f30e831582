"""GPU parity of the compat path: HIP (through the C ABI) vs golden vectors and the oracle.

Bar (BASELINE.json north_star): integer outputs bit-exact; soft symbols within 1e-5.  Hard
decisions are compared bit-exact outside a tie band of 1e-9 rad around the decision thresholds
(atan2 differs between libms by an ulp); positions in the band are counted and reported.
"""
import numpy as np
import pytest

import compat as O
from conftest import decoded_view, iq_to_c64

pytestmark = pytest.mark.gpu

SOFT_TOL = 1e-5
TIE = 1e-9


@pytest.fixture(scope="module")
def hip():
    from tetraear import _hip
    c = _hip.ctx()
    assert c.arch().startswith("gfx950")
    return c


def _tie_mask(symbols):
    """Positions whose differential phase lies within TIE of a decision threshold."""
    if len(symbols) < 2:
        return np.zeros(0, bool)
    s = np.asarray(symbols, np.complex128)
    d = s[1:] * np.conj(s[:-1])
    ph = np.angle(d)
    thr = np.array([-5, -3, 3, 5]) * np.pi / 8
    return np.min(np.abs(ph[:, None] - thr[None, :]), axis=1) < TIE


def _hard_equal(got, want, symbols):
    assert len(got) == len(want)
    tie = _tie_mask(symbols)
    bad = (got != want) & ~tie[:len(got)]
    assert not bad.any(), f"{int(bad.sum())} hard mismatches outside the tie band"
    return int(tie.sum())


def test_process_matches_golden(hip, g1):
    """The DEFAULT process() -- what the GUI's unchanged call (modern.py:2029) gets, one chunk at a
    time -- against the reference's own outputs, including the round-6 sweep chunks on which the
    opt-in time-blocked decimator leaves the bar (make_golden.py: SWEEP_CASES): soft symbols within
    1e-5 (measured: bit-exact but for the mixer's sin/cos ulps) and every hard decision equal -- no
    tie band."""
    from tetraear.signal import SignalProcessor
    z, meta = g1
    ties = worst = 0
    for i, m in enumerate(meta):
        x = iq_to_c64(z[f"c{i}_iq"])
        p = SignalProcessor(m["fs"])
        hard = p.process(x, m["freq_offset"])
        want_sym = z[f"c{i}_symbols"]
        assert p.symbols.dtype == want_sym.dtype, (i, m)
        assert p.symbols.shape == want_sym.shape, (i, m)
        if len(want_sym):
            err = np.max(np.abs(p.symbols - want_sym))
            worst = max(worst, err)
            assert err <= SOFT_TOL * max(1.0, np.max(np.abs(want_sym))), (i, m)
            if not m["freq_offset"]:
                assert np.array_equal(p.symbols, want_sym), (i, m)   # no libm on the path: bit-exact
        ties += _hard_equal(hard, z[f"c{i}_hard"], want_sym)
        assert np.array_equal(hard, z[f"c{i}_hard"]), (i, m, int(np.sum(hard != z[f"c{i}_hard"])))
    print(f"{len(meta)} cases, worst |d symbols| {worst:.3g}, tie-band positions: {ties}")


def test_intermediates(hip, g1):
    from tetraear.signal import SignalProcessor
    from tetraear.signal.processor import compat_plan
    from tetraear import _hip
    z, meta = g1
    for i, m in enumerate(meta):
        if not m["dec_ok"] or m["n"] == 0:
            continue
        x = iq_to_c64(z[f"c{i}_iq"])
        plan, M, rate = compat_plan(m["fs"], len(x), _hip.TETRA_CF32)
        out = np.empty(M, np.complex64)
        hip.check(hip.lib.tetra_decimate(hip.handle, plan, _hip.ptr(x), _hip.TETRA_CF32, 1, len(x), _hip.ptr(out)))
        assert np.array_equal(out, z[f"c{i}_decimated"]), (i, m)   # float32 IIR restated exactly
        if f"c{i}_filtered" in z.files:
            p = SignalProcessor(m["fs"])
            sh = z[f"c{i}_shifted"]
            if m["freq_offset"]:
                got = p.frequency_shift(z[f"c{i}_decimated"], m["freq_offset"], rate)
                assert np.max(np.abs(got - sh)) < 1e-12, (i, m)
            f = p.filter_signal(sh, 25000, rate)
            want = z[f"c{i}_filtered"]
            assert f.dtype == want.dtype
            if m["freq_offset"]:
                assert np.max(np.abs(f - want)) < 1e-9, (i, m)
            else:
                assert np.array_equal(f, want), (i, m)   # no libm in the path: bit-exact


def test_direct_method_calls(hip, g1):
    from tetraear.signal import SignalProcessor
    z, _ = g1
    p = SignalProcessor()
    x = z["direct_x128"]
    assert np.array_equal(p.filter_signal(x, bandwidth=25000), z["direct_filter_25k"])
    assert np.array_equal(p.filter_signal(x, bandwidth=50000), z["direct_filter_50k"])
    _hard_equal(p.demodulate_dqpsk(x), z["direct_demod"], x)
    assert np.array_equal(p.extract_symbols(x), z["direct_extract"])
    assert np.array_equal(p.extract_symbols(x, sample_rate=1.0e6), z["direct_extract_1M"])
    assert np.max(np.abs(p.frequency_shift(x, 1000) - z["direct_shift_1k"])) < 1e-12
    assert len(p.demodulate_dqpsk(np.array([]))) == 0
    assert len(p.demodulate_dqpsk(np.array([1.0 + 1.0j]))) == 0
    assert len(p.extract_symbols(np.array([]))) == 0
    assert len(p.filter_signal(np.array([]))) == 0


@pytest.mark.parametrize("decimator", ["sequential", "auto"])
def test_real_input_and_direct_calls_before_process(hip, decimator):
    """Real float32 chunks at 1.8 MSps (q = 7, where decimate's float32 and complex64 initial
    states differ in a last bit) equal the oracle's -- after filter_signal ran on a chunk of the same
    length and rate (it must not leave its taps in the plan process() reuses)."""
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(77)
    x = (0.4 * rng.standard_normal(22849)).astype(np.float32)
    p = SignalProcessor(1.8e6, decimator=decimator)
    p.filter_signal(x)   # 1.8 MSps taps, same chunk length as the process() call below
    h = p.process(x)
    o = O.SignalProcessor(1.8e6, decimator=decimator)
    ho = o.process(x)
    assert p.symbols.dtype == o.symbols.dtype and len(p.symbols) == len(o.symbols)
    assert np.max(np.abs(p.symbols - o.symbols)) <= SOFT_TOL
    _hard_equal(h, ho, o.symbols)


def test_process_batch_equals_per_channel(hip):
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(3)
    C, N = 12, 16384
    x = (0.3 * (rng.standard_normal((C, N)) + 1j * rng.standard_normal((C, N)))).astype(np.complex64)
    fo = (np.arange(C) - 6) * 1171.875
    p = SignalProcessor(2.4e6)
    hard, soft, ns = p.process_batch(x, fo)
    for c in range(C):
        h = p.process(x[c], fo[c])
        assert ns[c] == len(p.symbols)
        assert np.array_equal(hard[c, :ns[c] - 1], h)
        assert np.array_equal(soft[c, :ns[c]], p.symbols)


@pytest.mark.parametrize("decimator", ["sequential", "blocked"])
@pytest.mark.parametrize("N", [16383, 131071])
def test_odd_length_rows_vs_oracle(hip, N, decimator):
    """Odd-length complex64 rows in a multi-channel batch (row starts only 8-byte aligned): the
    banked sequential decimator and the latency mode's time-blocked one, each equal to its oracle
    for every channel."""
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(N)
    C = 5
    x = (0.3 * (rng.standard_normal((C, N)) + 1j * rng.standard_normal((C, N)))).astype(np.complex64)
    fo = [0.0, 1171.875, -2343.75, 0.0, 3515.625]
    hard, soft, ns = SignalProcessor(2.4e6, decimator=decimator).process_batch(x, fo)
    for c in range(C):
        o = O.SignalProcessor(2.4e6, decimator=decimator)
        h = o.process(x[c], fo[c])
        assert ns[c] == len(o.symbols)
        assert np.max(np.abs(soft[c, :ns[c]] - o.symbols)) <= SOFT_TOL
        _hard_equal(hard[c, :ns[c] - 1], h, o.symbols)


@pytest.mark.parametrize("decimator", ["sequential", "blocked"])
def test_full_size_batch_vs_oracle(hip, decimator):
    """131072-sample GUI chunks (modern.py:1919) over a channel batch, spot-checked vs the oracle,
    in both decimator forms."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import _signals
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(99)
    C, N = 8, 131072
    xs, fo = [], []
    for c in range(C):
        x, _ = _signals.family("tetra" if c % 2 == 0 else "noise", rng, N, 2.4e6)
        xs.append(x)
        fo.append((c - 4) * 1171.875 * (c % 3 != 0))
    x = np.stack(xs)
    p = SignalProcessor(2.4e6, decimator=decimator)
    hard, soft, ns = p.process_batch(x, fo)
    for c in (0, 3, 7):
        o = O.SignalProcessor(2.4e6, decimator=decimator)
        h = o.process(x[c], fo[c])
        assert ns[c] == len(o.symbols)
        assert np.max(np.abs(soft[c, :ns[c]] - o.symbols)) <= SOFT_TOL
        _hard_equal(hard[c, :ns[c] - 1], h, o.symbols)


def test_latency_mode_long_chunk_vs_oracle(hip):
    """One channel of 520000 samples through the default form: past k_extract_lat's 3584 symbols
    per phase (k_extract over the |y|^2 prepass serves it) -- equal to the oracle."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import _signals
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(520)
    x, _ = _signals.family("tetra", rng, 520000, 2.4e6)
    p = SignalProcessor(2.4e6)
    h = p.process(x, 1171.875)
    o = O.SignalProcessor(2.4e6, decimator="sequential")
    ho = o.process(x, 1171.875)
    assert len(p.symbols) == len(o.symbols) > 3584
    assert np.max(np.abs(p.symbols - o.symbols)) <= SOFT_TOL
    _hard_equal(h, ho, o.symbols)


def test_decoder_matches_golden(hip, g2):
    from tetraear.core import TetraDecoder
    z, recs = g2
    for i, r in enumerate(recs):
        sym = z[f"s{i}_sym"]
        d = TetraDecoder(auto_decrypt=False)
        bits, mapped = d.symbols_to_bits(sym)
        assert np.array_equal(bits, z[f"s{i}_bits"]) and np.array_equal(mapped, z[f"s{i}_mapped"]), i
        for thr in (0.9, 0.85, 0.8, 0.75, 0.7):
            pos, mc = d.find_sync(bits, threshold=thr, return_max_corr=True)
            assert pos == r[f"fs_{thr}"][0] and mc == r[f"fs_{thr}"][1], (i, thr)
        frames = d.decode(sym)
        # decode() == the reference's frame list: the MAC PDU stage drops CRC-failed slots without
        # a MAC PDU and settles mac_pdu / encrypted / encryption_algorithm (decoder.py:994-1100)
        assert [decoded_view(f) for f in frames] == [decoded_view(g) for g in r["decoded"]], i
        st = d.protocol_parser.stats
        for k in ("total_bursts", "crc_pass", "crc_fail", "clear_mode_frames", "encrypted_frames"):
            assert st[k] == r["stats"][k], (i, k)


def test_decode_batch_equals_single(hip, g2):
    """decode_batch over all g2 streams == consecutive decode() calls on one decoder (the parser's
    fragment buffer / SYSINFO state and statistics carry across streams in both)."""
    from tetraear.core import TetraDecoder
    z, recs = g2
    streams = [z[f"s{i}_sym"] for i in range(len(recs))]
    d = TetraDecoder(auto_decrypt=False)
    batch = d.decode_batch(streams)
    seq = TetraDecoder(auto_decrypt=False)
    for s, fb in zip(streams, batch):
        assert [decoded_view(f) for f in fb] == [decoded_view(f) for f in seq.decode(s)]
    assert d.protocol_parser.stats == seq.protocol_parser.stats
    assert (d.protocol_parser.mcc, d.protocol_parser.mnc, d.protocol_parser.colour_code) == \
        (seq.protocol_parser.mcc, seq.protocol_parser.mnc, seq.protocol_parser.colour_code)


def test_parser_matches_golden(hip, g3):
    from tetraear.core import TetraProtocolParser, BurstType
    z = g3
    p = TetraProtocolParser()
    kat = np.array([(b >> (7 - k)) & 1 for b in b"123456789" for k in range(8)])
    assert int("".join(map(str, p._calculate_crc16(kat))), 2) == 0x29B1
    for v, c, ok in zip(z["crc_vecs"], z["crc_of_vecs"], z["check_crc"]):
        assert np.array_equal(p._calculate_crc16(v), c)
        assert p._check_crc(v) == bool(ok)
    for v, ok in zip(z["crc510_vecs"], z["check510"]):
        assert p._check_crc(v) == bool(ok)
    for n, ok in enumerate(z["crc_short"]):
        assert p._check_crc(np.ones(n, int)) == bool(ok)
    q = TetraProtocolParser()
    for s, L, t, ts, d, ok in zip(z["burst_syms"], z["burst_len"], z["burst_type"], z["burst_ts"],
                                  z["burst_data"], z["burst_crc_ok"]):
        b = q.parse_burst(s[:L], slot_number=1)
        assert b.burst_type.value == t and b.crc_ok == bool(ok)
        assert np.array_equal(b.training_sequence, ts[ts != 255])
        assert np.array_equal(b.data_bits, d[d != 255])
    st = q.stats
    assert [st["total_bursts"], st["crc_pass"], st["crc_fail"]] == list(z["burst_stats"])
    assert q.parse_burst(np.zeros(100, int)) is None
    assert q._check_sync_pattern(np.array(q.SYNC_CONTINUOUS_DOWNLINK)) is True
    assert q._check_sync_pattern(np.zeros(22, int)) is False
    assert isinstance(q._detect_burst_type(np.zeros(255, int)), BurstType)


def test_bench_compat_pipeline_matches_serial(hip):
    """bench.py --chain compat: the two-stream pipeline (consecutive batches' whole chains on two
    contexts / streams) gives every batch the serial chain's results."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    C, N = 64, 131072
    iq = torch.round(0.25 * torch.randn((C, N, 2), generator=g, device=dev) * 32768) / 32768
    ser = bench.CompatStep(_hip_ctx_on_torch_stream(), iq, C, N)
    ser()
    torch.cuda.synchronize(dev)
    want = [t.clone() for t in (ser.nsym, ser.hard, ser.soft, ser.nsync, ser.rec)]
    pip = bench.CompatStep(_hip_ctx_on_torch_stream(), iq, C, N).pipeline()
    for _ in range(3):
        pip()
    torch.cuda.synchronize(dev)
    for ln in pip.lanes:
        got = (ln.nsym, ln.hard, ln.soft, ln.nsync, ln.rec)
        ns = want[0]
        assert torch.equal(got[0], ns) and torch.equal(got[3], want[3])
        for ch in range(C):
            n = int(ns[ch])
            assert torch.equal(got[1][ch, :n - 1], want[1][ch, :n - 1])
            assert torch.equal(got[2][ch, :n], want[2][ch, :n])
            k = int(want[3][ch])
            assert torch.equal(got[4][ch, :k], want[4][ch, :k])


def _hip_ctx_on_torch_stream():
    import ctypes
    import torch
    from tetraear import _hip
    c = _hip.Context()
    s = torch.cuda.current_stream(torch.device("cuda", 0))
    c.check(c.lib.tetra_set_stream(c.handle, ctypes.c_void_p(s.cuda_stream)), "set_stream")
    return c


def test_lmac_packed_equals_global_rows(hip, g2):
    """tetra_lmac_compat packs each stream's bits into LDS when the row fits (k_lmac: PackedStream)
    and reads symbols from global memory otherwise (Stream).  The same g2 streams through both --
    a tight row stride, then one past the LDS cap (LMAC_LDS_MAX, 48 KB of packed bits) -- give the
    same syncs, records and burst bits."""
    from tetraear import _hip
    from tetraear.core.decoder import cascade_table
    z, recs = g2
    streams = [np.asarray(z[f"s{i}_sym"], np.int64) for i in range(len(recs))]
    C = len(streams)
    c = _hip.ctx()
    out = []
    for stride in (max(len(s) for s in streams), 200_000):
        sym = np.zeros((C, stride), np.int64)
        for i, s in enumerate(streams):
            sym[i, :len(s)] = s
        ns = np.array([len(s) for s in streams], np.int32)
        nsync = np.zeros(C, np.int32)
        rec = np.zeros((C, _hip.MAX_SYNC, _hip.F_FIELDS), np.int32)
        fb = np.zeros((C, _hip.MAX_SYNC, 510), np.uint8)
        bb = np.zeros((C, _hip.MAX_SYNC, 510), np.uint8)
        c.check(c.lib.tetra_lmac_compat(c.handle, _hip.ptr(sym), _hip.ptr(ns), C, stride, _hip.ptr(cascade_table()),
                                        _hip.ptr(nsync), _hip.ptr(rec), _hip.ptr(fb), _hip.ptr(bb)), "tetra_lmac_compat")
        out.append((nsync, rec, fb, bb))
    (n1, r1, f1, b1), (n2, r2, f2, b2) = out
    assert np.array_equal(n1, n2) and n1.sum() > 0
    for i in range(C):
        k = int(n1[i])
        assert np.array_equal(r1[i, :k], r2[i, :k])
        assert np.array_equal(f1[i, :k], f2[i, :k]) and np.array_equal(b1[i, :k], b2[i, :k])


def test_blocked_decimator_equals_its_oracle(hip, g1):
    """The opt-in latency mode (decimator="blocked": time-blocked decimator and filtfilt, C <= 64,
    q <= 16).  Every G1 case it serves equals the oracle's restatement of that form
    (oracle/compat.py: decimate_blocked): hard symbols exactly, .symbols exactly without a mixer and
    within 1e-12 with one (device sin/cos ulps) -- including the round-6 sweep chunks, where that
    form is off the reference (tests/test_compat_blocked.py).  The default / "sequential" form is
    the scipy-exact one on the same call."""
    from tetraear.signal import SignalProcessor
    z, meta = g1
    served = 0
    for i, m in enumerate(meta):
        x = iq_to_c64(z[f"c{i}_iq"])
        if not m["dec_ok"] or m["q"] < 2 or not O.blocked_fits(1, len(x), m["q"]):
            continue
        p = SignalProcessor(m["fs"], decimator="blocked")
        hard = p.process(x, m["freq_offset"])
        o = O.SignalProcessor(m["fs"], decimator="blocked")
        want = o.process(x, m["freq_offset"])
        assert np.array_equal(hard, want), (i, m)
        tol = 0.0 if m["freq_offset"] == 0 else 1e-12
        assert p.symbols.shape == o.symbols.shape, (i, m)
        assert not len(o.symbols) or np.max(np.abs(p.symbols - o.symbols)) <= tol, (i, m)
        ps = SignalProcessor(m["fs"], decimator="sequential")
        hs = ps.process(x, m["freq_offset"])
        want_sym = z[f"c{i}_symbols"]
        assert ps.symbols.shape == want_sym.shape, (i, m)
        assert not len(want_sym) or \
            np.max(np.abs(ps.symbols - want_sym)) <= (0.0 if m["freq_offset"] == 0 else SOFT_TOL), (i, m)
        _hard_equal(hs, z[f"c{i}_hard"], want_sym)
        served += 1
    assert served >= 20


@pytest.mark.parametrize("dtype", [np.complex64, np.complex128])
def test_blocked_batch_and_limits(hip, dtype):
    """A 64-channel batch in the opt-in latency mode decimates time-blocked channel by channel as
    the oracle does (cf32 and cf64); the default form gives every channel the same result in a batch
    of 1, 64 or 65 (a row's output must not depend on the batch size) equal to the
    sequential oracle; the blocked form outside its limits (65 channels, q = 83) is refused."""
    from tetraear.signal import SignalProcessor
    from tetraear import _hip
    rng = np.random.default_rng(11)
    N = 20000
    x = (0.3 * (rng.standard_normal((65, N)) + 1j * rng.standard_normal((65, N)))).astype(dtype)
    fo = (np.arange(65) % 5 - 2) * 1171.875
    pb = SignalProcessor(2.4e6, decimator="blocked")
    hard, soft, ns = pb.process_batch(x[:64], fo[:64])
    p = SignalProcessor(2.4e6)
    h64, s64, n64 = p.process_batch(x[:64], fo[:64])
    h65, s65, n65 = p.process_batch(x, fo)
    for c in (0, 17, 63):
        o = O.SignalProcessor(2.4e6, decimator="blocked")
        want = o.process(x[c], fo[c])
        assert ns[c] == len(o.symbols) and np.array_equal(hard[c, :ns[c] - 1], want), c
        assert np.max(np.abs(soft[c, :ns[c]] - o.symbols)) <= 1e-12, c
        seq = O.SignalProcessor(2.4e6).process(x[c], fo[c])
        h1 = p.process(x[c], fo[c])
        assert np.array_equal(h65[c, :n65[c] - 1], seq) and np.array_equal(h64[c, :n64[c] - 1], seq), c
        assert np.array_equal(h1, seq), c
        assert np.array_equal(s64[c, :n64[c]], s65[c, :n65[c]]) and np.array_equal(p.symbols, s65[c, :n65[c]]), c
    with pytest.raises(_hip.TetraHipError):
        pb.process_batch(x, fo)
    with pytest.raises(_hip.TetraHipError):
        SignalProcessor(20e6, decimator="blocked").process(x[0].astype(dtype))


@pytest.mark.parametrize("N,fs", [(100, 2.4e6), (14, 240000.0), (400, 1.8e6)])
def test_real_short_mixed_offsets_batch_equals_process(hip, N, fs):
    """a batch of real rows too short for filtfilt with the mixer on for some rows only is
    split in two launches; its mixer-off rows must still be decided with real arithmetic as
    process() decides them (processor.py:102-166 on a real array), and equal the oracle."""
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(N)
    x = (0.4 * rng.standard_normal((4, N))).astype(np.float32)
    x[1, ::7] = 0.0   # exact zeros: signed-zero products decide differently in complex arithmetic
    fo = [0.0, 1171.875, 0.0, -2343.75]
    p = SignalProcessor(fs)
    hard, soft, ns = p.process_batch(x, fo)
    for c in range(4):
        h = p.process(x[c], fo[c])
        o = O.SignalProcessor(fs)
        ho = o.process(x[c], fo[c])
        assert ns[c] == len(p.symbols) == len(o.symbols), c
        assert np.array_equal(hard[c, :max(ns[c] - 1, 0)], h) and np.array_equal(h, ho), (c, fo[c])
