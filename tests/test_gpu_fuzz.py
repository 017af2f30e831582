"""Seeded random-geometry parity sweep (GPU through the C ABI vs the CPU oracle).

The other GPU tests pin chosen geometries; this sweep draws the ones nobody chose -- channel counts,
chunk lengths, sample rates, offsets, SNRs, input formats -- from fixed seeds, so a failure names a
reproducible case.  Bars are the same as the focused tests: compat soft symbols within 1e-5 and
hard decisions bit-exact outside the 1e-9 rad tie band (test_gpu_compat.py); the ETSI chain bit-exact
(symbols, soft bits, hard dibits, burst positions, decoded bits and CRC flags); scanner counts up to
the counted decision-edge ulps (test_scanner.py); gate statistics within GATE_DB_TOL and decisions
outside that band (test_spectrum.py); the channeliser within Y_TOL (test_wideband.py).

Covered: the default compat process() against the sequential (reference-order) oracle, compat
batches (latency and throughput kernels) and the direct SignalProcessor methods,
compat decoder streams, the ETSI chain with its lower MAC (cell given and acquired) and its component
methods, the streaming ETSI receiver over random chunk patterns (round 6), the scanner detector, the AFC gate, the wideband channeliser, its chunked timing (overlapping chunks, round 6) and its stream over capture pieces, device-tensor batches.  Each
host-side bug the sweep found keeps its case here ("sweep").
"""
import numpy as np
import pytest

import compat as O
import etsi as E
from test_gpu_compat import SOFT_TOL, _hard_equal

pytestmark = pytest.mark.gpu

# TETRA_FUZZ_SCALE=k runs k times as many seeds of every sweep (exploration; the default is the
# committed set the round-end suite runs)
SCALE = max(1, int(__import__("os").environ.get("TETRA_FUZZ_SCALE", "1")))

# reference rates: process() decimates by int(fs / 240e3) above 480 kHz (processor.py:245-256),
# so these reach q = 1 (no decimation), 4, 7, 8, 10, 13 and 41
COMPAT_RATES = [240e3, 1.0e6, 1.8e6, 2.0e6, 2.4e6, 3.2e6, 10e6]
ETSI_RATES = [1.8e6, 1.9e6, 2.0e6, 2.1e6, 2.2e6, 2.3e6, 2.4e6]


def _compat_case(seed):
    rng = np.random.default_rng(1000 + seed)
    fs = COMPAT_RATES[seed % len(COMPAT_RATES)]
    C = int(rng.integers(1, 6))
    tiny = rng.uniform() < 0.3   # around decimate's and filtfilt's padlen (27 and 15 samples)
    N = int(rng.integers(1, 500 if tiny else (60000 if fs < 5e6 else 200000)))
    decimator = ("sequential", "auto")[int(rng.integers(0, 2))]
    dtype = (np.complex64, np.complex128, np.float32)[int(rng.integers(0, 3))]
    fo = [float(rng.choice([0.0, rng.uniform(-4000, 4000)])) for _ in range(C)]
    if rng.uniform() < 0.3:
        fo = [0.0] * C
    return rng, fs, C, N, decimator, dtype, fo


@pytest.mark.parametrize("seed", range(42 * SCALE))
def test_compat_random_geometry_vs_oracle(seed):
    from tetraear.signal import SignalProcessor
    rng, fs, C, N, decimator, dtype, fo = _compat_case(seed)
    x = rng.uniform(0.05, 1.0) * (rng.standard_normal((C, N)) + 1j * rng.standard_normal((C, N)))
    x = (x.real if dtype == np.float32 else x).astype(dtype)   # real input: the reference accepts it too
    if rng.uniform() < 0.15 and N:
        x[:, rng.integers(0, N, size=max(1, N // 9))] = 0   # exact zeros: signed-zero products in the decision
    hard, soft, ns = SignalProcessor(fs, decimator=decimator).process_batch(x, fo)
    for c in range(C):
        o = O.SignalProcessor(fs, decimator=decimator)
        h = o.process(x[c], fo[c])
        case = (seed, fs, C, N, decimator, dtype.__name__, c)
        assert ns[c] == len(o.symbols), case
        if ns[c]:
            assert np.max(np.abs(soft[c, :ns[c]] - o.symbols)) <= SOFT_TOL, case
        _hard_equal(hard[c, :max(int(ns[c]) - 1, 0)], h, o.symbols)
    # one channel again through process(): the single-channel (latency) entry agrees with the batch
    p = SignalProcessor(fs, decimator=decimator)
    h1 = p.process(x[0], fo[0])
    assert len(p.symbols) == ns[0]
    if ns[0]:
        assert np.max(np.abs(p.symbols - soft[0, :ns[0]])) <= SOFT_TOL
    o = O.SignalProcessor(fs, decimator=decimator)
    _hard_equal(h1, o.process(x[0], fo[0]), o.symbols)


@pytest.mark.parametrize("seed", range(10 * SCALE))
def test_default_process_vs_reference_order(seed):
    """Cross-form: what an unchanged caller gets -- SignalProcessor(fs).process()
    on one GUI chunk and process_batch on a few -- against the SEQUENTIAL oracle (scipy's order,
    pinned to the reference's fixtures), never against the oracle of the same form.  Chunks of the
    round-6 form sweep (_signals.sweep_chunks: the GUI's chunk size, families and AFC offsets);
    soft symbols within 1e-5 and every hard decision equal, no tie band.  A time-blocked default
    fails this on the sweep's known cases (tests/test_compat_default_form.py)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import _signals
    from tetraear.signal import SignalProcessor
    chunks = list(_signals.sweep_chunks(seed, 4))
    p = SignalProcessor(2.4e6)
    want = []
    for k, fam, fo, x, _ in chunks:
        o = O.SignalProcessor(2.4e6, decimator="sequential")
        h = o.process(x, fo)
        want.append((h, o.symbols))
        got = p.process(x, fo)
        case = (seed, k, fam, fo)
        assert p.symbols.dtype == o.symbols.dtype and len(p.symbols) == len(o.symbols), case
        assert np.max(np.abs(p.symbols - o.symbols)) <= SOFT_TOL, case
        assert np.array_equal(got, h), case + (np.flatnonzero(got != h)[:8],)
    hard, soft, ns = p.process_batch(np.stack([c[3] for c in chunks]), [c[2] for c in chunks])
    for (h, sym), k in zip(want, range(len(chunks))):
        assert ns[k] == len(sym) and np.max(np.abs(soft[k, :ns[k]] - sym)) <= SOFT_TOL, (seed, k)
        assert np.array_equal(hard[k, :ns[k] - 1], h), (seed, k)


@pytest.mark.parametrize("seed", range(42 * SCALE))
def test_etsi_random_geometry_vs_oracle(seed):
    from tetraear.signal.etsi import EtsiReceiver, synth
    from tetraear.core.etsi import EtsiLowerMac
    rng = np.random.default_rng(2000 + seed)
    fs = ETSI_RATES[seed % len(ETSI_RATES)]
    C = int(rng.integers(1, 9))
    N = int(rng.integers(2, 6000 if rng.uniform() < 0.25 else 150000))
    snr = float(rng.uniform(4.0, 24.0))
    cfo = float(rng.uniform(0.0, 700.0))
    sc16 = bool(rng.integers(0, 2))
    iq, cells = synth(C, 150000, fs=fs, seed=3000 + seed, snr_db=snr, cfo_max=cfo)[:2]
    iq = iq[:, :N]
    inp = iq
    if sc16:
        inp = np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
        iq = (inp[..., 0].astype(np.float32) / 32768 + 1j * (inp[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    hard, soft, sym, ns = EtsiReceiver(fs).demod_batch(inp)
    rx = E.Receiver(fs)
    Ne = N - N % 2
    case = (seed, fs, C, N, round(snr, 1), round(cfo), "sc16" if sc16 else "cf32")
    for ch in range(C):
        so, sbo, ho, _ = rx.demod(iq[ch, :Ne])
        n = int(ns[ch])
        assert n == len(so), case + (ch,)
        assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :max(n - 1, 0)], ho), case + (ch,)
        assert np.array_equal(soft[ch, :2 * max(n - 1, 0)], sbo), case + (ch,)
    res = EtsiLowerMac().decode_batch(soft, hard, ns, cells)
    for ch in range(C):
        n = int(ns[ch])
        if n < 2:
            assert res[ch] == [], case + (ch,)
            continue
        want = rx.lower_mac(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], int(cells[ch]))
        got = res[ch]
        assert [(f["position"], f["burst_kind"]) for f in got] == [(s, k) for s, k, _ in want], case + (ch,)
        for f, (_, _, dec) in zip(got, want):
            assert len(f["blocks"]) == len(dec), case + (ch,)
            for b, (kind, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), case + (ch,)
    # no cell given: acquisition from the BSCH (tetra_lmac_etsi_acquire) against the oracle's
    from tetraear.core.etsi import UNKNOWN_CELL
    lm = EtsiLowerMac()
    res = lm.decode_batch(soft, hard, ns)
    for ch in range(C):
        n = int(ns[ch])
        if n < 2:
            assert res[ch] == [] and int(lm.cell_state[ch]) == UNKNOWN_CELL, case + (ch,)
            continue
        want, init = rx.lower_mac_acquire(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], UNKNOWN_CELL)
        assert int(lm.cell_state[ch]) == init, case + (ch,)
        assert [(f["position"], f["burst_kind"]) for f in res[ch]] == [(s, k) for s, k, _ in want], case + (ch,)
        for f, (_, _, dec) in zip(res[ch], want):
            for b, (kind, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), case + (ch,)


@pytest.mark.parametrize("seed", range(14 * SCALE))
def test_etsi_stream_random_chunks_vs_oracle(seed):
    """The streaming receiver (round 6) over chunk sequences nobody chose: every CLI rate, 1-4
    channels, chunk patterns mixing tiny chunks (a few samples: windows too short for the filter,
    k_track_skip), odd-sized and full ones, cf32 / SC16, cell given or acquired -- per chunk the
    symbols, soft bits, dibits, bursts (negative positions across seams), decoded bits, CRC flags and
    acquired cells equal the oracle Stream's (tests/test_gpu_stream.py's bar)."""
    from tetraear.signal.etsi import EtsiStream, synth
    from tetraear.core.etsi import EtsiLowerMac
    rng = np.random.default_rng(5000 + seed)
    fs = ETSI_RATES[seed % len(ETSI_RATES)]
    C = int(rng.integers(1, 5))
    n1 = int(131072 * fs / 2.4e6)
    pattern = []
    for _ in range(int(rng.integers(0, 4))):
        u = rng.uniform()
        pattern.append(int(rng.integers(2, 60)) if u < 0.35 else int(rng.integers(60, 5000)) if u < 0.7
                       else int(rng.integers(5000, n1 + 1)))
    pattern.insert(int(rng.integers(0, len(pattern) + 1)), int(rng.integers(20000, n1 + 1)))   # bounds the chunk count
    total = int(rng.integers(2 * n1, 4 * n1))
    sc16 = bool(rng.integers(0, 2))
    acquire = bool(rng.integers(0, 2))
    snr = float(rng.uniform(8.0, 24.0))
    iq, cells = synth(C, total, fs=fs, seed=6000 + seed, snr_db=snr, cfo_max=float(rng.uniform(0, 600)))[:2]
    inp = iq
    if sc16:
        inp = np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
        iq = (inp[..., 0].astype(np.float32) / 32768 + 1j * (inp[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    streams = [E.Stream(fs, cell_init=None if acquire else int(cells[ch])) for ch in range(C)]
    st, lm = EtsiStream(fs, C), EtsiLowerMac()
    at, k = 0, 0
    case = (seed, fs, C, pattern, total, "sc16" if sc16 else "cf32", "acquire" if acquire else "given")
    while at < total:
        n = min(pattern[k % len(pattern)], total - at)
        n -= n % 2
        if n == 0:
            break
        hard, soft, sym, ns = st.demod(inp[:, at:at + n])
        frames = lm.decode_stream(soft, hard, ns, None if acquire else cells)
        for ch in range(C):
            w = streams[ch].push(iq[ch, at:at + n])
            m = int(ns[ch])
            where = case + (k, at, n, ch)
            assert m == len(w["symbols"]), where
            assert np.array_equal(sym[ch, :m], w["symbols"]), where
            assert np.array_equal(hard[ch, :max(m - 1, 0)], w["hard"]), where
            assert np.array_equal(soft[ch, :2 * max(m - 1, 0)], w["soft"]), where
            assert [(f["position"], f["burst_kind"]) for f in frames[ch]] == [(p, kd) for p, kd, _ in w["bursts"]], where
            for f, (_, _, dec) in zip(frames[ch], w["bursts"]):
                for b, (kind, bits, ok) in zip(f["blocks"], dec):
                    assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), where
            if acquire:
                assert int(lm.cell_state[ch]) == w["cell"], where
        at += n
        k += 1


def _crc_burst_data(rng, fixed_tail):
    """216 type-2 burst data bits whose CRC-16 (the last 16) checks, with data[202:216] = fixed_tail
    (the sync bits the CRC field overlaps in a normal burst): data[0:16] solved over GF(2), the CRC
    being affine in its input."""
    d = rng.integers(0, 2, 216).astype(np.int64)
    d[202:216] = fixed_tail
    target = d[200:216].copy()
    d[:16] = 0
    c0 = O.calculate_crc16(np.zeros(200, np.int64))
    base = O.calculate_crc16(d[:200]) ^ target
    L = np.zeros((16, 16), np.int64)
    for i in range(16):
        e = np.zeros(200, np.int64)
        e[i] = 1
        L[:, i] = O.calculate_crc16(e) ^ c0
    # solve L x = base over GF(2) (Gauss-Jordan); L is invertible for 16 consecutive input bits
    A = np.concatenate([L, base[:, None]], 1) % 2
    for col in range(16):
        piv = col + int(np.argmax(A[col:, col]))
        assert A[piv, col] == 1
        A[[col, piv]] = A[[piv, col]]
        for r in range(16):
            if r != col and A[r, col]:
                A[r] ^= A[col]
    d[:16] = A[:, 16]
    assert O.check_crc(d)
    return d


@pytest.mark.parametrize("seed", range(24 * SCALE))
def test_decoder_random_streams_vs_oracle(seed):
    """Random symbol streams with bursts placed at random bit offsets: syncs with 0-4 bit errors,
    burst CRCs valid or 1-4 bits off (the reference accepts <= 2), both symbol alphabets -- the
    frames decode() keeps and their MAC PDU fields equal the oracle's decode_with_mac."""
    import mac as M
    from conftest import decoded_view
    from tetraear.core import TetraDecoder
    rng = np.random.default_rng(4000 + seed)
    nb = int(rng.integers(0, 12))
    nbits = int(rng.integers(600, 700 * max(nb, 1) + 600))
    bits = rng.integers(0, 2, nbits).astype(np.int64)
    at = 0
    for _ in range(nb):
        start = at + int(rng.integers(0, 120))
        if start + 510 > nbits:
            break
        if rng.uniform() < 0.8:
            start -= start % 2   # symbol-aligned (the slot parse reads whole symbols)
        sync = (O.SYNC_CONT if rng.uniform() < 0.5 else O.SYNC_DISC).astype(np.int64).copy()
        burst = rng.integers(0, 2, 510).astype(np.int64)
        data = _crc_burst_data(rng, sync[:14])
        burst[0:108], burst[122:230] = data[:108], data[108:]
        for i in rng.choice(216, size=int(rng.choice([0, 0, 0, 1, 2, 3, 4])), replace=False):
            j = i if i < 108 else i + 14
            burst[j] ^= 1   # CRC errors: <= 2 still pass (compat_oracle.c orc_check_crc)
        burst[216:238] = sync
        for i in rng.choice(22, size=int(rng.choice([0, 0, 1, 2, 3, 4])), replace=False):
            burst[216 + i] ^= 1   # sync bit errors: the decoder's 0.90 / 0.85 / 0.80 / adaptive cascade
        bits[start:start + 510] = burst
        at = start + 510
    bits = bits[:nbits - nbits % 2]
    sym = (2 * bits[0::2] + bits[1::2]).astype(np.uint8)
    u = rng.uniform()
    if u < 0.15:   # the 8-PSK alphabet branch of symbols_to_bits (decoder.py:150-160)
        sym = rng.integers(0, 8, len(sym)).astype(np.uint8)
    elif u < 0.25:   # wider integers, values outside both alphabets (mapped to 0 by the LUT branch)
        sym = np.where(rng.uniform(size=len(sym)) < 0.05, rng.integers(-3, 12, len(sym)), sym).astype(np.int64)
    d = TetraDecoder(auto_decrypt=False)
    got = [decoded_view(f) for f in d.decode(sym)]
    mp = M.MacParser()
    want = O.decode_with_mac(sym, mp)
    assert got == want, (seed, nb, nbits)
    st = d.protocol_parser.stats
    assert (st["clear_mode_frames"], st["encrypted_frames"]) == (mp.n_clear, mp.n_enc), seed


_DTYPES = (np.complex64, np.complex128, np.float32, np.float64)


def _rand_samples(rng, n, dtype):
    x = rng.uniform(0.01, 3.0) * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    if rng.uniform() < 0.1 and n:
        x[rng.integers(0, n, size=max(1, n // 7))] = 0   # exact zeros (|x| = 0, angle 0)
    return (x if np.dtype(dtype).kind == "c" else x.real).astype(dtype)


@pytest.mark.parametrize("seed", range(40 * SCALE))
def test_direct_methods_random_vs_oracle(seed):
    """The reference's SignalProcessor methods called directly (as modern.py / the tools do) on
    random lengths, rates, bandwidths and all four sample dtypes: filter_signal bit-exact (fp64
    DF-II-T, no libm), extract_symbols bit-exact, frequency_shift within 1e-12 (libm sin/cos),
    demodulate_dqpsk bit-exact outside the tie band -- each with the oracle's output dtype."""
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(5000 + seed)
    fs = float(rng.choice([240e3, 1.0e6, 1.8e6, 2.4e6]))
    p, o = SignalProcessor(fs), O.SignalProcessor(fs)
    dtype = _DTYPES[int(rng.integers(0, 4))]
    n = int(rng.integers(0, 40 if rng.uniform() < 0.25 else 20000))
    x = _rand_samples(rng, n, dtype)
    case = (seed, fs, dtype.__name__, n)
    rate = None if rng.uniform() < 0.5 else float(rng.choice([240e3, 500e3, 1.0e6, 2.4e6]))
    bw = float(rng.choice([25000, 12500, 50000, rng.uniform(1000, 400000)]))
    got, want = p.filter_signal(x, bandwidth=bw, sample_rate=rate), o.filter_signal(x, bandwidth=bw, sample_rate=rate)
    assert np.asarray(got).dtype == np.asarray(want).dtype and np.array_equal(got, want), case + ("filter", rate, bw)
    off = float(rng.uniform(-20000, 20000))
    got, want = p.frequency_shift(x, off, sample_rate=rate), o.frequency_shift(x, off, sample_rate=rate)
    assert got.dtype == want.dtype and got.shape == want.shape, case + ("shift",)
    if n:
        assert np.max(np.abs(got - want)) <= 1e-12 * max(1.0, float(np.max(np.abs(want)))), case + ("shift", off)
    got, want = p.extract_symbols(x, sample_rate=rate), o.extract_symbols(x, sample_rate=rate)
    assert np.asarray(got).dtype == np.asarray(want).dtype and np.array_equal(got, want), case + ("extract", rate)
    s = _rand_samples(rng, int(rng.integers(0, 3000)), dtype)
    got, want = p.demodulate_dqpsk(s), o.demodulate_dqpsk(s)
    assert got.dtype == want.dtype == np.uint8, case
    _hard_equal(got, want, s if np.iscomplexobj(s) else s.astype(np.complex128))


@pytest.mark.parametrize("seed", range(16 * SCALE))
def test_scanner_counts_random_vs_oracle(seed):
    """The scanner detector's counts (scanner.py:42-147, 204-231) on random batches: TETRA-like
    chunks, noise, tones, silence, clipped and tiny rows at random rates and lengths, both complex
    dtypes -- equal to the oracle's up to the counted decision-edge ulps (test_scanner.py)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import _signals
    from test_scanner import _compare_counts
    from tetraear.signal import scanner as S
    rng = np.random.default_rng(6000 + seed)
    fs = float(rng.choice([240e3, 1.0e6, 1.8e6, 2.4e6, 3.2e6]))
    N = int(rng.integers(0, 300 if rng.uniform() < 0.2 else 150000))
    rows = []
    for _ in range(int(rng.integers(1, 7))):
        kind = rng.choice(["tetra", "stress", "noise", "tone", "zero", "clip"])
        if kind == "zero":
            rows.append(np.zeros(N, np.complex64))
        elif kind == "clip":
            x = _signals.family("tetra", rng, N, fs)[0] * 40
            rows.append((np.clip(x.real, -1, 1) + 1j * np.clip(x.imag, -1, 1)).astype(np.complex64))
        else:
            rows.append(_signals.family(str(kind), rng, N, fs)[0])
    x = np.stack(rows).astype((np.complex64, np.complex128)[int(rng.integers(0, 2))])
    st = S.scan_counts(x, fs)
    for c in range(len(x)):
        _compare_counts(st[c], x[c], fs)


@pytest.mark.parametrize("seed", range(10 * SCALE))
def test_wideband_channelize_random_vs_oracle(seed, monkeypatch):
    """The C3 channeliser on random capture lengths (down to a few filter-bank blocks, ragged
    tails), both filter-bank designs, every analysis form the host can pick and a random prefix
    length: within test_wideband.py's Y_TOL of the float64 oracle, and a prefix request equal to the
    full result's prefix."""
    import wideband as W
    from test_wideband import Y_TOL
    from tetraear.signal.wideband import WidebandReceiver, synth_wideband
    rng = np.random.default_rng(7000 + seed)
    oversample = int(rng.choice([2, 4]))
    form = str(rng.choice(["1", "2", "3", "4"] if oversample == 2 else ["1", "2"]))
    monkeypatch.setenv("TETRA_WB_ANALYSIS", form)
    Nw = int(rng.integers(1600, 5000 if rng.uniform() < 0.3 else 600000))
    x = synth_wideband(Nw, seed=8000 + seed, snr_db=float(rng.uniform(5, 30)), oversample=oversample)[0]
    d = W.design(oversample=oversample)
    rx = WidebandReceiver(oversample=oversample)
    y = rx.channelize(x)
    want = W.channelize(x.astype(np.complex128), d)
    case = (seed, oversample, form, Nw)
    assert y.shape == want.shape, case
    if y.size:
        assert np.abs(y - want).max() <= Y_TOL * max(np.abs(want).max(), 1e-30), case
        k = int(rng.integers(1, y.shape[1] + 1))
        assert np.array_equal(rx.channelize(x, k), y[:, :k]), case + (k,)


@pytest.mark.parametrize("seed", range(12 * SCALE))
def test_afc_gate_random_vs_oracle(seed):
    """The signal-present / AFC gate on random batches (tones anywhere in or beside the band,
    TETRA-like bursts with CFO, noise at random levels, silence, chunks shorter than 2048 samples) at
    the CLI rates, complex64 or complex128: statistics within test_spectrum.py's GATE_DB_TOL of the
    float64 oracle; the decision, peak bin and AFC offset equal wherever the oracle's margins exceed
    that tolerance (a random case may sit inside the band, the fixed ones do not)."""
    import spectrum as SO
    from test_spectrum import GATE_DB_TOL
    from tetraear.signal.etsi import synth
    from tetraear.signal.spectrum import afc_gate
    rng = np.random.default_rng(9000 + seed)
    fs = float(rng.choice([1.8e6, 1.9e6, 2.0e6, 2.1e6, 2.2e6, 2.3e6, 2.4e6]))
    N = int(rng.integers(1000, 2100) if rng.uniform() < 0.15 else rng.integers(2048, 40000))
    rows = []
    n = np.arange(N)
    for _ in range(int(rng.integers(1, 7))):
        kind = rng.choice(["tone", "tetra", "noise", "zero"])
        sig = 10 ** rng.uniform(-6, -1) * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
        if kind == "tone":
            f = rng.uniform(-30000, 30000)
            sig = sig + 10 ** rng.uniform(-4, 0) * np.exp(2j * np.pi * f * n / fs)
        elif kind == "tetra":
            sig = synth(1, 2 * ((N + 1) // 2), fs=fs, seed=int(rng.integers(1, 1 << 30)),
                        snr_db=float(rng.uniform(0, 30)))[0][0][:N]
        elif kind == "zero":
            sig = np.zeros(N)
        rows.append(sig)
    x = np.stack(rows).astype((np.complex64, np.complex128)[int(rng.integers(0, 2))])
    got = afc_gate(x, fs)
    for i in range(len(x)):
        want = SO.gate_iq(x[i], fs)
        case = (seed, fs, N, i)
        assert float(got["valid"][i]) == want["valid"], case
        if not want["valid"]:
            assert not got["present"][i] and float(got["afc"][i]) == 0.0, case
            continue
        # the fp32 FFT resolves a bin to ~1e-7 of the frame's largest one: where the frame spans more
        # than ~100 dB (a strong tone outside the band over a -140 dB floor) the deep bins carry that
        # error into the noise mean, so there the statistics are held to 5x the tolerance (measured
        # 2.05e-3 dB at a 125 dB span, seed 44 of TETRA_FUZZ_SCALE=6); decisions unaffected
        p = SO.frame_power(x[i], SO.N_FFT)
        tol = GATE_DB_TOL if float(np.max(p)) - want["noise"] < 100 else 5 * GATE_DB_TOL
        for k in ("signal", "peak", "noise", "snr", "above"):
            assert abs(float(got[k][i]) - want[k]) <= tol, case + (k, float(got[k][i]), want[k])
        start, end, _, _ = SO.gate_bins(fs)
        top = np.sort(np.asarray(p[start:end], np.float64))[::-1]
        clear_peak = len(top) < 2 or top[0] - top[1] > 2 * GATE_DB_TOL
        margins = min(abs(want["snr"] - 15), abs(want["peak"] + 70), abs(want["above"] - 3))
        if clear_peak:
            assert float(got["peak_bin"][i]) == want["peak_bin"], case
            assert float(got["peak_freq"][i]) == want["peak_freq"], case
        if margins > 2 * GATE_DB_TOL:
            assert float(got["present"][i]) == want["present"], case + (want["snr"], want["peak"], want["above"])
            if clear_peak:
                assert float(got["afc"][i]) == want["afc"], case


@pytest.mark.parametrize("seed", range(8 * SCALE))
def test_compat_device_tensor_batches_equal_host(seed):
    """process_batch on device tensors -- complex64 / complex128 [C, N] or float32 / float64
    [C, N, 2], contiguous or a strided row selection, offsets on the host or as a device tensor --
    returns exactly what the host-array call returns (the tensor path reads the tensor's
    own format, made contiguous, never reinterpreted)."""
    import torch
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(9500 + seed)
    fs = float(rng.choice([1.8e6, 2.4e6]))
    C, N = int(rng.integers(1, 6)), int(rng.integers(100, 40000))
    x = (0.3 * (rng.standard_normal((2 * C, N)) + 1j * rng.standard_normal((2 * C, N))))
    x = x.astype((np.complex64, np.complex128)[int(rng.integers(0, 2))])
    fo = np.where(rng.uniform(size=C) < 0.5, 0.0, rng.uniform(-3000, 3000, C))
    host = x[::2]                                  # the rows the device call selects
    want = SignalProcessor(fs).process_batch(np.ascontiguousarray(host), fo)
    t = torch.from_numpy(x).cuda()[::2]            # non-contiguous: every other row
    if rng.uniform() < 0.5:
        t = torch.view_as_real(t.contiguous())     # [C, N, 2] real layout
    offs = torch.from_numpy(fo).cuda() if rng.uniform() < 0.5 else fo
    got = SignalProcessor(fs).process_batch(t, offs)
    for g, w in zip(got, want):
        assert np.array_equal(g, w), (seed, fs, C, N, x.dtype)


@pytest.fixture(scope="module")
def y72():
    """72 kHz rows from the GPU channel filter of two synthetic 2.4 MSps channels (the timing's input)."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths, synth
    iq = synth(2, 262144, seed=31, snr_db=18.0)[0]
    plan = etsi_plan()
    _, M2, _ = lengths(plan, iq.shape[1])
    y = np.zeros((2, M2), np.complex64)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), 2, iq.shape[1], _hip.ptr(y)), "chanfilt")
    return y


@pytest.mark.parametrize("seed", range(12 * SCALE))
def test_timing_chunks_random_vs_oracle(seed, y72):
    """tetra_etsi_timing_chunks (the wideband timing, round 6) at random geometries: rows, row length,
    chunk stride and length (overlapping, tiling or with gaps), the last chunk cut by the row's end,
    resampler group sizes, the grouped Oerder-Meyr sums or the timing's own pass -- every output of
    every chunk bit-identical to the oracle's timing of the chunk's samples."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan
    rng = np.random.default_rng(12000 + seed)
    M = int(rng.integers(1, 5))
    rowlen = int(rng.integers(16, 3 * y72.shape[1]))
    grouped = bool(rng.uniform() < 0.6)
    U = 4 * int(rng.integers(1, 17))
    stride = int(rng.integers(1, max(2, rowlen // 2)))
    if grouped:
        stride = max(4, stride - stride % 4)
    length = int(rng.integers(16, max(17, min(rowlen, 3 * stride) + 1)))
    nchunk = max(1, min((rowlen - 16) // stride + 1, int(rng.integers(1, 12))))
    rows = np.stack([np.resize(np.roll(y72[r % 2], int(rng.integers(0, y72.shape[1]))), rowlen)
                     for r in range(M)]).astype(np.complex64)
    if rng.uniform() < 0.3:   # a noise row among them
        rows[-1] = (rng.standard_normal(rowlen) + 1j * rng.standard_normal(rowlen)).astype(np.complex64)
    ngrp = -(-rowlen // U)
    om = np.stack([E.Receiver.om_group_partials(r, U) for r in rows]).astype(np.float32) if grouped else None
    C, sm = M * nchunk, length // 4 + 2
    sym = np.zeros((C, sm), np.complex64)
    soft, hard, ns = np.zeros((C, 2 * sm), np.int8), np.zeros((C, sm), np.uint8), np.zeros(C, np.int32)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_timing_chunks(c.handle, etsi_plan(), _hip.ptr(rows), M, rowlen, nchunk, stride, length,
                                           _hip.ptr(om), ngrp if grouped else 0, U, _hip.ptr(sym), _hip.ptr(soft),
                                           _hip.ptr(hard), _hip.ptr(ns), sm, None), "timing_chunks")
    ora = E.Receiver()
    case = (seed, M, rowlen, nchunk, stride, length, U, grouped)
    for r in range(M):
        for ci in range(nchunk):
            s0 = ci * stride
            L = min(length, rowlen - s0)
            A = E.Receiver.om_grouped(rows[r], s0, L, U, om[r]) if grouped else None
            so, sbo, ho, _ = ora.timing(rows[r, s0:s0 + L], om=A)
            ch = r * nchunk + ci
            n = int(ns[ch])
            assert n == len(so), case + (r, ci)
            assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :n - 1], ho), case + (r, ci)
            assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), case + (r, ci)


@pytest.mark.parametrize("seed", range(4 * SCALE))
def test_wideband_stream_random_pieces(seed):
    """WidebandStream (round 6) over random cuts of a random-length capture at a random SNR: every
    carrier's frames are the whole capture's -- stream positions within the timing phase, the same
    CRC-good bits (test_wideband.py's equality, on pieces nobody chose)."""
    from tetraear.signal import wideband as WB
    rng = np.random.default_rng(13000 + seed)
    Nw = int(rng.integers(600_000, 3_000_000))
    x, cells = WB.synth_wideband(Nw, seed=13100 + seed, snr_db=float(rng.uniform(20, 30)))[:2]
    whole = WB.WidebandReceiver().decode(x, cells)
    cuts = np.sort(rng.choice(np.arange(1, Nw), size=int(rng.integers(1, 5)), replace=False))
    st = WB.WidebandStream(cells)
    got = [[] for _ in range(len(cells))]
    for a, b in zip(np.r_[0, cuts], np.r_[cuts, Nw]):
        for k, fr in enumerate(st.decode(x[a:b])):
            got[k].extend(fr)
    case = (seed, Nw, cuts.tolist())
    for k in range(len(cells)):
        ws = [f["sample"] for f in whole[k]]
        gs = [f["stream_sample"] for f in got[k]]
        assert len(gs) == len(ws) and all(abs(p - q) <= 16 for p, q in zip(gs, ws)), case + (k, ws, gs)
        for fw, fg in zip(whole[k], got[k]):
            assert [tuple(b["bits"]) for b in fw["blocks"] if b["crc_ok"]] == \
                [tuple(b["bits"]) for b in fg["blocks"] if b["crc_ok"]], case + (k, fw["sample"])


@pytest.mark.parametrize("seed", range(12 * SCALE))
def test_etsi_components_random_vs_oracle(seed):
    """ETSI mode's component methods at random rates and lengths: filter_signal (the channel
    filter) and extract_symbols (timing) bit-identical to the oracle's chanfilt / timing, process()
    with a random AFC offset on an exact mixer-free split, and demodulate_dqpsk (Table 5.1 on given
    complex64 symbols, zeros included) bit-identical to eo_decide."""
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import synth
    rng = np.random.default_rng(9800 + seed)
    fs = ETSI_RATES[seed % len(ETSI_RATES)]
    N = int(rng.integers(2, 4000 if rng.uniform() < 0.25 else 140000))
    iq = synth(1, 140000, fs=fs, seed=9900 + seed, snr_db=float(rng.uniform(5, 25)))[0][0][:N]
    p, rx = SignalProcessor(fs, mode="etsi"), E.Receiver(fs)
    Ne = N - N % 2
    y = p.filter_signal(iq)
    yo = rx.chanfilt(iq[:Ne])
    assert np.array_equal(y, yo), (seed, fs, N)
    if len(yo) >= 16:
        s = p.extract_symbols(y)
        so, _, ho, _ = rx.timing(yo)
        assert np.array_equal(s, so), (seed, fs, N)
        hard = p.process(iq)
        assert np.array_equal(p.symbols, so) and np.array_equal(np.asarray(hard), ho), (seed, fs, N)
    nz = int(rng.integers(0, 3000))
    z = (rng.standard_normal(nz) + 1j * rng.standard_normal(nz)).astype(np.complex64)
    if len(z) > 4 and rng.uniform() < 0.5:
        z[rng.integers(0, len(z), size=len(z) // 5)] = 0
    assert np.array_equal(p.demodulate_dqpsk(z), E.Receiver.decide(z)), (seed, len(z))


@pytest.mark.parametrize("seed", range(6 * SCALE))
def test_compat_large_batches_vs_oracle(seed):
    """Batches past the latency mode's 64 channels (the throughput kernels: banked decimator, one
    wave per channel in filtfilt / extract / demod) at random rates, lengths and offsets: sampled
    channels equal the oracle's sequential chain."""
    from tetraear.signal import SignalProcessor
    rng = np.random.default_rng(9700 + seed)
    fs = COMPAT_RATES[1 + seed % (len(COMPAT_RATES) - 1)]
    C, N = int(rng.integers(65, 300)), int(rng.integers(30, 30000))
    x = (0.3 * (rng.standard_normal((C, N)) + 1j * rng.standard_normal((C, N)))).astype(np.complex64)
    fo = np.where(rng.uniform(size=C) < 0.3, 0.0, rng.uniform(-4000, 4000, C))
    hard, soft, ns = SignalProcessor(fs).process_batch(x, fo)
    for c in sorted({0, C - 1, *rng.integers(0, C, 4).tolist()}):
        o = O.SignalProcessor(fs)
        h = o.process(x[c], fo[c])
        case = (seed, fs, C, N, c)
        assert ns[c] == len(o.symbols), case
        if ns[c]:
            assert np.max(np.abs(soft[c, :ns[c]] - o.symbols)) <= SOFT_TOL, case
        _hard_equal(hard[c, :max(int(ns[c]) - 1, 0)], h, o.symbols)
