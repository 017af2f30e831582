"""GPU parity of the ETSI chain (HIP through the C ABI) against the CPU oracle.

The reference has no ETSI chain, so the oracle (oracle/etsi_oracle.c) is the specification:
its float operations are restated in the kernels, so soft symbols, soft bits, hard decisions,
burst positions and decoded bits are compared EXACTLY (bar: soft symbols within 1e-5, decoded
bits bit-exact).  Full-size runs are checked by round-trip properties (decoded payloads are the
transmitted ones, CRC pass rate).
"""
import numpy as np
import pytest

import etsi as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def synth_small():
    from tetraear.signal.etsi import synth
    iq, cells, kinds, payload, t0 = synth(6, 131072, seed=3, snr_db=16.0, cfo_max=600.0)
    return iq, cells, kinds, payload, t0


def test_plan_matches_oracle_design():
    from tetraear.signal.etsi import etsi_plan
    p = etsi_plan(2.4e6)
    d = E.design(2.4e6)
    assert np.array_equal(np.ctypeslib.as_array(p.h1)[:48], d["h1"])
    assert np.array_equal(np.ctypeslib.as_array(p.hp)[:321], d["hp"])
    assert p.gain == d["gain"] and p.soft_scale == d["soft_scale"]


def test_chanfilt_and_timing_bit_exact(synth_small):
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths, EtsiReceiver
    iq = synth_small[0]
    rx = E.Receiver()
    plan = etsi_plan()
    C, N = iq.shape
    _, M2, smax = lengths(plan, N)
    y = np.zeros((C, M2), np.complex64)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), C, N, _hip.ptr(y)))
    hard, soft, sym, ns = EtsiReceiver().demod_batch(iq)   # fused: y stays in LDS
    # the component path (chanfilt -> y in HBM -> k_timing) gives the same symbols
    sym2 = np.zeros_like(sym)
    soft2, hard2, ns2 = np.zeros_like(soft), np.zeros_like(hard), np.zeros_like(ns)
    c.check(c.lib.tetra_etsi_timing(c.handle, plan, _hip.ptr(y), C, M2, _hip.ptr(sym2), _hip.ptr(soft2),
                                    _hip.ptr(hard2), _hip.ptr(ns2), smax, None))
    assert np.array_equal(ns, ns2)
    for ch in range(C):
        n = int(ns[ch])
        assert np.array_equal(sym[ch, :n], sym2[ch, :n]) and np.array_equal(hard[ch, :n - 1], hard2[ch, :n - 1])
        assert np.array_equal(soft[ch, :2 * (n - 1)], soft2[ch, :2 * (n - 1)])
    for ch in range(C):
        yo = rx.chanfilt(iq[ch])
        assert len(yo) == M2 and np.array_equal(y[ch], yo), ch
        so, sbo, ho, diag = rx.timing(yo)
        n = int(ns[ch])
        assert n == len(so), ch
        assert np.array_equal(sym[ch, :n], so), ch          # bit-exact soft symbols
        assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), ch
        assert np.array_equal(hard[ch, :n - 1], ho), ch


@pytest.mark.parametrize("ring,lean", [(0, 0), (0, 1), (1, 0), (1, 1), (2, 0), (2, 1)])
def test_timing_forms_bit_exact(synth_small, ring, lean, monkeypatch):
    """Every k_timing form the host can pick (TETRA_TIMING_RING: Gardner windows from global memory,
    an LDS ring fed one or two blocks ahead; TETRA_TIMING_LEAN: the Oerder-Meyr pass with all quarters'
    loads together and d_j recomputed from the stored symbols, or round 3's form) equals the oracle's timing bit for bit, on full chunks and on ragged
    lengths (a partial last block, a chunk shorter than the ring's prefill)."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths
    monkeypatch.setenv("TETRA_TIMING_RING", str(ring))
    monkeypatch.setenv("TETRA_TIMING_LEAN", str(lean))
    iq = synth_small[0][:4]
    rx = E.Receiver()
    plan = etsi_plan()
    C, N = iq.shape
    _, M2, smax = lengths(plan, N)
    c = _hip.ctx()
    y = np.zeros((C, M2), np.complex64)
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), C, N, _hip.ptr(y)))
    for m2 in (M2, M2 - 37, 1001, 300, 17):
        yy = np.ascontiguousarray(y[:, :m2])
        sm = m2 // 4 + 2
        sym = np.zeros((C, sm), np.complex64)
        soft, hard, ns = np.zeros((C, 2 * sm), np.int8), np.zeros((C, sm), np.uint8), np.zeros(C, np.int32)
        c.check(c.lib.tetra_etsi_timing(c.handle, plan, _hip.ptr(yy), C, m2, _hip.ptr(sym), _hip.ptr(soft),
                                        _hip.ptr(hard), _hip.ptr(ns), sm, None))
        for ch in range(C):
            so, sbo, ho, _ = rx.timing(yy[ch])
            n = int(ns[ch])
            assert n == len(so), (m2, ch)
            assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :n - 1], ho), (m2, ch)
            assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), (m2, ch)


@pytest.mark.parametrize("m2,nchunk,U", [(3932, 3, 36), (1000, 5, 36), (1000, 4, 4), (2048, 3, 64), (404, 7, 12),
                                          (36, 4, 36), (20, 6, 36)])
def test_timing_om_geometries_bit_exact(synth_small, m2, nchunk, U):
    """tetra_etsi_timing_om, apart from the resampler: rows of nchunk chunks of real 72 kHz samples, the
    group partials from the oracle (eo_om_group_partials), and chunk boundaries on and off the groups
    (whole chunks of groups, heads and tails, chunks shorter than one group) -- the GPU's class sums
    and every output equal the oracle's timing with the grouped order."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths
    iq = synth_small[0][:2]
    plan = etsi_plan()
    C0, N = iq.shape
    _, M2, _ = lengths(plan, N)
    c = _hip.ctx()
    y0 = np.zeros((C0, M2), np.complex64)
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), C0, N, _hip.ptr(y0)))
    # carrier rows cut from the two channels' y (wrapping), nchunk chunks each
    rows = np.stack([np.resize(np.roll(y0[r % C0], 977 * r), nchunk * m2) for r in range(3)]).astype(np.complex64)
    ngrp = -(-nchunk * m2 // U)
    om = np.stack([E.Receiver.om_group_partials(r, U) for r in rows]).astype(np.float32)
    assert om.shape == (3, ngrp, 4)
    C, sm = 3 * nchunk, m2 // 4 + 2
    sym = np.zeros((C, sm), np.complex64)
    soft, hard, ns = np.zeros((C, 2 * sm), np.int8), np.zeros((C, sm), np.uint8), np.zeros(C, np.int32)
    c.check(c.lib.tetra_etsi_timing_om(c.handle, plan, _hip.ptr(rows), C, m2, _hip.ptr(om), nchunk, ngrp, U,
                                       _hip.ptr(sym), _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), sm, None),
            "etsi_timing_om")
    ora = E.Receiver()
    for r in range(3):
        for ci in range(nchunk):
            s0 = ci * m2
            A = E.Receiver.om_grouped(rows[r], s0, m2, U, om[r])
            so, sbo, ho, _ = ora.timing(rows[r, s0:s0 + m2], om=A)
            ch = r * nchunk + ci
            n = int(ns[ch])
            assert n == len(so), (r, ci)
            assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :n - 1], ho), (r, ci)
            assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), (r, ci)


def test_timing_om_rejects_bad_geometry():
    """The grouped-order entry point returns an error code (no launch) for geometries its class sums
    do not cover: C not a multiple of nchunk, M2 not a multiple of 4, U not a multiple of 4 or > 64,
    partials that do not cover the rows."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan
    plan = etsi_plan()
    c = _hip.ctx()
    y = np.zeros((4, 400), np.complex64)
    om = np.zeros((2, 40, 4), np.float32)
    sym, soft = np.zeros((4, 102), np.complex64), np.zeros((4, 204), np.int8)
    hard, ns = np.zeros((4, 102), np.uint8), np.zeros(4, np.int32)
    for C, m2, nchunk, ngrp, U in ((4, 400, 3, 40, 36), (4, 398, 2, 40, 36), (4, 400, 2, 40, 18),
                                   (4, 400, 2, 40, 68), (4, 400, 2, 10, 36)):
        rc = c.lib.tetra_etsi_timing_om(c.handle, plan, _hip.ptr(y), C, m2, _hip.ptr(om), nchunk, ngrp, U,
                                        _hip.ptr(sym), _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), 102, None)
        assert rc != 0, (C, m2, nchunk, ngrp, U)


@pytest.mark.parametrize("rowlen,nchunk,stride,length,U,grouped", [
    (12000, 3, 3932, 5012, 36, True), (12000, 3, 3932, 5012, 36, False), (11879, 3, 3932, 5011, 36, True),
    (5000, 4, 1000, 1999, 4, True), (3000, 5, 500, 1337, 64, True), (4100, 6, 640, 1000, 12, False),
    (700, 3, 200, 360, 36, True), (100, 2, 40, 60, 36, True)])
def test_timing_chunks_geometries_bit_exact(synth_small, rowlen, nchunk, stride, length, U, grouped):
    """tetra_etsi_timing_chunks, apart from the resampler: chunk c of each row is row[c stride,
    min(c stride + length, rowlen)) -- overlapping chunks, the last cut by the row's end, odd
    lengths, chunk starts on and off the groups, the grouped class sums or the timing's own pass --
    and every output equals the oracle's timing of the chunk's samples."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths
    iq = synth_small[0][:2]
    plan = etsi_plan()
    C0, N = iq.shape
    _, M2, _ = lengths(plan, N)
    c = _hip.ctx()
    y0 = np.zeros((C0, M2), np.complex64)
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), C0, N, _hip.ptr(y0)))
    rows = np.stack([np.resize(np.roll(y0[r % C0], 977 * r), rowlen) for r in range(3)]).astype(np.complex64)
    ngrp = -(-rowlen // U)
    om = np.stack([E.Receiver.om_group_partials(r, U) for r in rows]).astype(np.float32) if grouped else None
    C, sm = 3 * nchunk, length // 4 + 2
    sym = np.zeros((C, sm), np.complex64)
    soft, hard, ns = np.zeros((C, 2 * sm), np.int8), np.zeros((C, sm), np.uint8), np.zeros(C, np.int32)
    c.check(c.lib.tetra_etsi_timing_chunks(c.handle, plan, _hip.ptr(rows), 3, rowlen, nchunk, stride, length,
                                           _hip.ptr(om), ngrp if grouped else 0, U, _hip.ptr(sym), _hip.ptr(soft),
                                           _hip.ptr(hard), _hip.ptr(ns), sm, None), "etsi_timing_chunks")
    ora = E.Receiver()
    for r in range(3):
        for ci in range(nchunk):
            s0 = ci * stride
            L = min(length, rowlen - s0)
            A = E.Receiver.om_grouped(rows[r], s0, L, U, om[r]) if grouped else None
            so, sbo, ho, _ = ora.timing(rows[r, s0:s0 + L], om=A)
            ch = r * nchunk + ci
            n = int(ns[ch])
            assert n == len(so), (r, ci)
            assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :n - 1], ho), (r, ci)
            assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), (r, ci)


def test_timing_chunks_rejects_bad_geometry():
    """tetra_etsi_timing_chunks returns an error code (no launch) for a chunk shorter than 16 samples
    (length, or the last chunk cut by the row's end), smax < length / 4 + 2, and with partials a
    stride not a multiple of 4, U not a multiple of 4 or > 64, or partials short of the row."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan
    plan = etsi_plan()
    c = _hip.ctx()
    y = np.zeros((2, 1000), np.complex64)
    om = np.zeros((2, 40, 4), np.float32)
    sym, soft = np.zeros((8, 200), np.complex64), np.zeros((8, 400), np.int8)
    hard, ns = np.zeros((8, 200), np.uint8), np.zeros(8, np.int32)
    for nchunk, stride, length, smax, U, ngrp in ((2, 400, 12, 200, 36, 40), (4, 330, 400, 200, 36, 40),
                                                  (2, 400, 800, 150, 36, 40), (2, 402, 500, 200, 36, 40),
                                                  (2, 400, 500, 200, 18, 40), (2, 400, 500, 200, 68, 40),
                                                  (2, 400, 500, 200, 36, 20)):
        rc = c.lib.tetra_etsi_timing_chunks(c.handle, plan, _hip.ptr(y), 2, 1000, nchunk, stride, length,
                                            _hip.ptr(om), ngrp, U, _hip.ptr(sym), _hip.ptr(soft), _hip.ptr(hard),
                                            _hip.ptr(ns), smax, None)
        assert rc != 0, (nchunk, stride, length, smax, U, ngrp)


def test_lower_mac_matches_oracle(synth_small):
    from tetraear.signal.etsi import EtsiReceiver
    from tetraear.core.etsi import EtsiLowerMac
    iq, cells, kinds, payload, t0 = synth_small
    hard, soft, sym, ns = EtsiReceiver().demod_batch(iq)
    res = EtsiLowerMac().decode_batch(soft, hard, ns, cells)
    rx = E.Receiver()
    total_ok = 0
    for ch in range(len(iq)):
        n = int(ns[ch])
        want = rx.lower_mac(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], int(cells[ch]))
        got = res[ch]
        assert [(f["position"], f["burst_kind"]) for f in got] == [(s, k) for s, k, _ in want], ch
        for f, (_, _, dec) in zip(got, want):
            assert len(f["blocks"]) == len(dec)
            for b, (kind, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), ch
                total_ok += ok
        sent = {tuple(p) for bb in payload[ch] for p in bb}
        for f in got:
            for b in f["blocks"]:
                if b["crc_ok"]:
                    assert tuple(np.pad(b["bits"], (0, 268 - len(b["bits"])))) in sent
    assert total_ok >= 12


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_block_codec_vs_oracle(kind):
    """Encoder and decoder components bit-exact vs the oracle, including noisy soft inputs."""
    from tetraear import _hip
    rng = np.random.default_rng(kind)
    K, a, n2, n1 = E.KIND_PARAMS[kind]
    F = 64
    inits = rng.integers(0, 2 ** 32, F, dtype=np.uint64).astype(np.uint32) | 3
    t1 = rng.integers(0, 2, (F, n1)).astype(np.uint8)
    t5 = np.zeros((F, K), np.uint8)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_encode_blocks(c.handle, _hip.ptr(t1), F, kind, _hip.ptr(inits), _hip.ptr(t5)))
    for f in range(F):
        assert np.array_equal(t5[f], E.encode_block(t1[f], kind, E.scramble_seq(int(inits[f]), K)))
    soft = (np.where(t5 == 0, 40, -40) + rng.normal(0, 16, t5.shape)).clip(-127, 127).astype(np.int8)
    soft[F // 2:] = rng.integers(-127, 128, (F - F // 2, K)).astype(np.int8)   # pure noise: ties, CRC fails
    dec = np.zeros((F, n1), np.uint8)
    ok = np.zeros(F, np.uint8)
    c.check(c.lib.tetra_etsi_decode_blocks(c.handle, _hip.ptr(soft), F, kind, _hip.ptr(inits), _hip.ptr(dec),
                                           _hip.ptr(ok)))
    for f in range(F):
        bits, o = E.Receiver.decode_block(soft[f], kind, E.scramble_seq(int(inits[f]), K))
        assert np.array_equal(dec[f], bits) and bool(ok[f]) == o, f
    assert ok[:F // 2].mean() > 0.9


def test_process_and_decode_surface():
    """SignalProcessor(mode='etsi').process -> TetraDecoder(mode='etsi').decode round trip with no
    cell configured: four consecutive chunks of one capture through one decoder, which acquires the
    cell from a BSCH and keeps it.  Frames carry the reference's frame-dict keys."""
    from tetraear.signal import SignalProcessor
    from tetraear.core import TetraDecoder
    from tetraear.signal.etsi import synth
    iq, cells, kinds, payload, t0 = synth(1, 4 * 131072, seed=11, snr_db=20.0, cfo_max=300.0)
    p = SignalProcessor(2.4e6, mode="etsi")
    d = TetraDecoder(mode="etsi")
    sent = {tuple(x) for bb in payload[0] for x in bb}
    oks = []
    for k in range(4):
        hard = p.process(iq[0, k * 131072:(k + 1) * 131072])
        assert hard.dtype == np.uint8 and len(p.symbols) == len(hard) + 1
        frames = d.decode(hard)
        for f in frames:
            for key in ("type", "type_name", "number", "timeslot", "bits", "header", "position", "encrypted",
                        "encryption_algorithm", "key_id", "additional_info", "burst_crc"):
                assert key in f, key
            # the MAC stage ran once per CRC-good SCH/F / SCH/HD block (never on the BSCH)
            assert len(f["mac_pdus"]) <= sum(b["channel"] != "BSCH" and b["crc_ok"] for b in f["blocks"])
        oks += [b for f in frames for b in f["blocks"] if b["crc_ok"]]
    assert len(oks) >= 2
    assert all(tuple(np.pad(b["bits"], (0, 268 - len(b["bits"])))) in sent for b in oks)
    from tetraear.core.etsi import cell_of
    if any(b["channel"] == "BSCH" for b in oks):   # a sync burst decoded: the cell is the transmitted one
        assert (d._etsi.mcc, d._etsi.mnc, d._etsi.colour_code) == cell_of(int(cells[0]))


def test_cell_acquisition_vs_oracle(synth_small):
    """tetra_lmac_etsi_acquire (no cell given): BSCH first with colour code 0, the cell from the
    last CRC-good SYNC PDU, then SCH/F + SCH/HD with it -- block for block equal to the oracle's
    restatement (etsi.Receiver.lower_mac_acquire), the acquired inits equal to the oracle's, and
    to the synthesised cell wherever a BSCH decoded."""
    from tetraear.signal.etsi import EtsiReceiver
    from tetraear.core.etsi import EtsiLowerMac, UNKNOWN_CELL
    iq, cells, kinds, payload, t0 = synth_small
    hard, soft, sym, ns = EtsiReceiver().demod_batch(iq)
    lm = EtsiLowerMac()
    res = lm.decode_batch(soft, hard, ns)
    rx = E.Receiver()
    nacq = nok = 0
    for ch in range(len(iq)):
        n = int(ns[ch])
        want, init = rx.lower_mac_acquire(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], UNKNOWN_CELL)
        assert int(lm.cell_state[ch]) == init, ch
        if init != UNKNOWN_CELL:
            nacq += 1
            assert init == int(cells[ch]), ch
        got = res[ch]
        assert [(f["position"], f["burst_kind"]) for f in got] == [(s, k) for s, k, _ in want], ch
        for f, (_, _, dec) in zip(got, want):
            for b, (kind, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), ch
                nok += ok
    assert nacq >= 2 and nok >= 6


def test_cell_acquisition_stream():
    """A 4-chunk capture per channel decoded chunk by chunk with no cell configured: the cell is
    acquired from the first CRC-good BSCH and kept by the next chunks; every acquired cell is the
    transmitted one; >= 97 % of the blocks of chunks decoded with the cell known pass the CRC; the
    oracle's restatement carried across the same chunks gives the same inits and blocks."""
    from tetraear.signal.etsi import synth, EtsiReceiver
    from tetraear.core.etsi import EtsiLowerMac, UNKNOWN_CELL
    C, L, K = 48, 131072, 4
    iq, cells, kinds, payload, t0 = synth(C, K * L, seed=23, snr_db=18.0, cfo_max=600.0)
    rx, lm, orc = EtsiReceiver(), EtsiLowerMac(), E.Receiver()
    state = [UNKNOWN_CELL] * C
    nblk = nok = 0
    for k in range(K):
        hard, soft, sym, ns = rx.demod_batch(iq[:, k * L:(k + 1) * L])
        known_before = np.array([int(v) != UNKNOWN_CELL for v in lm.cell_state]) if lm.cell_state is not None \
            else np.zeros(C, bool)
        res = lm.decode_batch(soft, hard, ns)
        for ch in range(C):
            n = int(ns[ch])
            want, state[ch] = orc.lower_mac_acquire(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], state[ch])
            assert int(lm.cell_state[ch]) == state[ch], (k, ch)
            if state[ch] != UNKNOWN_CELL:
                assert state[ch] == int(cells[ch]), (k, ch)
            if ch % 8 == 0:
                assert [[(b["crc_ok"], tuple(b["bits"])) for b in f["blocks"]] for f in res[ch]] == \
                    [[(bool(ok), tuple(bits)) for _, bits, ok in dec] for _, _, dec in want], (k, ch)
            if known_before[ch] or state[ch] != UNKNOWN_CELL:
                for f in res[ch]:
                    for b in f["blocks"]:
                        nblk += 1
                        nok += b["crc_ok"]
    acquired = sum(int(v) != UNKNOWN_CELL for v in lm.cell_state)
    assert acquired >= 0.85 * C, acquired
    assert nok / nblk >= 0.97, (nok, nblk)


def test_etsi_surface_methods():
    """ETSI mode's component methods: demodulate_dqpsk = Table 5.1 decisions on given symbols
    (ideal constellation walk decoded exactly; bit-identical to the oracle's eo_decide on the
    receiver's symbols); filter_signal / extract_symbols = the channel filter and timing stages,
    whose composition is process()."""
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import synth
    p = SignalProcessor(2.4e6, mode="etsi")
    rng = np.random.default_rng(4)
    bits = rng.integers(0, 2, 2 * 999)
    steps = np.where(bits[0::2] == 0, np.where(bits[1::2] == 0, 1, 3), np.where(bits[1::2] == 0, -1, -3))
    x = np.exp(1j * (0.3 + np.pi / 4 * np.concatenate([[0], np.cumsum(steps)]))).astype(np.complex64)
    want = (bits[0::2] * 2 + bits[1::2]).astype(np.uint8)
    assert np.array_equal(p.demodulate_dqpsk(x), want)
    assert np.array_equal(p.demodulate_dqpsk(x.astype(np.complex128)), want)
    assert len(p.demodulate_dqpsk(x[:1])) == 0
    iq = synth(1, 131072, seed=13, snr_db=15.0)[0][0]
    hard = p.process(iq)
    sym = p.symbols
    assert np.array_equal(p.demodulate_dqpsk(sym), E.Receiver.decide(sym))
    assert np.mean(p.demodulate_dqpsk(sym) == hard) > 0.9   # the fused decision also corrects the CFO
    y = p.filter_signal(iq)
    assert np.array_equal(y, E.Receiver().chanfilt(iq))
    assert np.array_equal(p.extract_symbols(y), sym)
    assert np.array_equal(p.extract_symbols(iq, sample_rate=2.4e6), sym)


def test_env_selects_etsi_chain(monkeypatch):
    """TETRAEAR_DEMOD=etsi: the reference's unchanged construction calls
    (SignalProcessor(sample_rate=...), TetraDecoder(auto_decrypt=...), modern.py:1886-1887) run the
    north-star chain."""
    from tetraear.signal import SignalProcessor
    from tetraear.core import TetraDecoder
    from tetraear.signal.etsi import synth
    monkeypatch.setenv("TETRAEAR_DEMOD", "etsi")
    p = SignalProcessor(sample_rate=2.4e6)
    d = TetraDecoder(auto_decrypt=False)
    assert p.mode == "etsi" and d.mode == "etsi"
    iq = synth(1, 131072, seed=11, snr_db=20.0, cfo_max=300.0)[0][0]
    hard = p.process(iq)
    assert hasattr(hard, "soft_bits") and len(hard.soft_bits) == 2 * len(hard)
    frames = d.decode(hard)
    assert all("blocks" in f for f in frames)


def test_full_size_round_trip():
    """Bench-shaped batch (2.4 MSps, 131072-sample chunks): round-trip property at scale."""
    from tetraear.signal.etsi import synth, EtsiReceiver
    from tetraear.core.etsi import EtsiLowerMac
    C = 256
    iq, cells, kinds, payload, t0 = synth(C, 131072, seed=5, snr_db=18.0, cfo_max=600.0)
    hard, soft, sym, ns = EtsiReceiver().demod_batch(iq)
    res = EtsiLowerMac().decode_batch(soft, hard, ns, cells)
    nblk = nok = 0
    for ch in range(C):
        sent = {tuple(p) for bb in payload[ch] for p in bb}
        for f in res[ch]:
            for b in f["blocks"]:
                nblk += 1
                if b["crc_ok"]:
                    nok += 1
                    assert tuple(np.pad(b["bits"], (0, 268 - len(b["bits"])))) in sent
    assert nblk >= 3 * C
    assert nok / nblk > 0.97, (nok, nblk)


def test_bench_pipeline_matches_serial(monkeypatch):
    """bench.py's step variants give the same per-step results as the single-stream fused chain:
    the two-stream pipeline (front: fused demod, back: lower MAC, double-buffered symbol outputs),
    the same with consecutive demods on two front streams (TETRA_ETSI_FRONT2=1), the split demod
    (chanfilt -> y in HBM -> timing) pipelined, and the host-fed (PCIe) mode; the SC16 pipeline
    against the SC16 single-stream chain."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import BenchStep
    dev = torch.device("cuda", 0)
    # a context of this test's own: tetra_set_stream(None) puts it on the null stream (torch's
    # current stream, where BenchStep's torch buffers are made), which must not leak into the
    # shared thread-local context the other tests use
    c = _hip.Context()
    c.check(c.lib.tetra_set_stream(c.handle, None), "set_stream")
    outs = {"cf32": [], "sc16": []}   # SC16 steps compare among themselves (other input)
    for pipe, demod, host, fmt, f2 in ((False, "fused", False, "cf32", "0"), (True, "fused", False, "cf32", "0"),
                                       (True, "fused", False, "cf32", "1"), (True, "split", False, "cf32", "0"),
                                       (True, "fused", True, "cf32", "0"), (False, "split", True, "cf32", "0"),
                                       (True, "fused", False, "sc16", "0"), (False, "fused", False, "sc16", "0")):
        monkeypatch.setenv("TETRA_ETSI_FRONT2", f2)
        st = BenchStep(c, 64, 131072, 2.4e6, seed=11, device=dev, demod=demod, iq_format=fmt)
        if pipe:
            st.pipeline()
            assert len(st.contexts()) == 2 + (f2 == "1")
        if host:
            st.host_feed()
        for _ in range(3):
            st()
        torch.cuda.synchronize(dev)
        soft, hard, ns = st.soft.cpu(), st.hard.cpu(), st.nsym.cpu()
        nb, bursts, nk, blocks, t1 = st.nburst.cpu(), st.bursts.cpu(), st.nblock.cpu(), st.blocks.cpu(), st.type1.cpu()
        # the written parts only (the buffers are torch.empty: padding differs between instances)
        n1 = {0: 268, 1: 124, 2: 60}   # type-1 bits per block kind (the rest of a type1 row is padding)
        outs[fmt].append([ns, nb, nk] + [x for ch in range(64) for x in (
            soft[ch, :2 * max(int(ns[ch]) - 1, 0)], hard[ch, :max(int(ns[ch]) - 1, 0)], bursts[ch, :int(nb[ch])],
            blocks[ch, :int(nk[ch])])] + [t1[ch, j, :n1[int(blocks[ch, j, 0])]] for ch in range(64)
                                          for j in range(int(nk[ch]))])
        assert st.quality()["crc_ok"] > 64
    for group in outs.values():
        for o in group[1:]:
            for a, b in zip(group[0], o):
                assert torch.equal(a, b)


@pytest.mark.parametrize("N", [131072, 70002, 20000, 3000])
def test_sc16_chanfilt_component_vs_oracle(N):
    """tetra_etsi_chanfilt_fmt on SC16 (y written to HBM: k_chanfilt_r<.., false>, or k_chanfilt<uint2>
    for rows that are not a multiple of four samples) equals the oracle's channel filter on the
    1/32768-scaled samples, bit for bit."""
    from tetraear import _hip
    from tetraear.signal.etsi import synth, EtsiReceiver, lengths
    C = 3
    iq = synth(C, N, seed=21, snr_db=20.0)[0]
    q = np.stack([np.round(iq.real * 32768), np.round(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
    x = (q[..., 0].astype(np.float32) / 32768 + 1j * (q[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    rx = EtsiReceiver()
    _, M2, _ = lengths(rx.plan, N)
    y = np.zeros((C, M2), np.complex64)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_chanfilt_fmt(c.handle, rx.plan, _hip.ptr(np.ascontiguousarray(q)), _hip.TETRA_SC16, C, N,
                                          _hip.ptr(y)), "chanfilt_fmt")
    o = E.Receiver()
    for ch in range(C):
        assert np.array_equal(y[ch], o.chanfilt(x[ch])), ch


def test_sc16_ingest_matches_cf32(synth_small):
    """SC16 (int16 I/Q, the BladeRF wire format) filtered straight from 4 B/sample equals the
    cf32 path on the same samples scaled by 1/32768 (capture.py:241-269), bit for bit."""
    from tetraear.signal.etsi import EtsiReceiver
    iq = synth_small[0]
    q = np.stack([np.round(iq.real * 32768), np.round(iq.imag * 32768)], -1).astype(np.int16)
    x = (q[..., 0].astype(np.float32) / 32768 + 1j * (q[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    rx = EtsiReceiver()
    a = rx.demod_batch(x)
    b = rx.demod_batch(q)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
    # odd-length and minimum-length rows take the same path
    c = rx.demod_batch(q[:2, :9001])
    d = rx.demod_batch(x[:2, :9001])
    for u, v in zip(c, d):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("fmt", ["cf32", "sc16"])
@pytest.mark.parametrize("N", [262144, 134408, 131072, 70002, 70001, 40000, 23408, 20000, 9001, 3000])
def test_demod_lengths_vs_oracle(N, fmt):
    """Chunk lengths around the kernels' structure: longer than the fused path's LDS output buffer
    (component path; 134408 gives 4000 outputs, just past YLDS = 3904), the 128 Ki design point (fused; SC16 on
    k_chanfilt_r, register stage 1; 70002, a row of SC16 not a multiple of four samples, on k_chanfilt<uint2>,
    which re-stages y into the freed image and stage-1 buffer), mid lengths on the per-wave cf32 filter (odd wave-tile counts, quarters that
    end mid-tile), short (the per-wave filter on fewer than four waves), odd (trimmed to even like
    demod_batch does), and barely long enough -- for both input formats (SC16 against the oracle on
    its 1/32768-scaled samples)."""
    from tetraear.signal.etsi import synth, EtsiReceiver
    C = 3
    iq = synth(C, 262144, seed=9, snr_db=20.0)[0][:, :N]
    inp = iq
    if fmt == "sc16":
        inp = np.stack([np.round(iq.real * 32768), np.round(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
        iq = (inp[..., 0].astype(np.float32) / 32768 + 1j * (inp[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    rx = E.Receiver()
    hard, soft, sym, ns = EtsiReceiver().demod_batch(inp)
    Ne = N - N % 2
    for ch in range(C):
        so, sbo, ho, _ = rx.demod(iq[ch, :Ne])
        n = int(ns[ch])
        assert n == len(so), (N, ch)
        assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :max(n - 1, 0)], ho)
        assert np.array_equal(soft[ch, :2 * max(n - 1, 0)], sbo)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [0, 1, 2, 47, 48, 400, 3300, 3301, 3500])
def test_process_edge_lengths(N):
    """process() on empty, one-sample, sub-filter and barely-demodulable chunks: the same symbols
    as the oracle (empty where the oracle has none), never an exception -- the reference's
    process() returns an empty uint8 array for an empty chunk (processor.py:239-241)."""
    from tetraear.signal import SignalProcessor
    x = (0.2 * np.random.default_rng(N).standard_normal(N) + 0j).astype(np.complex64)
    p = SignalProcessor(2.4e6, mode="etsi")
    hard = p.process(x)
    assert hard.dtype == np.uint8
    so, sbo, ho, _ = E.Receiver().demod(x[:N - N % 2])
    if len(so) < 2:
        assert len(hard) == 0
    else:
        assert np.array_equal(np.asarray(hard), ho) and np.array_equal(p.symbols, so)
        assert np.array_equal(hard.soft_bits, sbo)


@pytest.mark.gpu
def test_lower_mac_empty_and_low_snr():
    """The lower MAC beside channels with no symbols (0 and 1): those give no bursts; two channels
    demodulated at 6 dB Es/N0 (marginal: bursts found, CRCs failing) match the oracle block
    for block."""
    from tetraear.core.etsi import EtsiLowerMac
    from tetraear.signal.etsi import synth, EtsiReceiver
    iq, cells2, _, _, _ = synth(2, 131072, seed=21, snr_db=6.0)
    h2, s2, _, n2 = EtsiReceiver().demod_batch(iq)
    sm = h2.shape[1]
    hard = np.concatenate([np.zeros((2, sm), np.uint8), h2])
    soft = np.concatenate([np.zeros((2, 2 * sm), np.int8), s2])
    ns = np.concatenate([np.array([0, 1], np.int32), n2])
    cells = np.concatenate([np.array([3, 7], np.uint32), cells2])
    res = EtsiLowerMac().decode_batch(soft, hard, ns, cells)
    assert res[0] == [] and res[1] == []
    rx = E.Receiver()
    nfail = nblk = 0
    for ch in (2, 3):
        n = int(ns[ch])
        want = rx.lower_mac(soft[ch, :2 * (n - 1)], hard[ch, :n - 1], int(cells[ch]))
        got = res[ch]
        assert len(got) == len(want)
        for f, (start, bk, blocks) in zip(got, want):
            assert f["position"] == start and f["burst_kind"] == bk
            assert [b["crc_ok"] for b in f["blocks"]] == [bool(ok) for _, _, ok in blocks]
            for b, (_, t1, _) in zip(f["blocks"], blocks):
                assert np.array_equal(b["bits"], t1)
                nblk += 1
                nfail += not b["crc_ok"]
    assert nblk > 0


@pytest.mark.parametrize("extra", [1, 2, 3, 4])
def test_lower_mac_row_alignments(synth_small, extra):
    """The Viterbi loads a block as aligned dwords and realigns them (load_seg): rows of odd and even
    width (row bases at every byte alignment mod 4), each channel's symbols shifted to END at its
    row's end, so the last channel's last blocks reach the buffer's final bytes.  Block for block
    equal to the oracle on the same rows."""
    from tetraear.signal.etsi import EtsiReceiver
    from tetraear.core.etsi import EtsiLowerMac
    iq, cells, _, _, _ = synth_small
    hard, soft, _, ns = EtsiReceiver().demod_batch(iq)
    C = len(iq)
    sm = int(ns.max()) + extra
    h2 = np.zeros((C, sm), np.uint8)
    s2 = np.zeros((C, 2 * sm), np.int8)
    ns2 = np.full(C, sm, np.int32)
    for ch in range(C):
        n = int(ns[ch])
        pad = sm - n
        h2[ch, pad:pad + n - 1] = hard[ch, :n - 1]
        s2[ch, 2 * pad:2 * (pad + n - 1)] = soft[ch, :2 * (n - 1)]
    res = EtsiLowerMac().decode_batch(s2, h2, ns2, cells)
    rx = E.Receiver()
    nblk = 0
    for ch in range(C):
        want = rx.lower_mac(s2[ch, :2 * (sm - 1)], h2[ch, :sm - 1], int(cells[ch]))
        got = res[ch]
        assert [(f["position"], f["burst_kind"]) for f in got] == [(s, k) for s, k, _ in want], ch
        for f, (_, _, dec) in zip(got, want):
            for b, (_, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), ch
                nblk += 1
    assert nblk >= 12


def test_lower_mac_unaligned_device_buffers(synth_small):
    """tetra_lmac_etsi on caller-owned device buffers at odd offsets (soft bits and type-1 bits at byte
    offset 1, burst / block records at 4 bytes): the same results as the host-buffer call."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import EtsiReceiver
    iq, cells, _, _, _ = synth_small
    hard, soft, _, ns = EtsiReceiver().demod_batch(iq)
    C, sm = hard.shape
    MB, MJ = _hip.ETSI_MAXB, _hip.ETSI_MAXJ
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(np.ascontiguousarray(cells, np.uint32)), C))

    def run(dev):
        if not dev:
            outs = [np.zeros(C, np.int32), np.zeros((C, MB, 2), np.int32), np.zeros(C, np.int32),
                    np.zeros((C, MJ, 4), np.int32), np.zeros((C, MJ, 268), np.uint8)]
            ins = [soft, hard, ns]
            ptrs = [_hip.ptr(a) for a in ins + outs]
        else:
            d = torch.device("cuda:0")
            sb = torch.zeros(C * 2 * sm + 1, dtype=torch.int8, device=d)
            sb[1:] = torch.from_numpy(soft.reshape(-1))
            hd = torch.from_numpy(hard.reshape(-1)).to(d)
            nsd = torch.from_numpy(ns).to(d)
            i32 = [torch.zeros(n + 1, dtype=torch.int32, device=d) for n in (C, C * MB * 2, C, C * MJ * 4)]
            t1 = torch.zeros(C * MJ * 268 + 1, dtype=torch.uint8, device=d)
            ptrs = [sb.data_ptr() + 1, hd.data_ptr(), nsd.data_ptr()] + [t.data_ptr() + 4 for t in i32] + \
                [t1.data_ptr() + 1]
            outs = (i32, t1)
        c.check(c.lib.tetra_lmac_etsi(c.handle, ptrs[0], ptrs[1], ptrs[2], C, sm, *ptrs[3:]))
        if dev:
            torch.cuda.synchronize()
            i32, t1 = outs
            return [t[1:].cpu().numpy() for t in i32] + [t1[1:].cpu().numpy()]
        return [o.reshape(-1) for o in outs]

    want, got = run(False), run(True)
    # compared over the entries the call writes (the host-buffer path copies back the rest unset)
    assert np.array_equal(want[0], got[0]) and np.array_equal(want[2], got[2])
    nb, nk = want[0], want[2]
    wb, gb = want[1].reshape(C, MB, 2), got[1].reshape(C, MB, 2)
    wk, gk = want[3].reshape(C, MJ, 4), got[3].reshape(C, MJ, 4)
    wt, gt = want[4].reshape(C, MJ, 268), got[4].reshape(C, MJ, 268)
    ngood = 0
    for ch in range(C):
        assert np.array_equal(wb[ch, :nb[ch]], gb[ch, :nb[ch]])
        assert np.array_equal(wk[ch, :nk[ch]], gk[ch, :nk[ch]])
        for j in range(nk[ch]):
            n1 = E.KIND_PARAMS[int(wk[ch, j, 0])][3]
            assert np.array_equal(wt[ch, j, :n1], gt[ch, j, :n1]), (ch, j)
            ngood += int(wk[ch, j, 1])
    assert ngood >= 12


def test_fused_demod_many_channels():
    """The fused cf32 demod over more channels than the chip holds workgroups at once (two per CU: the
    grid runs in three waves of workgroups): bit-identical to the component path (chanfilt -> y in HBM
    -> k_timing) for every channel, and to the oracle for channels of the second and third waves."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths
    dev = torch.device("cuda", 0)
    G = 2 * torch.cuda.get_device_properties(0).multi_processor_count
    C, N = 2 * G + 37, 131072
    c = _hip.ctx()
    plan = etsi_plan()
    _, M2, smax = lengths(plan, N)
    iq = torch.empty((C, N, 2), dtype=torch.float32, device=dev)
    nb = c.lib.tetra_synth_bursts_per_channel(N, 2.4e6)
    cells = torch.empty(C, dtype=torch.int32, device=dev)
    kinds = torch.empty((C, nb), dtype=torch.int32, device=dev)
    pay = torch.empty((C, nb, 2, 268), dtype=torch.uint8, device=dev)
    c.check(c.lib.tetra_synth_etsi(c.handle, C, N, 2.4e6, 77, 16.0, 600.0, _hip.ptr(iq), _hip.ptr(cells),
                                   _hip.ptr(kinds), _hip.ptr(pay), None), "synth")

    def outs():
        return (torch.zeros((C, smax, 2), dtype=torch.float32, device=dev),
                torch.zeros((C, 2 * smax), dtype=torch.int8, device=dev),
                torch.zeros((C, smax), dtype=torch.uint8, device=dev),
                torch.zeros(C, dtype=torch.int32, device=dev),
                torch.zeros((C, 4), dtype=torch.float32, device=dev))
    a = outs()
    c.check(c.lib.tetra_demod_etsi_fmt(c.handle, plan, _hip.ptr(iq), _hip.TETRA_CF32, C, N, *[_hip.ptr(t) for t in a[:4]],
                                       smax, _hip.ptr(a[4])), "demod")
    y = torch.empty((C, M2, 2), dtype=torch.float32, device=dev)
    c.check(c.lib.tetra_etsi_chanfilt(c.handle, plan, _hip.ptr(iq), C, N, _hip.ptr(y)), "chanfilt")
    bo = outs()
    c.check(c.lib.tetra_etsi_timing(c.handle, plan, _hip.ptr(y), C, M2, *[_hip.ptr(t) for t in bo[:4]], smax,
                                    _hip.ptr(bo[4])), "timing")
    torch.cuda.synchronize(dev)
    assert torch.equal(a[3], bo[3]) and int(a[3].min()) > 900
    assert torch.equal(a[0], bo[0]) and torch.equal(a[2], bo[2]) and torch.equal(a[4], bo[4])
    assert torch.equal(a[1], bo[1])
    rx = E.Receiver()
    for ch in (3, G + 5, 2 * G + 1, C - 1):
        x = iq[ch].cpu().numpy().view(np.complex64)[:, 0]
        so, sbo, ho, _ = rx.demod(x)
        n = int(a[3][ch])
        assert n == len(so), ch
        sym = a[0][ch, :n].cpu().numpy().view(np.complex64)[:, 0]
        assert np.array_equal(sym, so) and np.array_equal(a[2][ch, :n - 1].cpu().numpy(), ho), ch
        assert np.array_equal(a[1][ch, :2 * (n - 1)].cpu().numpy(), sbo), ch


def test_c4_full_chain_4096_bursts():
    """BASELINE configs[3] (C4): the full receive chain -- channel filter, timing, decision, burst
    sync, descramble, deinterleave, RCPC Viterbi, CRC -- over >= 4096 synthetic TETRA bursts on one
    GPU (bench.py's step on a C4-sized batch): every CRC-passing block carries a transmitted
    payload, >= 97 % of the blocks pass at 18 dB Es/N0, and a sample of channels matches the oracle
    burst for burst and bit for bit."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import BenchStep
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    C, N = 1536, 131072   # ~2.8 complete bursts per 131072-sample chunk
    st = BenchStep(c, C, N, 2.4e6, seed=44, device=dev, cells="given")
    st()
    torch.cuda.synchronize(dev)
    nb = st.nburst.cpu().numpy()
    assert int(nb.sum()) >= 4096, int(nb.sum())
    nk, blocks, t1 = st.nblock.cpu().numpy(), st.blocks.cpu().numpy(), st.type1.cpu().numpy()
    payload = st.payload.cpu().numpy()
    n1 = {0: 268, 1: 124, 2: 60}
    nblk = nok = 0
    for ch in range(C):
        sent = {tuple(p) for bb in payload[ch] for p in bb}
        for j in range(int(nk[ch])):
            kind, ok = int(blocks[ch, j, 0]), int(blocks[ch, j, 1])
            nblk += 1
            if ok:
                nok += 1
                bits = np.pad(t1[ch, j, :n1[kind]], (0, 268 - n1[kind]))
                assert tuple(bits) in sent, (ch, j)
    assert nok / nblk > 0.97, (nok, nblk)
    # oracle, burst for burst, on a sample of channels
    rx = E.Receiver()
    soft, hard, ns = st.soft.cpu().numpy(), st.hard.cpu().numpy(), st.nsym.cpu().numpy()
    cells = st.cells.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    iq = st.iq
    for ch in (0, 511, 1024, C - 1):
        x = iq[ch].cpu().numpy().view(np.complex64)[:, 0]
        so, sbo, ho, _ = rx.demod(x)
        n = int(ns[ch])
        assert n == len(so) and np.array_equal(hard[ch, :n - 1], ho) and np.array_equal(soft[ch, :2 * (n - 1)], sbo)
        want = rx.lower_mac(sbo, ho, int(cells[ch]))
        assert len(want) == int(nb[ch])
        k = 0
        for start, bk, blks in want:
            for _, tb, okb in blks:
                assert int(blocks[ch, k, 1]) == int(bool(okb))
                assert np.array_equal(t1[ch, k, :len(tb)], tb)
                k += 1
        assert k == int(nk[ch])
    # the same batch through the acquiring lower MAC (one chunk, no earlier state): a channel acquires its cell
    # from a sync burst in the chunk, and every block of a channel that did decodes as with the cell given
    acq = BenchStep(c, C, N, 2.4e6, seed=44, device=dev, cells="acquire")
    acq()
    torch.cuda.synchronize(dev)
    state = acq.cell_state.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    ab, at1 = acq.blocks.cpu().numpy(), acq.type1.cpu().numpy()
    bursts = st.bursts.cpu().numpy()
    nacq = 0
    for ch in range(C):
        has_sb = any(int(bursts[ch, b, 1]) == 2 for b in range(int(nb[ch])))
        sb_ok = False
        q = 0
        for b in range(int(nb[ch])):
            if int(bursts[ch, b, 1]) == 2 and blocks[ch, q, 1]:
                sb_ok = True
            q += 1 if int(bursts[ch, b, 1]) == 0 else 2
        assert (state[ch] == cells[ch]) == sb_ok or (not has_sb and state[ch] == 3), ch
        if sb_ok:
            nacq += 1
            assert np.array_equal(ab[ch, :int(nk[ch])], blocks[ch, :int(nk[ch])]), ch
            for j in range(int(nk[ch])):
                n1j = n1[int(blocks[ch, j, 0])]
                assert np.array_equal(at1[ch, j, :n1j], t1[ch, j, :n1j]), (ch, j)
    assert nacq >= C // 3   # ~2.8 bursts per chunk, a quarter of them sync bursts


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_block_codec_vs_independent_spec(kind):
    """The GPU encoder equals the independent spec restatement (oracle/etsi_spec.py, which shares
    no code with etsi_oracle.c), and every CRC-good block the GPU decoder returns is a maximum-
    likelihood codeword: its re-encoding correlates with the received soft bits at least as well as
    the transmitted one (scored by the spec encoder)."""
    import etsi_spec as S
    from tetraear import _hip
    rng = np.random.default_rng(30 + kind)
    n1, K = S.KINDS[kind]["n1"], S.KINDS[kind]["K"]
    F = 96
    inits = ((rng.integers(0, 2 ** 30, F).astype(np.uint64) << 2) | 3).astype(np.uint32)
    t1 = rng.integers(0, 2, (F, n1)).astype(np.uint8)
    t5 = np.zeros((F, K), np.uint8)
    c = _hip.ctx()
    c.check(c.lib.tetra_etsi_encode_blocks(c.handle, _hip.ptr(t1), F, kind, _hip.ptr(inits), _hip.ptr(t5)))
    for f in range(F):
        assert np.array_equal(t5[f], S.encode(t1[f], kind, int(inits[f]))), f
    sigma = np.where(np.arange(F) % 3 == 0, 24.0, 16.0)[:, None]   # 65-88 of 96 blocks CRC-good
    soft = np.clip(np.rint(np.where(t5 == 0, 32.0, -32.0) + rng.normal(0, 1, t5.shape) * sigma), -127, 127)
    soft = soft.astype(np.int8)
    dec = np.zeros((F, n1), np.uint8)
    ok = np.zeros(F, np.uint8)
    c.check(c.lib.tetra_etsi_decode_blocks(c.handle, _hip.ptr(soft), F, kind, _hip.ptr(inits), _hip.ptr(dec),
                                           _hip.ptr(ok)))
    ngood = 0
    for f in range(F):
        if ok[f]:   # a CRC-good block's path is type-1 + its CRC + zero tail
            ngood += 1
            m_dec = S.codeword_metric(soft[f], S.type2(dec[f]), kind, int(inits[f]))
            m_tx = S.codeword_metric(soft[f], S.type2(t1[f]), kind, int(inits[f]))
            assert m_dec >= m_tx, (f, m_dec, m_tx)
    assert ngood >= F // 2


def _check_blocks_transmitted(st, C):
    """(blocks, CRC-good) of the step's last batch; asserts every CRC-good block's type-1 bits are
    one of the channel's transmitted payloads (vectorised over a channel's payload rows)."""
    nk, blocks, t1 = st.nblock.cpu().numpy(), st.blocks.cpu().numpy(), st.type1.cpu().numpy()
    payload = st.payload.cpu().numpy()
    n1 = np.array([268, 124, 60])
    nblk = nok = 0
    for ch in range(C):
        k = int(nk[ch])
        nblk += k
        sent = payload[ch].reshape(-1, 268)
        for j in range(k):
            if blocks[ch, j, 1]:
                nok += 1
                bits = t1[ch, j].copy()
                bits[n1[int(blocks[ch, j, 0])]:] = 0
                assert np.any(np.all(sent == bits[None, :], axis=1)), (ch, j)
    return nblk, nok


def test_c5_full_shard_8192x131072():
    """BASELINE configs[4] (C5) at its per-GPU shard, the bench's own step: 8192 channels x 131072 cf32
    samples (8.6 GB resident in HBM).  Every CRC-good block carries a transmitted payload, >= 97 % of
    the blocks pass at 18 dB Es/N0, and channels 0, 4095 and 8191 equal the oracle burst for burst
    and bit for bit (soft symbols, soft bits, hard dibits, decoded type-1 bits, CRC flags)."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import BenchStep
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    C, N = 8192, 131072
    st = BenchStep(c, C, N, 2.4e6, seed=1000, device=dev, cells="given")   # bench.py's rank-0 seed
    st()
    torch.cuda.synchronize(dev)
    nblk, nok = _check_blocks_transmitted(st, C)
    assert nblk >= 3 * C and nok / nblk >= 0.97, (nok, nblk)
    rx = E.Receiver()
    soft, hard, ns = st.soft.cpu().numpy(), st.hard.cpu().numpy(), st.nsym.cpu().numpy()
    sym = st.sym.cpu().numpy()
    nb, blocks, t1 = st.nburst.cpu().numpy(), st.blocks.cpu().numpy(), st.type1.cpu().numpy()
    cells = st.cells.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    for ch in (0, 4095, 8191):
        x = st.iq[ch].cpu().numpy().view(np.complex64)[:, 0]
        so, sbo, ho, _ = rx.demod(x)
        n = int(ns[ch])
        assert n == len(so) and np.array_equal(sym[ch, :n].view(np.complex64)[:, 0], so), ch
        assert np.array_equal(hard[ch, :n - 1], ho) and np.array_equal(soft[ch, :2 * (n - 1)], sbo), ch
        want = rx.lower_mac(sbo, ho, int(cells[ch]))
        assert len(want) == int(nb[ch]), ch
        k = 0
        for start, bk, blks in want:
            for _, tb, okb in blks:
                assert int(blocks[ch, k, 1]) == int(bool(okb)) and np.array_equal(t1[ch, k, :len(tb)], tb), (ch, k)
                k += 1
        assert k == int(st.nblock[ch])


def test_acquire_streaming_chunks():
    """bench.py --cells acquire: each channel is one continuous capture of 8 chunks decoded as one
    stream (timing loops carried, the lower MAC resuming on the previous chunk's unconsumed dibits),
    with no cell configured.  By the last chunk every channel whose capture holds a CRC-good sync
    burst has acquired its cell; the last step decodes >= 99 % of the bursts on air and >= 97 % of its
    blocks pass the CRC, each a transmitted payload, with the same bits as the cell-given stream over
    the same capture.  One step past the capture's end restarts it as a new capture (stream_resets)."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import BenchStep
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    C, N, K = 1024, 131072, 8
    acq = BenchStep(c, C, N, 2.4e6, seed=55, device=dev, cells="acquire", chunks=K)
    for _ in range(K):
        acq()
    torch.cuda.synchronize(dev)
    q = acq.quality()
    assert q["chunk"] == K - 1 and q["crc_ok_frac"] >= 0.97 and q["stream_resets"] == 0, q
    assert q["decoded_frac"] >= 0.99, q
    nblk, nok = _check_blocks_transmitted(acq, C)
    assert nok / nblk >= 0.97
    assert q["cells_acquired"] >= int(0.98 * C), q
    blocks_a, t1_a, nk_a = acq.blocks.cpu().numpy(), acq.type1.cpu().numpy(), acq.nblock.cpu().numpy()
    got = acq.cell_state.cpu().numpy() == acq.cells.cpu().numpy()
    acq()   # past the end: a new capture from chunk 0
    torch.cuda.synchronize(dev)
    assert acq.quality()["stream_resets"] == 1
    del acq
    giv = BenchStep(c, C, N, 2.4e6, seed=55, device=dev, cells="given", chunks=K)
    for _ in range(K):
        giv()
    torch.cuda.synchronize(dev)
    nk, blocks_g, t1_g = giv.nblock.cpu().numpy(), giv.blocks.cpu().numpy(), giv.type1.cpu().numpy()
    n1 = (268, 124, 60)   # type-1 bits of SCH/F, SCH/HD, BSCH: the row past them is not written
    for ch in np.nonzero(got)[0]:
        k = int(nk[ch])
        assert k == int(nk_a[ch]), ch
        assert np.array_equal(blocks_a[ch, :k], blocks_g[ch, :k]), ch
        for j in range(k):
            n = n1[int(blocks_g[ch, j, 0])]
            assert np.array_equal(t1_a[ch, j, :n], t1_g[ch, j, :n]), (ch, j)


def test_etsi_frames_mac_per_block():
    """TetraDecoder(mode='etsi') runs the MAC PDU stage once per CRC-good SCH/F / SCH/HD block, in
    order, and never on the BSCH (whose MAC-SYNC layout would read as PDU type / encryption mode) or
    on CRC-failed blocks: the frames' PDUs equal a fresh parser's parse_mac_pdu over exactly those
    blocks in the same order."""
    from tetraear.core import TetraDecoder
    from tetraear.core.etsi import EtsiLowerMac
    from tetraear.core.protocol import TetraProtocolParser
    rng = np.random.default_rng(8)
    res_hdr = np.array([0, 0, 0, 0, 0, 0, 1, 1], np.uint8)   # MAC-RESOURCE, clear (type 00, mode 00)

    def blk(ch, n, ok, head=None):
        b = rng.integers(0, 2, n).astype(np.uint8)
        if head is not None:
            b[:len(head)] = head
        return {"channel": ch, "crc_ok": ok, "bits": b, "block": 0}
    enc = np.array([0, 0, 1, 1], np.uint8)   # a BSCH whose first bits would read as an encrypted MAC-RESOURCE
    raw = [
        {"position": 510, "burst": "SB", "burst_kind": 2, "timeslot": 1,
         "blocks": [blk("BSCH", 60, True, enc), blk("SCH/HD", 124, True, res_hdr)]},
        {"position": 1020, "burst": "NDB (p)", "burst_kind": 1, "timeslot": 2,
         "blocks": [blk("SCH/HD", 124, False, enc), blk("SCH/HD", 124, True, res_hdr)]},
        {"position": 1530, "burst": "NDB (n)", "burst_kind": 0, "timeslot": 3, "blocks": [blk("SCH/F", 268, True)]},
        {"position": 2040, "burst": "NDB (n)", "burst_kind": 0, "timeslot": 0, "blocks": [blk("SCH/F", 268, False)]},
    ]
    for f in raw:
        f["crc_ok"] = all(b["crc_ok"] for b in f["blocks"])
    d = TetraDecoder(mode="etsi")
    d._etsi = EtsiLowerMac()
    frames = d._etsi_frames(raw)
    ref = TetraProtocolParser()
    want = [ref.parse_mac_pdu(b["bits"].astype(np.int64)) for f in raw for b in f["blocks"]
            if b["channel"] != "BSCH" and b["crc_ok"]]
    got = [p for f in frames for p in f["mac_pdus"]]
    assert [(p["type"], p["encrypted"], p["address"], p["length"], p["data"]) for p in got] == \
        [(p.pdu_type.name, p.encrypted, p.address, p.length, p.data) for p in want if p is not None]
    sb = [f for f in frames if f["burst_kind"] == 2]
    assert sb and sb[0]["header"][:8] == "00000011"   # the header is the SCH/HD block's, not the BSCH's
    assert d.protocol_parser.stats["total_bursts"] == 4


CLI_RATES = [1.8e6, 1.9e6, 2.0e6, 2.1e6, 2.2e6, 2.3e6, 2.4e6]   # modern.py:5518-5519, 5630-5638


@pytest.mark.parametrize("fs", CLI_RATES)
def test_every_cli_rate_vs_oracle_and_round_trip(fs):
    """The ETSI chain at each rate the reference's CLI / GUI slider offers (1.8-2.4 MSps, 0.1 MHz
    steps): 64 channels of a 54.6 ms chunk at 18 dB Es/N0.  Soft symbols, soft bits and hard dibits
    bit-identical to the oracle on four channels (cf32 and SC16); >= 97 % of the decoded blocks
    CRC-good, each a transmitted payload.  2.4 MSps runs the fused kernels, the others the
    generic-rate channel filter (k_chanfilt_g) + k_timing."""
    from tetraear import _hip
    from tetraear.signal.etsi import EtsiReceiver, synth, etsi_plan, lengths
    from tetraear.core.etsi import EtsiLowerMac
    N = 2 * int(round(131072 * fs / 2.4e6 / 2))
    C = 64
    iq, cells, kinds, payload, t0 = synth(C, N, fs=fs, seed=int(fs) // 1000, snr_db=18.0)
    rx = EtsiReceiver(fs)
    hard, soft, sym, ns = rx.demod_batch(iq)
    orc = E.Receiver(fs)
    for ch in (0, 1, 31, 63):
        so, sbo, ho, _ = orc.demod(iq[ch])
        n = int(ns[ch])
        assert n == len(so) and 960 < n < 990, (ch, n, len(so))
        assert np.array_equal(sym[ch, :n], so) and np.array_equal(hard[ch, :n - 1], ho), ch
        assert np.array_equal(soft[ch, :2 * (n - 1)], sbo), ch
    # SC16 wire format: the same bits as cf32 of the scaled samples
    sc = np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
    h2, s2, y2, n2 = rx.demod_batch(sc)
    assert np.array_equal(n2, ns) and np.array_equal(y2, sym) and np.array_equal(h2, hard) and np.array_equal(s2, soft)
    res = EtsiLowerMac().decode_batch(soft, hard, ns, cells)
    nblk = nok = 0
    for ch in range(C):
        sent = payload[ch].reshape(-1, 268)
        for f in res[ch]:
            for b in f["blocks"]:
                nblk += 1
                if b["crc_ok"]:
                    nok += 1
                    bits = np.pad(b["bits"], (0, 268 - len(b["bits"])))
                    assert np.any(np.all(sent == bits[None, :], axis=1)), ch
    assert nblk >= 3 * C and nok / nblk >= 0.97, (nok, nblk)
    c = _hip.ctx()
    p = etsi_plan(fs)
    name = ctypes_name(c, p, N)
    assert name == ("k_chanfilt_r" if fs == 2.4e6 else "k_chanfilt_g"), name


def ctypes_name(c, plan, N):
    import ctypes
    name = ctypes.create_string_buffer(64)
    lds = ctypes.c_int64(0)
    c.check(c.lib.tetra_etsi_kernel_info(c.handle, plan, 0, N, 1, name, 64, ctypes.byref(lds)), "kernel_info")
    return name.value.decode()


@pytest.mark.parametrize("fmt", ["cf32", "sc16"])
def test_generic_kernel_equals_fused_at_2400k(fmt):
    """The generic-rate channel filter run on the canonical 2.4 MSps plan (TETRA_ETSI_FORCE_GENERIC)
    gives the same 72 kHz samples as the specialised per-wave kernel (stage 2 on MFMA), and the same
    symbols through k_timing as the fused demod: two independent implementations of eo_chanfilt's
    operation order agree bit for bit (odd chunk lengths included)."""
    from tetraear import _hip
    from tetraear.signal.etsi import etsi_plan, lengths, synth
    for N in (131072, 65538, 20002):
        iq = synth(5, N, seed=N, snr_db=16.0)[0]
        x = iq if fmt == "cf32" else np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(
            -32768, 32767).astype(np.int16)
        f = _hip.TETRA_CF32 if fmt == "cf32" else _hip.TETRA_SC16
        pc, pg = etsi_plan(2.4e6), etsi_plan(2.4e6, force_generic=True)
        _, M2, sm = lengths(pc, N)
        c = _hip.ctx()
        ya, yb = np.zeros((5, M2), np.complex64), np.ones((5, M2), np.complex64)
        c.check(c.lib.tetra_etsi_chanfilt_fmt(c.handle, pc, _hip.ptr(x), f, 5, N, _hip.ptr(ya)), "chanfilt")
        c.check(c.lib.tetra_etsi_chanfilt_fmt(c.handle, pg, _hip.ptr(x), f, 5, N, _hip.ptr(yb)), "chanfilt_g")
        assert np.array_equal(ya, yb), N
        outs = []
        for p in (pc, pg):
            o = (np.zeros((5, sm), np.complex64), np.zeros((5, 2 * sm), np.int8), np.zeros((5, sm), np.uint8),
                 np.zeros(5, np.int32))
            c.check(c.lib.tetra_demod_etsi_fmt(c.handle, p, _hip.ptr(x), f, 5, N, *[_hip.ptr(a) for a in o], sm, None))
            outs.append(o)
        # equal over what the calls define (the symbols [0, nsym), the decisions [0, nsym - 1)): past
        # nsym the outputs are unspecified (k_timing writes zeros there, the fused tail nothing)
        assert np.array_equal(outs[0][3], outs[1][3]), N
        for ch in range(5):
            n = int(outs[0][3][ch])
            assert np.array_equal(outs[0][0][ch, :n], outs[1][0][ch, :n]), (N, ch)
            assert np.array_equal(outs[0][1][ch, :2 * (n - 1)], outs[1][1][ch, :2 * (n - 1)]), (N, ch)
            assert np.array_equal(outs[0][2][ch, :n - 1], outs[1][2][ch, :n - 1]), (N, ch)


def test_unsupported_rate_never_raises_into_the_loop(caplog):
    """SURVEY §5's contract for the north-star chain: a SignalProcessor(mode='etsi') built for a rate
    no channel-filter plan serves (20 MSps is the wideband capture's rate) logs and returns empty
    output, as the reference's process() does when decimation fails (processor.py:253-257); the
    library itself answers such a plan with TETRA_E_INVALID."""
    import logging
    from tetraear import _hip
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import etsi_plan
    p = SignalProcessor(20e6, mode="etsi")
    with caplog.at_level(logging.WARNING):
        out = p.process(np.zeros(131072, np.complex64))
    assert out.dtype == np.uint8 and len(out) == 0 and len(p.symbols) == 0
    assert any("ETSI demodulation unavailable" in r.message for r in caplog.records)
    bad = etsi_plan(1.8e6)
    bad2 = _hip.EtsiPlan.from_buffer_copy(bad)
    bad2.Lp = 5000
    c = _hip.ctx()
    x = np.zeros((1, 131072), np.complex64)
    y = np.zeros((1, 8192), np.complex64)
    assert c.lib.tetra_etsi_chanfilt(c.handle, bad2, _hip.ptr(x), 1, 131072, _hip.ptr(y)) == -1


def test_hard_symbol_decode_rate():
    """TetraDecoder(mode='etsi').decode() on plain uint8 dibits (a caller that kept only process()'s
    hard symbols, not their soft_bits) decodes with +-64 pseudo-soft bits: the Viterbi then runs on
    hard decisions.  Measured against the soft-decision path on the same demodulated chunks: at 18 dB
    Es/N0 both decode >= 97 % of the blocks; at 9 dB the hard path keeps a share of them but never beats
    the soft one by more than noise, and every CRC-good block is a transmitted payload."""
    from tetraear.signal.etsi import EtsiReceiver, synth
    from tetraear.core.etsi import EtsiLowerMac
    C = 48
    rates = {}
    for snr in (18.0, 9.0):
        iq, cells, kinds, payload, t0 = synth(C, 131072, seed=int(snr) + 40, snr_db=snr)
        hard, soft, sym, ns = EtsiReceiver().demod_batch(iq)
        res = {}
        for mode in ("soft", "hard"):
            nblk = nok = 0
            for ch in range(C):
                n = int(ns[ch])
                lm = EtsiLowerMac(*__import__("tetraear.core.etsi", fromlist=["cell_of"]).cell_of(int(cells[ch])))
                frames = lm.decode(hard[ch, :n - 1], soft[ch, :2 * (n - 1)] if mode == "soft" else None)
                sent = payload[ch].reshape(-1, 268)
                for f in frames:
                    for b in f["blocks"]:
                        nblk += 1
                        if b["crc_ok"]:
                            nok += 1
                            bits = np.pad(b["bits"], (0, 268 - len(b["bits"])))
                            assert np.any(np.all(sent == bits[None, :], axis=1)), (snr, mode, ch)
            res[mode] = (nok, nblk)
        rates[snr] = res
    for mode in ("soft", "hard"):
        nok, nblk = rates[18.0][mode]
        assert nblk >= 3 * C and nok / nblk >= 0.97, (mode, nok, nblk)
    (sk, sn), (hk, hn) = rates[9.0]["soft"], rates[9.0]["hard"]
    assert sn == hn and hk <= sk + 2 and hk / hn >= 0.3, rates[9.0]
    print("decode rates (ok, blocks):", rates)
