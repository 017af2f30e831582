"""Wideband channeliser (C3): oracle self-consistency on the CPU, GPU parity.

The reference has no channeliser, so oracle/wideband.py (float64) is the specification.  The GPU
runs the filter bank in fp32 with a rocFFT transform: its 72 kHz output y is held to the oracle
within a tolerance written below; from y on (timing, decision, lower MAC) the chain is the ETSI
one and is compared bit-exactly / by round trip, as in test_gpu_etsi.py.
"""
import numpy as np
import pytest

import wideband as W

# GPU y vs the float64 oracle: fp32 fold + 800-point fp32 FFT + 45-tap fp32 resampler
Y_TOL = 2e-5   # of max |y| over the carriers compared


def test_design_matches_oracle():
    from tetraear.signal.wideband import wb_design
    h, g = wb_design()
    d = W.design()
    assert np.array_equal(h, d["h"]) and np.array_equal(g, d["g"])


def test_oracle_filter_bank_round_trip():
    """synthesis -> analysis recovers a carrier's baseband tone at its own bin (unit gain, right
    frequency sign), and far carriers see nothing."""
    d = W.design()
    M, D = d["M"], d["D"]
    nbb = 300
    s = np.zeros((M, nbb), complex)
    f = 3000.0
    s[5] = np.exp(2j * np.pi * f * np.arange(nbb) / (d["fs"] / D))
    x = W.synthesize(s, d, nbb * D)
    v = W.analysis(x, d)
    seg = v[:, 40:60]
    assert np.allclose(np.abs(seg[5]), 1.0, atol=2e-3)
    assert np.allclose(np.angle(seg[5, 1:] / seg[5, :-1]), 2 * np.pi * f / (d["fs"] / D), atol=1e-6)
    assert np.abs(seg[100]).max() < 1e-5 and np.abs(seg[405]).max() < 1e-5


def test_lengths_match_oracle():
    from tetraear.signal.wideband import wb_plan
    p = wb_plan()
    d = W.design()
    for Nw in (1600, 1601, 20000, 1_100_000, 10_000_000):
        assert p.lengths(Nw) == W.lengths(d, Nw), Nw


def test_chunking_layouts():
    """Overlapping chunks cover every carrier row to its end (each chunk m2 + ov samples but the
    last, which the row's end cuts and which is never longer); ov = 0 is the tiled layout."""
    from tetraear.signal.wideband import BURST_SAMPLES, OV_CHUNK, chunking, wb_plan
    p = wb_plan()
    assert OV_CHUNK >= BURST_SAMPLES and OV_CHUNK % 4 == 0
    for Nw in (1_120_000, 3_300_000, 10_000_000, 2_000_000, 60_000):
        _, n72 = p.lengths(Nw)
        ck = chunking(p, Nw)
        assert ck.rowlen == n72 and ck.length == min(ck.stride + OV_CHUNK, n72)
        last = n72 - (ck.nchunk - 1) * ck.stride
        assert 16 <= last <= ck.length, Nw
        assert ck.nchunk == 1 or n72 - (ck.nchunk - 2) * ck.stride > ck.length   # no chunk to spare
        t = chunking(p, Nw, ov=0) if n72 >= ck.stride else None
        if t is not None:
            assert t.nchunk == n72 // t.stride and t.length == t.stride and t.rowlen == t.nchunk * t.stride


def test_merge_chunks_keeps_each_burst_once():
    """merge_chunks: a burst two overlapping chunks both decoded (positions within the timing phase)
    is kept once, in row order; bursts a slot apart, or in other carriers, are all kept; the blocks
    follow their bursts."""
    from tetraear.signal.wideband import merge_chunks
    M, nchunk, stride = 2, 3, 1000
    C = M * nchunk
    nb, bursts = np.zeros(C, np.int32), np.zeros((C, 8, 2), np.int32)
    nk, blocks = np.zeros(C, np.int32), np.zeros((C, 16, 4), np.int32)
    pos = {0: [10, 520], 1: [2, 512], 2: [0], 3: [10], 4: [], 5: [3, 513]}   # start bits per chunk
    for ch, ps in pos.items():
        nb[ch] = len(ps)
        for j, b in enumerate(ps):
            bursts[ch, j] = (b, j % 3)
            blocks[ch, nk[ch]] = (0, 1, j, 0)
            nk[ch] += 1
    keep, kb = merge_chunks(nb, bursts, nk, blocks, M, nchunk, stride)
    # carrier 0 in row order: 20, 1004 (chunk 1), 1040 (chunk 0: its copy), 2000 (chunk 2), 2024 (chunk 1:
    # its copy); the first copy in row order stays
    assert keep[0, :2].tolist() == [True, False] and keep[1, :2].tolist() == [True, False] and keep[2, 0]
    assert keep[3, 0] and keep[5, :2].tolist() == [True, True]
    rows = {}
    for ch in range(C):
        for j in range(nb[ch]):
            if keep[ch, j]:
                rows.setdefault(ch // nchunk, []).append((ch % nchunk) * stride + 2 * int(bursts[ch, j, 0]))
    for k, r in rows.items():
        r.sort()
        assert all(b - a > 64 for a, b in zip(r, r[1:])), (k, r)
    assert len(rows[0]) == 3 and len(rows[1]) == 3   # 20, ~1020, ~2024 / 20, 2006, ~3026
    assert np.array_equal(kb, keep[np.arange(C)[:, None], np.clip(blocks[..., 2], 0, 7)] &
                          (np.arange(16)[None, :] < nk[:, None]))


def test_wideband_stream_host_logic(monkeypatch):
    """WidebandStream's host side on the CPU (decode stubbed): buffers start whole periods (20000
    input samples -> 72 outputs) into the previous one, keep the last CARRY_Y outputs' input, and
    a frame seen again from the next buffer (same stream position to within the tolerance) is
    emitted once."""
    from tetraear.signal import wideband as WB
    st = None
    p = WB.wb_plan()
    calls = []

    def fake_decode(self, x, cells):
        _, n72 = p.lengths(len(x))
        calls.append((len(x), n72))
        y0 = st.y0
        out = [[], []]
        for k in range(2):   # a burst every 1020 stream outputs, carrier 1 offset by 500
            a0 = (y0 - 500 * k + 1019) // 1020 * 1020 + 500 * k
            for a in range(a0, y0 + n72 - 1020, 1020):
                out[k].append({"sample": a - y0 + (3 if len(calls) % 2 else 0), "blocks": []})
        return out

    monkeypatch.setattr(WB.WidebandReceiver, "decode", fake_decode)
    st = WB.WidebandStream(np.zeros(p.M, np.uint32))
    st.M = 2
    st.last = np.full(2, -(1 << 62), np.int64)
    got = [[], []]
    total = 0
    for n in (700_000, 5_000, 1_300_000, 2_000_003, 999_999):
        before = len(st.tail)
        fr = st.decode(np.zeros(n, np.complex64))
        total += n
        assert (total - len(st.tail)) % st.per == 0                  # buffers start on whole periods
        assert st.y0 == (total - len(st.tail)) // st.per * st.ups    # ... at that stream position
        _, n72 = p.lengths(before + n)
        if n72 > st.CARRY_Y:
            assert p.lengths(len(st.tail))[1] >= st.CARRY_Y - st.ups   # the carried outputs
        for k in range(2):
            got[k].extend(f["stream_sample"] for f in fr[k])
    n72 = p.lengths(total)[1]
    for k in range(2):   # every burst of the stream once, at its position (to within the phase)
        want = list(range(500 * k, n72 - 1020, 1020))
        assert len(got[k]) == len(want) and all(0 <= g - w <= 3 for g, w in zip(got[k], want)), k


@pytest.fixture(scope="module")
def capture():
    from tetraear.signal.wideband import synth_wideband
    Nw = 1_120_000   # 56 ms: one 3932-sample timing chunk per carrier
    return synth_wideband(Nw, seed=11, snr_db=30.0, cfo_max=300.0)


@pytest.mark.gpu
def test_synth_matches_oracle():
    """The device generator is the oracle's synthesis of the same carrier baseband."""
    from tetraear import _hip
    from tetraear.signal.wideband import wb_plan
    c = _hip.ctx()
    p = wb_plan()
    d = W.design()
    Nw = 40_000
    nbb = Nw // p.D + 1
    x = np.empty(Nw, np.complex64)
    cells = np.empty(p.M, np.uint32)
    c.check(c.lib.tetra_synth_wideband(c.handle, p.c, Nw, 5, 1000.0, 300.0, _hip.ptr(x), _hip.ptr(cells), None, None,
                                       None), "synth_wideband")
    s = np.empty((p.M, nbb), np.complex64)
    c.check(c.lib.tetra_synth_etsi(c.handle, p.M, nbb, p.fs / p.D, 5, 1000.0, 300.0, _hip.ptr(s), _hip.ptr(cells),
                                   None, None, None), "synth_etsi")
    want = W.synthesize(s, d, Nw)
    assert np.abs(x - want).max() <= 1e-5 * np.abs(want).max()


@pytest.mark.gpu
def test_channelize_vs_oracle(capture):
    from tetraear.signal.wideband import WidebandReceiver
    x = capture[0]
    d = W.design()
    rx = WidebandReceiver()
    y = rx.channelize(x)
    _, n72 = W.lengths(d, len(x))
    assert y.shape == (d["M"], n72)
    want = W.channelize(x.astype(np.complex128), d)
    err = np.abs(y - want).max()
    assert err <= Y_TOL * np.abs(want).max(), err
    # a partial row (n_keep < n72) is the same prefix
    y2 = rx.channelize(x, 1000)
    assert np.array_equal(y2, y[:, :1000])


@pytest.mark.gpu
@pytest.mark.parametrize("oversample,form", [(2, "1"), (2, "2"), (2, "3"), (2, "4"), (4, "1"), (4, "2")])
def test_channelize_every_analysis_form(oversample, form, monkeypatch):
    """Both filter-bank designs (D = M / 2 and M / 4) through each analysis kernel the host can pick
    (TETRA_WB_ANALYSIS: 1 one block per iteration with the fold on three waves, 2 two blocks, 3 one
    block with every twiddle in LDS, 4 one block with the fold inside the radix-8 butterflies), held
    to the oracle of that design; a capture long enough for several blocks per workgroup and a ragged
    tail."""
    from tetraear.signal.wideband import WidebandReceiver, synth_wideband
    monkeypatch.setenv("TETRA_WB_ANALYSIS", form)
    x = synth_wideband(400_037, seed=5, snr_db=20.0, oversample=oversample)[0]
    d = W.design(oversample=oversample)
    y = WidebandReceiver(oversample=oversample).channelize(x)
    want = W.channelize(x.astype(np.complex128), d)
    assert y.shape == want.shape
    assert np.abs(y - want).max() <= Y_TOL * np.abs(want).max()


@pytest.mark.gpu
def test_one_block_analysis_forms_bit_identical(monkeypatch):
    """D = M / 2: the one-block analysis forms -- the fold on three waves (1, the default), the fold
    inside the radix-8 butterflies with the twiddles in LDS (3) or in registers (4) -- give
    bit-identical y (same operations, same order)."""
    from tetraear.signal.wideband import WidebandReceiver, synth_wideband
    x = synth_wideband(500_003, seed=13, snr_db=20.0, oversample=2)[0]
    rx = WidebandReceiver(oversample=2)
    ys = []
    for form in ("1", "3", "4"):
        monkeypatch.setenv("TETRA_WB_ANALYSIS", form)
        ys.append(rx.channelize(x))
    assert np.array_equal(ys[0], ys[1]) and np.array_equal(ys[0], ys[2])


@pytest.mark.gpu
def test_wideband_timing_bit_exact(capture, monkeypatch):
    """From y on the chain is the ETSI one: the GPU timing on the channeliser's own output equals
    oracle/etsi.py on the same y, carrier by carrier (TETRA_WB_OM=0: the timing's own Oerder-Meyr
    pass over y, the ETSI chain's order; the grouped form: test_wideband_timing_om_bit_exact)."""
    import etsi as E
    from tetraear.signal.wideband import WidebandReceiver, chunking
    monkeypatch.setenv("TETRA_WB_OM", "0")
    x = capture[0]
    rx = WidebandReceiver()
    hard, soft, sym, ns = rx.demod(x)
    ck = chunking(rx.plan, len(x), rx.m2)
    assert ns.shape[1] == ck.nchunk == 1 and ck.length == ck.rowlen   # one chunk: the whole row
    y = rx.channelize(x, ck.rowlen)
    ora = E.Receiver()
    for k in (0, 1, 399, 400, 401, 799):
        so, sbo, ho, _ = ora.timing(y[k])
        n = int(ns[k, 0])
        assert n == len(so), k
        assert np.array_equal(sym[k, 0, :n], so) and np.array_equal(hard[k, 0, :n - 1], ho)
        assert np.array_equal(soft[k, 0, :2 * (n - 1)], sbo)


@pytest.mark.gpu
def test_wideband_round_trip(capture):
    """800 carriers through channeliser + timing + lower MAC: every CRC-passing block is one the
    carrier transmitted, and nearly all blocks pass."""
    from tetraear.core.etsi import EtsiLowerMac
    from tetraear.signal.wideband import WidebandReceiver
    x, cells, kinds, payload, t0 = capture
    rx = WidebandReceiver()
    hard, soft, sym, ns = rx.demod(x)
    M, nchunk = ns.shape
    res = EtsiLowerMac().decode_batch(soft.reshape(M * nchunk, -1), hard.reshape(M * nchunk, -1), ns.reshape(-1),
                                      np.repeat(cells, nchunk))
    nblk = nok = 0
    for i, frames in enumerate(res):
        sent = {tuple(p) for bb in payload[i // nchunk] for p in bb}
        for f in frames:
            for b in f["blocks"]:
                nblk += 1
                if b["crc_ok"]:
                    nok += 1
                    assert tuple(np.pad(b["bits"], (0, 268 - len(b["bits"])))) in sent
    assert nblk >= 2 * M
    assert nok / nblk > 0.97, (nok, nblk)


@pytest.mark.gpu
def test_bench_wideband_pipeline_matches_serial(monkeypatch):
    """bench.py --chain wideband: the two-stream pipeline (channeliser of capture k+1 beside the
    timing + lower MAC of capture k, y double-buffered) and the three-stream one (TETRA_WB_STAGES=3:
    channeliser, timing and lower MAC of three captures, the timing's outputs double-buffered too)
    give every step the serial chain's results."""
    import torch
    from tetraear import _hip
    from tetraear.signal.wideband import BenchStep
    dev = torch.device("cuda", 0)
    outs = []
    for pipe, stages in ((False, "2"), (True, "2"), (True, "3")):
        monkeypatch.setenv("TETRA_WB_STAGES", stages)
        c = _hip.Context()
        c.check(c.lib.tetra_set_stream(c.handle, None), "set_stream")
        st = BenchStep(c, 2_000_000, seed=3, device=dev)
        if pipe:
            st.pipeline()
        assert len(st.contexts()) == (1 if not pipe else int(stages))   # what bench.py profiles
        for _ in range(3):
            st()
        torch.cuda.synchronize(dev)
        ns, nb, nk = st.nsym.cpu(), st.nburst.cpu(), st.nblock.cpu()
        soft, hard, blocks, t1 = st.soft.cpu(), st.hard.cpu(), st.blocks.cpu(), st.type1.cpu()
        n1 = {0: 268, 1: 124, 2: 60}
        outs.append([ns, nb, nk, st.wf.cpu()] + [x for ch in range(st.C) for x in (
            soft[ch, :2 * max(int(ns[ch]) - 1, 0)], hard[ch, :max(int(ns[ch]) - 1, 0)],
            blocks[ch, :int(nk[ch])])] + [t1[ch, j, :n1[int(blocks[ch, j, 0])]] for ch in range(st.C)
                                          for j in range(int(nk[ch]))])
        q = st.quality()   # each burst once (merge_chunks); the rows' whole bursts nearly all decoded
        assert q["crc_ok"] > 0 and q["bursts"] <= q["per_chunk"]["bursts"] and q["decoded_frac"] > 0.8, q
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.fixture(scope="module")
def capture3():
    from tetraear.signal.wideband import synth_wideband
    return synth_wideband(3_300_000, seed=17, snr_db=25.0, cfo_max=300.0)   # three timing chunks per carrier


@pytest.mark.gpu
def test_resampler_om_partials_bit_exact(capture3):
    """tetra_channelize_om: y is tetra_channelize's, and every whole group's Oerder-Meyr class partials
    equal oracle eo_om_group_partials on that y."""
    import etsi as E
    from tetraear.signal.wideband import WidebandReceiver, chunking
    x = capture3[0]
    rx = WidebandReceiver()
    n_keep = chunking(rx.plan, len(x), rx.m2).rowlen
    y, om = rx.channelize_om(x, n_keep)
    assert np.array_equal(y, rx.channelize(x, n_keep))
    U = rx.plan.c.up
    whole = n_keep // U
    for k in (0, 1, 255, 400, 799):
        P = E.Receiver.om_group_partials(y[k], U)
        assert np.array_equal(om[k, :whole], P[:whole]), k


@pytest.mark.gpu
@pytest.mark.parametrize("grouped", [True, False])
def test_wideband_timing_om_bit_exact(capture3, grouped, monkeypatch):
    """The wideband timing over overlapping chunks (tetra_etsi_timing_chunks) equals the oracle's
    timing of each chunk's samples, chunk by chunk -- the last chunk (cut by the row's end) and
    chunks whose start is not on a resampler group (heads and tails) included; grouped: the
    Oerder-Meyr class sums from the resampler's partials in the grouped order, else the timing's own
    pass over y."""
    import etsi as E
    from tetraear.signal.wideband import WidebandReceiver, chunking
    monkeypatch.setenv("TETRA_WB_OM", "1" if grouped else "0")
    x = capture3[0]
    rx = WidebandReceiver()
    assert rx.grouped_om() == grouped
    ck = chunking(rx.plan, len(x), rx.m2)
    assert ck.nchunk == 3 and ck.length > ck.stride and ck.rowlen - 2 * ck.stride < ck.length
    hard, soft, sym, ns = rx.demod(x)
    y, _ = rx.channelize_om(x, ck.rowlen)
    U = rx.plan.c.up
    ora = E.Receiver()
    for k in (0, 3, 399, 400, 798):
        P = E.Receiver.om_group_partials(y[k], U)
        for ci in range(ck.nchunk):
            s = ci * ck.stride
            L = min(ck.length, ck.rowlen - s)
            A = E.Receiver.om_grouped(y[k], s, L, U, P) if grouped else None
            so, sbo, ho, _ = ora.timing(y[k, s:s + L], om=A)
            n = int(ns[k, ci])
            assert n == len(so), (k, ci)
            assert np.array_equal(sym[k, ci, :n], so) and np.array_equal(hard[k, ci, :n - 1], ho), (k, ci)
            assert np.array_equal(soft[k, ci, :2 * (n - 1)], sbo), (k, ci)


@pytest.mark.gpu
def test_timing_om_is_tiled_chunks(capture3):
    """tetra_etsi_timing_om (chunks tiling the rows) is tetra_etsi_timing_chunks with stride = len."""
    from tetraear import _hip
    from tetraear.signal.wideband import WidebandReceiver, chunking
    x = capture3[0]
    rx = WidebandReceiver()
    ck = chunking(rx.plan, len(x), rx.m2, ov=0)
    y, om = rx.channelize_om(x, ck.rowlen)
    M, U, sm = rx.plan.M, rx.plan.c.up, ck.length // 4 + 2
    C = M * ck.nchunk
    c = _hip.ctx()
    outs = []
    for form in ("om", "chunks"):
        o = [np.zeros((C, sm), np.complex64), np.zeros((C, 2 * sm), np.int8), np.zeros((C, sm), np.uint8),
             np.zeros(C, np.int32)]
        if form == "om":
            c.check(c.lib.tetra_etsi_timing_om(c.handle, rx.etsi, _hip.ptr(y), C, ck.length, _hip.ptr(om), ck.nchunk,
                                               om.shape[1], U, *[_hip.ptr(a) for a in o], sm, None), "timing_om")
        else:
            c.check(c.lib.tetra_etsi_timing_chunks(c.handle, rx.etsi, _hip.ptr(y), M, ck.rowlen, ck.nchunk, ck.stride,
                                                   ck.length, _hip.ptr(om), om.shape[1], U,
                                                   *[_hip.ptr(a) for a in o], sm, None), "timing_chunks")
        outs.append(o)
    ns = outs[0][3]
    assert np.array_equal(ns, outs[1][3]) and ns.min() > 0
    for ch in range(C):
        n = int(ns[ch])
        assert np.array_equal(outs[0][0][ch, :n], outs[1][0][ch, :n])
        assert np.array_equal(outs[0][1][ch, :2 * (n - 1)], outs[1][1][ch, :2 * (n - 1)])
        assert np.array_equal(outs[0][2][ch, :n - 1], outs[1][2][ch, :n - 1])


@pytest.mark.gpu
def test_wideband_overlap_decodes_every_burst(capture3):
    """Overlapping chunks lose no burst at a chunk seam: every burst wholly inside a carrier's row is
    decoded once (WidebandReceiver.decode merges the copies two chunks share), its CRC-good blocks are
    ones the carrier sent, and the tiled layout (ov = 0, rounds 1-6) decodes fewer."""
    from tetraear.signal import wideband as WB
    x, cells, kinds, payload, t0 = capture3
    rx = WB.WidebandReceiver()
    ck = WB.chunking(rx.plan, len(x), rx.m2)
    frames = rx.decode(x, cells)
    whole = ck.rowlen // WB.BURST_SAMPLES - 1   # slots wholly inside the row, whatever the phase
    nb = nok = 0
    for k, fr in enumerate(frames):
        samples = [f["sample"] for f in fr]
        assert samples == sorted(samples) and np.all(np.diff(samples) >= WB.BURST_SAMPLES - 16), k
        assert len(fr) >= whole, (k, len(fr))
        sent = {tuple(p) for bb in payload[k] for p in bb}
        for f in fr:
            for b in f["blocks"]:
                nb += 1
                if b["crc_ok"]:
                    nok += 1
                    assert tuple(np.pad(b["bits"], (0, 268 - len(b["bits"])))) in sent
    assert nok / nb > 0.97, (nok, nb)
    tiled = WB.WidebandReceiver()
    orig = WB.OV_CHUNK
    try:
        WB.OV_CHUNK = 0
        ft = tiled.decode(x, cells)
    finally:
        WB.OV_CHUNK = orig
    assert sum(map(len, ft)) < sum(map(len, frames)) - rx.plan.M   # >= 1 burst per carrier lost at the seams


@pytest.mark.gpu
def test_wideband_stream_equals_whole_capture(capture3):
    """WidebandStream over pieces of a capture (seams anywhere, one piece shorter than a chunk)
    decodes the bursts the whole capture does: per carrier the same stream positions (within the
    timing phase) and the same CRC-good bits -- none lost or doubled at the pieces' seams."""
    from tetraear.signal import wideband as WB
    x, cells = capture3[0], capture3[1]
    whole = WB.WidebandReceiver().decode(x, cells)
    st = WB.WidebandStream(cells)
    got = [[] for _ in range(len(cells))]
    for a, b in ((0, 1_234_567), (1_234_567, 1_300_001), (1_300_001, 2_711_113), (2_711_113, len(x))):
        for k, fr in enumerate(st.decode(x[a:b])):
            got[k].extend(fr)
    nmatch = 0
    for k in range(len(cells)):
        ws = [f["sample"] for f in whole[k]]
        gs = [f["stream_sample"] for f in got[k]]
        assert len(gs) == len(ws) and all(abs(p - q) <= 16 for p, q in zip(gs, ws)), (k, ws, gs)
        for fw, fg in zip(whole[k], got[k]):
            bw = [tuple(b["bits"]) for b in fw["blocks"] if b["crc_ok"]]
            bg = [tuple(b["bits"]) for b in fg["blocks"] if b["crc_ok"]]
            assert bw == bg, (k, fw["sample"])
            nmatch += len(bw)
    assert nmatch > 2 * len(cells)


@pytest.mark.gpu
@pytest.mark.parametrize("oversample", [2, 4])
def test_channelize_period_shift_bit_exact(capture3, oversample):
    """What WidebandStream's tail rests on: a capture cut a whole number of its periods in (whole
    resampler periods and whole cycles of the filter bank's mixer term, (-1)^(k j) at D = M / 2,
    (-i)^(k j) at M / 4) channelises to the uncut capture's outputs, bit for bit; at D = M / 2 one
    resampler period (25 blocks, odd) negates the odd carriers."""
    from tetraear.signal.wideband import WidebandReceiver, WidebandStream, synth_wideband
    x, cells = capture3[0], capture3[1]
    if oversample == 4:
        x = synth_wideband(2_000_000, seed=23, snr_db=25.0, oversample=4)[0]
    rx = WidebandReceiver(oversample=oversample)
    st = WidebandStream(cells, oversample=oversample)
    p = rx.plan
    assert st.per == 20000 and st.ups == 72 and st.per % (p.D * p.c.down) == 0
    y = rx.channelize(x)
    for k in (1, 37, 65):
        yk = rx.channelize(x[k * st.per:])
        assert np.array_equal(yk, y[:, k * st.ups:k * st.ups + yk.shape[1]]), k
    if oversample == 2:
        y1 = rx.channelize(x[p.D * p.c.down:])
        ref = y[:, p.c.up:p.c.up + y1.shape[1]]
        assert np.array_equal(y1[0::2], ref[0::2]) and np.array_equal(y1[1::2], -ref[1::2])
