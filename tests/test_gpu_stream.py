"""GPU parity of the streaming ETSI receiver (tetra_etsi_stream_window + tetra_demod_etsi_stream +
tetra_lmac_etsi_stream) against its CPU restatement oracle/etsi.py Stream, chunk after chunk of one
continuous capture (the reference's capture loops stream 128 Ki chunks,
/root/reference/tetraear/ui/modern.py:1901-1919, continuous_capture.py:20).

Bar: bit-identical -- per chunk the symbols (the carried one first), soft bits, hard dibits, the burst
positions (relative to the chunk, negative across the seam), kinds, decoded type-1 bits, CRC flags and
the acquired cells; and on the synthesised capture >= 99 % of the bursts on air after the first chunk
decoded.  Parity unpinned against the reference (it has no ETSI chain).
"""
import ctypes

import numpy as np
import pytest

import etsi as E

pytestmark = pytest.mark.gpu

L = 131072


def _oracle_chunks(iq, fs, sizes, cells=None, fmt="cf32"):
    """The oracle stream of each channel over the chunk sequence: per chunk per channel its dict."""
    C = iq.shape[0]
    streams = [E.Stream(fs, cell_init=None if cells is None else int(cells[ch])) for ch in range(C)]
    out = []
    for at, n in sizes:
        out.append([streams[ch].push(iq[ch, at:at + n]) for ch in range(C)])
    return out


def _chunk_plan(n_total, sizes):
    out, at, i = [], 0, 0
    while at < n_total:
        n = min(sizes[i % len(sizes)], n_total - at)
        n -= n % 2
        if n == 0:
            break
        out.append((at, n))
        at += n
        i += 1
    return out


def _compare(k, got_demod, got_frames, want, C):
    hard, soft, sym, ns = got_demod
    for ch in range(C):
        w = want[ch]
        n = int(ns[ch])
        case = (k, ch)
        assert n == len(w["symbols"]), case + (n, len(w["symbols"]))
        assert np.array_equal(sym[ch, :n], w["symbols"]), case
        assert np.array_equal(hard[ch, :max(n - 1, 0)], w["hard"]), case
        assert np.array_equal(soft[ch, :2 * max(n - 1, 0)], w["soft"]), case
        got = got_frames[ch]
        assert [(f["position"], f["burst_kind"]) for f in got] == [(p, kd) for p, kd, _ in w["bursts"]], case
        for f, (_, _, dec) in zip(got, w["bursts"]):
            assert len(f["blocks"]) == len(dec), case
            for b, (kind, bits, ok) in zip(f["blocks"], dec):
                assert b["crc_ok"] == ok and np.array_equal(b["bits"], bits), case


@pytest.mark.parametrize("sizes,acquire", [([L], False), ([L], True), ([50000, 77778, L, 3000], False)])
def test_stream_bit_identical_to_oracle(sizes, acquire):
    from tetraear.signal.etsi import EtsiStream, synth
    from tetraear.core.etsi import EtsiLowerMac
    C, K = 6, 6
    iq, cells, kinds, payload, t0 = synth(C, K * L, seed=31, snr_db=16.0, cfo_max=600.0)
    plan = _chunk_plan(K * L, sizes)
    want = _oracle_chunks(iq, 2.4e6, plan, None if acquire else cells)
    st, lm = EtsiStream(2.4e6, C), EtsiLowerMac()
    for k, (at, n) in enumerate(plan):
        d = st.demod(iq[:, at:at + n])
        frames = lm.decode_stream(d[1], d[0], d[3], None if acquire else cells)
        _compare(k, d, frames, want[k], C)
        if acquire:
            assert [int(v) for v in lm.cell_state] == [want[k][ch]["cell"] for ch in range(C)], k
    assert (np.asarray(st.track["acquired"]) == 1).all()


def test_stream_decodes_every_burst_on_air():
    """8 consecutive 128 Ki chunks of 32 channels, cells acquired: the bursts decoded per channel-chunk
    after the first chunk are >= 99 % of those on air (3.86 per chunk), the blocks >= 97 % CRC-good."""
    from tetraear.signal.etsi import EtsiStream, synth
    from tetraear.core.etsi import EtsiLowerMac
    C, K = 32, 8
    iq, cells, kinds, payload, t0 = synth(C, K * L, seed=41, snr_db=18.0, cfo_max=600.0)
    st, lm = EtsiStream(2.4e6, C), EtsiLowerMac()
    nb = nblk = nok = 0
    for k in range(K):
        hard, soft, sym, ns = st.demod(iq[:, k * L:(k + 1) * L])
        frames = lm.decode_stream(soft, hard, ns)
        if k == 0:
            continue
        for ch in range(C):
            nb += len(frames[ch])
            for f in frames[ch]:
                nblk += len(f["blocks"])
                nok += sum(b["crc_ok"] for b in f["blocks"])
    on_air = C * (K - 1) * L / 34000   # one 255-symbol slot = 34000 samples at 2.4 MSps
    assert nb >= 0.99 * on_air, (nb, on_air)
    assert nok >= 0.97 * nblk, (nok, nblk)
    assert sum(int(v) == int(c) for v, c in zip(lm.cell_state, cells)) >= 0.9 * C


def test_sc16_stream_equals_cf32_stream():
    from tetraear.signal.etsi import EtsiStream, synth
    C, K = 4, 4
    iq, cells = synth(C, K * L, seed=43, snr_db=18.0)[:2]
    q = np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
    a, b = EtsiStream(2.4e6, C), EtsiStream(2.4e6, C)
    for k in range(K):
        ra = a.demod(iq[:, k * L:(k + 1) * L])
        rb = b.demod(q[:, k * L:(k + 1) * L])
        for x, y in zip(ra, rb):
            assert np.array_equal(x, y), k


def test_stream_mixed_formats_continue_in_cf32():
    """Chunks of one stream in different formats -- SC16, then cf32, then SC16 with the AFC mixer on
    (which takes cf32) -- decode as the all-cf32 stream of the same samples does (SC16 -> cf32 is
    exact), instead of failing."""
    from tetraear.signal.etsi import EtsiStream, synth
    C, K = 2, 4
    iq = synth(C, K * L, seed=45, snr_db=18.0)[0]
    q = np.stack([np.rint(iq.real * 32768), np.rint(iq.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
    f = (q[..., 0].astype(np.float32) / 32768 + 1j * (q[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    offs = [None, None, [100.0, -50.0], None]
    a, b = EtsiStream(2.4e6, C), EtsiStream(2.4e6, C)
    for k in range(K):
        sl = slice(k * L, (k + 1) * L)
        ra = a.demod(f[:, sl], offs[k])
        rb = b.demod(f[:, sl] if k == 1 else q[:, sl], offs[k])
        for x, y in zip(ra, rb):
            assert np.array_equal(x, y), k


@pytest.mark.parametrize("fs", [1.8e6, 2.1e6])
def test_stream_other_rates_vs_oracle(fs):
    """The generic-rate chain (k_chanfilt_g + k_timing) streams the same way."""
    from tetraear.signal.etsi import EtsiStream, synth
    from tetraear.core.etsi import EtsiLowerMac
    C = 3
    n = int(L * fs / 2.4e6) // 2 * 2
    iq, cells = synth(C, 5 * n, fs=fs, seed=47, snr_db=18.0)[:2]
    plan = _chunk_plan(5 * n, [n])
    want = _oracle_chunks(iq, fs, plan, cells)
    st, lm = EtsiStream(fs, C), EtsiLowerMac()
    for k, (at, m) in enumerate(plan):
        d = st.demod(iq[:, at:at + m])
        _compare(k, d, lm.decode_stream(d[1], d[0], d[3], cells), want[k], C)


def test_resident_capture_windows_in_place():
    """A capture resident on the device as [C][K N] rows streamed in place (ld = K N, the window a
    pointer into the row: the bench's layout) equals the host-window path, and the lower MAC writing
    its tail into the next buffer of a double-buffered pair equals it writing into its own rows."""
    import torch
    from tetraear import _hip
    from tetraear.signal.etsi import EtsiStream, etsi_plan, lengths, stream_window, synth, TRACK, RESERVE
    C, K = 5, 4
    iq, cells = synth(C, K * L, seed=53, snr_db=18.0)[:2]
    host = EtsiStream(2.4e6, C)
    dev = torch.from_numpy(iq.view(np.float32).reshape(C, K * L, 2).copy()).cuda()
    plan = etsi_plan(2.4e6)
    c = _hip.ctx()
    track = torch.zeros(C * TRACK.itemsize // 4, dtype=torch.int32, device="cuda")
    x_total = y_done = 0
    _, M2max, smx = lengths(plan, L + 4096)
    stride = RESERVE + smx + 1
    bufs = [(torch.zeros((C, stride, 2), dtype=torch.float32, device="cuda"),
             torch.zeros((C, 2 * stride), dtype=torch.int8, device="cuda"),
             torch.zeros((C, stride), dtype=torch.uint8, device="cuda"),
             torch.zeros(C, dtype=torch.int32, device="cuda")) for _ in range(2)]
    lead = torch.full((C,), 2 * RESERVE, dtype=torch.int32, device="cuda")
    c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(cells), C), "set_cells")
    from tetraear.core.etsi import EtsiLowerMac
    lm = EtsiLowerMac()
    for k in range(K):
        want = host.demod(iq[:, k * L:(k + 1) * L])
        wf = lm.decode_stream(want[1], want[0], want[3], cells)
        s, W, yoff, y_next = stream_window(plan, x_total, y_done, L)
        sym, soft, hard, ns = bufs[k & 1]
        _, M2, sm = lengths(plan, W)
        smax = sm + 1
        ptr = dev.data_ptr() + 8 * s
        c.check(c.lib.tetra_demod_etsi_stream(c.handle, plan, ctypes.c_void_p(ptr), _hip.TETRA_CF32, C, K * L, W,
                                              int(yoff), _hip.ptr(track), ctypes.c_void_p(sym.data_ptr() + 8 * RESERVE),
                                              ctypes.c_void_p(soft.data_ptr() + 2 * RESERVE),
                                              ctypes.c_void_p(hard.data_ptr() + RESERVE), _hip.ptr(ns), smax, stride,
                                              None), "demod_stream")
        nsym = ns
        nb = torch.zeros(C, dtype=torch.int32, device="cuda")
        bursts = torch.zeros((C, 8, 2), dtype=torch.int32, device="cuda")
        nk = torch.zeros(C, dtype=torch.int32, device="cuda")
        blocks = torch.zeros((C, 16, 4), dtype=torch.int32, device="cuda")
        t1 = torch.zeros((C, 16, 268), dtype=torch.uint8, device="cuda")
        _, nsoft, nhard, _ = bufs[(k + 1) & 1]
        c.check(c.lib.tetra_lmac_etsi_stream(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), C, stride,
                                             _hip.ptr(lead), _hip.ptr(nsoft), _hip.ptr(nhard), None, _hip.ptr(nb),
                                             _hip.ptr(bursts), _hip.ptr(nk), _hip.ptr(blocks), _hip.ptr(t1)),
                "lmac_stream")
        c.synchronize()
        x_total += L
        y_done = y_next
        n = ns.cpu().numpy()
        h = hard.cpu().numpy()
        sy = sym.cpu().numpy().view(np.complex64)[..., 0]
        for ch in range(C):
            assert n[ch] == want[3][ch], (k, ch)
            assert np.array_equal(h[ch, RESERVE:RESERVE + n[ch] - 1], want[0][ch, :n[ch] - 1]), (k, ch)
            assert np.array_equal(sy[ch, RESERVE:RESERVE + n[ch]], want[2][ch, :n[ch]]), (k, ch)
        bt = bursts.cpu().numpy()
        nbh = nb.cpu().numpy()
        for ch in range(C):
            assert [tuple(bt[ch, b]) for b in range(nbh[ch])] == [(f["position"], f["burst_kind"]) for f in wf[ch]]


def test_process_and_decode_stream_across_seams():
    """The GUI's call pattern -- SignalProcessor(mode='etsi').process(chunk) then
    TetraDecoder(mode='etsi').decode(hard), chunk after chunk -- is the stream: the frames equal the
    oracle stream's bursts chunk by chunk, every slot after the first chunk decoded."""
    from tetraear.signal import SignalProcessor
    from tetraear.core import TetraDecoder
    from tetraear.signal.etsi import synth
    K = 6
    iq, cells = synth(1, K * L, seed=59, snr_db=18.0, cfo_max=300.0)[:2]
    p, d = SignalProcessor(2.4e6, mode="etsi"), TetraDecoder(mode="etsi")
    orc = E.Stream(2.4e6)
    nslots = 0
    for k in range(K):
        hard = p.process(iq[0, k * L:(k + 1) * L])
        assert len(p.symbols) == len(hard) + 1
        raw = d._etsi_rx().decode(hard)
        w = orc.push(iq[0, k * L:(k + 1) * L])
        assert np.array_equal(np.asarray(hard), w["hard"]) and np.array_equal(p.symbols, w["symbols"]), k
        assert [(f["position"], f["burst_kind"]) for f in raw] == [(q, kd) for q, kd, _ in w["bursts"]], k
        nslots += len(raw) if k else 0
    assert nslots >= int((K - 1) * L / 34000)


def test_process_odd_chunks_carry_the_last_sample():
    """process() chunks of odd length: the stream takes whole sample pairs, so each odd chunk's last
    sample goes in front of the next call's -- no sample is dropped and the stream stays the
    capture's: each call equals the oracle stream pushed with the pieces the carry produces."""
    from tetraear.signal.etsi import EtsiReceiver, synth
    iq = synth(1, 4 * L, seed=63, snr_db=18.0)[0][0]
    sizes = [65537, 65535, 131071, 131073, 3, 1, 50000]
    rx, orc = EtsiReceiver(), E.Stream(2.4e6)
    at, carry = 0, np.zeros(0, np.complex64)
    for k, n in enumerate(sizes):
        hard, sym = rx.process(iq[at:at + n])
        piece = np.concatenate([carry, iq[at:at + n]])
        carry = piece[len(piece) - len(piece) % 2:]
        piece = piece[:len(piece) - len(piece) % 2]
        at += n
        if len(piece) == 0:
            assert len(hard) == 0, k
            continue
        w = orc.push(piece)
        assert np.array_equal(np.asarray(hard), w["hard"]) and np.array_equal(sym, w["symbols"]), k
    assert orc.x_total == at - len(carry)


def test_stream_mixer_phase_is_continuous():
    """With an AFC offset the mixer runs on each window at the capture's global sample index, so the
    stream with the offset decodes as the stream of the pre-shifted capture does (every slot after
    the first chunk, CRC-good), and its first chunk equals the chunk mixed from its start."""
    from tetraear.signal.etsi import EtsiStream, EtsiReceiver, synth
    from tetraear.core.etsi import EtsiLowerMac
    C, K, f = 2, 5, 4 * 1171.875
    iq, cells = synth(C, K * L, seed=61, snr_db=20.0, cfo_max=100.0)[:2]
    n = np.arange(K * L)
    shifted = (iq * np.exp(2j * np.pi * f * n / 2.4e6)[None, :]).astype(np.complex64)   # +f, the mixer removes it
    st, lm = EtsiStream(2.4e6, C), EtsiLowerMac()
    good = total = 0
    for k in range(K):
        d = st.demod(shifted[:, k * L:(k + 1) * L], [f] * C)
        if k == 0:
            one = EtsiReceiver()
            h0, s0 = one.process(shifted[0, :L], f, stream=False)
            assert np.array_equal(d[0][0, :len(h0)], np.asarray(h0))
        fr = lm.decode_stream(d[1], d[0], d[3], cells)
        if k:
            for ch in range(C):
                total += len(fr[ch])
                good += sum(all(b["crc_ok"] for b in x["blocks"]) for x in fr[ch])
    assert total >= int(C * (K - 1) * L / 34000) and good >= 0.97 * total
