"""The streaming ETSI receiver's CPU restatement (oracle/etsi.py Stream) and the product's host-only
window arithmetic (tetra_etsi_stream_window), on the CPU.

The reference's callers stream one continuous capture in 128 Ki chunks
(/root/reference/tetraear/ui/modern.py:1901-1919, continuous_capture.py:20).  The stream decodes
consecutive chunks as one symbol stream:
  * every window's channel-filter outputs are the whole capture's, bit for bit (the window starts at
    a multiple of q1 * down input samples, so its polyphase phases are the capture's);
  * the first chunk is the non-streaming receiver's output exactly;
  * every burst transmitted whole after the receiver's first chunk is decoded, the ones across chunk
    seams included, with CRC-good blocks (clean and noisy captures, CFO, odd chunk lengths, every
    CLI rate);
  * the product computes the same windows as the oracle.
The GPU is held to this oracle bit for bit in tests/test_gpu_stream.py.
"""
import numpy as np
import pytest

import etsi as E


def _capture(seed, nsamp, fs=2.4e6, snr=20.0, cfo=150.0, nbursts=None):
    rng = np.random.default_rng(seed)
    cell = E.scramble_init(int(rng.integers(200, 800)), int(rng.integers(0, 1000)), int(rng.integers(0, 64)))
    scr = E.scramble_seq(cell, 432)
    nb = nbursts or int(nsamp / fs * 18000 / 255) + 2
    bits, jobs = E.burst_stream(rng, nb, scr)
    t0 = float(rng.uniform(0.0, 0.9))
    x = E.modulate(bits, nsamp, fs=fs, t0=t0, phase0=float(rng.uniform(0, 6.28)), cfo=cfo, snr_db=snr, rng=rng)
    return x, cell, jobs, t0


def _chunks(n_total, sizes):
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


def test_windows_reproduce_the_whole_capture_filter_outputs():
    x, cell, _, _ = _capture(1, 6 * 131072)
    rx = E.Receiver()
    yfull = rx.chanfilt(x)
    st = E.Stream(2.4e6, cell_init=cell)
    done = 0
    for at, n in _chunks(len(x), [131072, 50000, 77778, 131072, 1000, 9000]):
        r = st.push(x[at:at + n])
        s, W = r["window"]
        y = r["y"]
        y0 = 3 * s // 100          # the window's first output in the capture's numbering
        assert np.array_equal(y, yfull[y0:y0 + len(y)]), (at, n, s)
        assert y0 + r["yoff"] == done or (done == 0 and r["yoff"] == 0)
        done = y0 + len(y)
    assert done == len(yfull)


def test_first_chunk_is_the_chunk_on_its_own():
    x, cell, _, _ = _capture(2, 131072)
    st = E.Stream(2.4e6, cell_init=cell)
    r = st.push(x)
    so, sbo, ho, _ = E.Receiver().demod(x)
    assert np.array_equal(r["symbols"], so) and np.array_equal(r["soft"], sbo) and np.array_equal(r["hard"], ho)


@pytest.mark.parametrize("sizes,snr,cfo", [([131072], 20.0, 150.0), ([131072], 12.0, 500.0),
                                           ([50000, 77778, 131072], 18.0, -300.0), ([20000], 25.0, 0.0)])
def test_every_burst_after_the_first_chunk_is_decoded(sizes, snr, cfo):
    """Bursts of the continuous downlink start every 510 bits; every one that starts after the first
    chunk's acquisition (and ends inside the capture) is found at its position, seams included, and
    at these SNRs its blocks pass the CRC."""
    n_total = 8 * 131072
    x, cell, jobs, t0 = _capture(3, n_total, snr=snr, cfo=cfo)
    st = E.Stream(2.4e6, cell_init=cell)
    found, seams = [], 0
    base = 0   # dibits of previous chunks (positions are per chunk)
    for at, n in _chunks(n_total, sizes):
        r = st.push(x[at:at + n])
        for pos, kind, dec in r["bursts"]:
            g = 2 * base + pos   # bit position in the stream's dibits
            found.append((g, kind, all(ok for _, _, ok in dec)))
            seams += pos < 0
        base += len(r["hard"])
    pos = [g for g, _, _ in found]
    assert all(b - a == 510 for a, b in zip(pos, pos[1:])), pos[:6]     # one burst every slot, none lost
    # the bursts on air after the first one: the capture holds n_total / 34000 slots
    assert len(found) >= int(n_total / 34000) - 2, (len(found), n_total / 34000)
    assert np.mean([ok for _, _, ok in found]) >= (1.0 if snr >= 18 else 0.95)
    assert seams >= 1   # some burst did straddle a seam and was decoded


@pytest.mark.parametrize("fs", [1.8e6, 2.0e6, 2.2e6])
def test_stream_at_other_cli_rates(fs):
    n_total = int(6 * 131072 * fs / 2.4e6) // 2 * 2
    x, cell, jobs, t0 = _capture(4, n_total, fs=fs)
    st = E.Stream(fs, cell_init=cell)
    rx = E.Receiver(fs)
    yfull = rx.chanfilt(x)
    found, base = [], 0
    d = rx.d
    for at, n in _chunks(n_total, [int(131072 * fs / 2.4e6) // 2 * 2]):
        r = st.push(x[at:at + n])
        s, W = r["window"]
        y0 = d["up"] * s // (d["q1"] * d["down"])
        assert np.array_equal(r["y"], yfull[y0:y0 + len(r["y"])])
        found += [2 * base + p for p, _, dec in r["bursts"] if all(ok for _, _, ok in dec)]
        base += len(r["hard"])
    assert all(b - a == 510 for a, b in zip(found, found[1:]))
    assert len(found) >= int(n_total / fs * 18000 / 255) - 2


@pytest.mark.parametrize("t0", [0.1, 0.5, 0.9])
def test_retune_mid_stream_recovers_in_the_first_chunk(t0):
    """The GUI retunes the capture without a new processor (modern.py:1903-1909, the loop then keeps
    calling process()): the stream carries the old signal's timing into a new one with another symbol
    phase, CFO and carrier phase.  The Gardner loop pulls in within the first chunk: from the second
    chunk on every burst is found and CRC-good, as for a fresh stream on the new signal."""
    L = 131072
    xa, _, _, _ = _capture(7, 3 * L, cfo=120.0)
    xb, cb, _, _ = _capture(8, 5 * L, cfo=-300.0)
    rng = np.random.default_rng(9)
    xb = E.modulate(E.burst_stream(rng, 40, E.scramble_seq(cb, 432))[0], 5 * L, t0=t0, phase0=2.0, cfo=-300.0,
                    snr_db=18.0, rng=rng)
    st = E.Stream(2.4e6, cell_init=cb)
    for k in range(3):
        st.push(xa[k * L:(k + 1) * L])
    got = []
    for k in range(5):
        r = st.push(xb[k * L:(k + 1) * L])
        got.append((len(r["bursts"]), sum(all(ok for _, _, ok in dec) for _, _, dec in r["bursts"])))
    assert all(n >= 3 and ok == n for n, ok in got[1:]), got
    assert got[0][1] >= 1, got


def _sync_pdu(rng, mcc, mnc, cc):
    """60 BSCH type-1 bits carrying a cell: colour code at 4..9, MCC 31..40, MNC 41..54 (the fields
    bsch_cell_init reads), the rest random."""
    t = rng.integers(0, 2, 60).astype(np.uint8)
    for v, lo, n in ((cc, 4, 6), (mcc, 31, 10), (mnc, 41, 14)):
        t[lo:lo + n] = [(v >> (n - 1 - i)) & 1 for i in range(n)]
    return t


def test_acquisition_carries_across_chunks():
    """No cell given: the first CRC-good BSCH sets the cell, the next chunks keep it."""
    rng = np.random.default_rng(5)
    mcc, mnc, cc = 262, 1010, 17
    cell = E.scramble_init(mcc, mnc, cc)
    scr = E.scramble_seq(cell, 432)
    parts = []
    for i in range(28):
        bt = (0, 1, 2, 0)[i % 4]
        pay = [_sync_pdu(rng, mcc, mnc, cc), rng.integers(0, 2, 124).astype(np.uint8)] if bt == 2 else None
        parts.append(E.make_burst(bt, rng, scr, pay)[0])
    x = E.modulate(np.concatenate(parts), 6 * 131072, t0=0.3, phase0=1.0, cfo=80.0, snr_db=20.0, rng=rng)
    st = E.Stream(2.4e6)
    cells = []
    for at, n in _chunks(len(x), [131072]):
        r = st.push(x[at:at + n])
        cells.append(r["cell"])
    assert cells[-1] == cell and cells.count(cell) >= len(cells) - 2


def test_product_window_arithmetic_equals_the_oracle():
    """tetra_etsi_stream_window (host code of the product, no GPU) gives the oracle's windows for
    every supported rate and chunk pattern, the first chunk, tiny chunks and chunks of one sample pair."""
    from tetraear.signal.etsi import etsi_plan, stream_window
    for fs in (2.4e6, 1.8e6, 1.9e6, 2.0e6, 2.1e6, 2.2e6, 2.3e6):
        plan = etsi_plan(fs)
        st = E.Stream(fs)
        for n in (131072, 2, 40, 1200, 131072, 50002, 8, 131072):
            want = st.window(n)
            s, W, yoff, y_next = stream_window(plan, st.x_total, st.y_done, n)
            assert (s, W, yoff) == want[:3], (fs, n)
            assert W % 2 == 0 and s % 2 == 0, (fs, n, s, W)   # whole sample pairs (the kernels' loads)
            st.x_total += n
            st.y_done = max(st.y_done, E.stream_lengths(st.rx.d, st.x_total)[1])
            assert y_next == st.y_done
