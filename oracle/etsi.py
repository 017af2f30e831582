"""CPU oracle for the ETSI receive chain + a transmitter for round-trip tests (TEST INFRASTRUCTURE).

PARITY UNPINNED against the reference: /root/reference has no descrambler, deinterleaver, Viterbi,
Gardner or polyphase channel filter.  This oracle is pinned instead by
  * known answers: CRC-16 check value 0xD64E for "123456789", residue 0x1D0F;
  * transmitter -> receiver round trips (tests/test_etsi_oracle.py);
and the HIP kernels are checked against it (bit-exact coding, soft symbols within 1e-5).
Restated spec: EN 300 392-2 §5.3, §8.2.3-§8.2.5, §9.4.4 (see etsi_oracle.c header).
"""
import ctypes
import os

import numpy as np
from scipy import signal as _design

from compat import lib as _lib_loader  # same liboracle.so

FS_NOMINAL = 2.4e6
SYMBOL_RATE = 18000.0
KIND = {"SCH/F": 0, "SCH/HD": 1, "BSCH": 2}
KIND_PARAMS = {0: (432, 103, 288, 268), 1: (216, 101, 144, 124), 2: (120, 11, 80, 60)}  # K, a, n2, n1
# eo_track / tetra_etsi_track: the streaming receiver's per-channel timing state
TRACK = np.dtype([("base", np.float32), ("delta", np.float32), ("pr", np.float32), ("pi", np.float32),
                  ("acquired", np.int32), ("reserved", np.int32, 3)])
MAXB = 8          # bursts per chunk row (ETSI_MAXB)
RESERVE = 256     # dibits ahead of a streaming row: the previous chunk's unconsumed tail (<= 509 bits)
MARGIN = 8        # y samples a streaming window re-computes before the first new output
BURST_NDB_N, BURST_NDB_P, BURST_SB = 0, 1, 2

Q_BITS = np.array([1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 1, 0, 1, 1, 0, 1], np.uint8)
N_BITS = np.array([1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0], np.uint8)
P_BITS = np.array([0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0], np.uint8)
Y_BITS = np.array([1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 0, 0, 0,
                   0, 1, 1, 0, 0, 1, 1, 1], np.uint8)
F_BITS = np.array([1] * 8 + [0] * 64 + [1] * 8, np.uint8)

_bound = False


def lib():
    global _bound
    L = _lib_loader()
    if not _bound:
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.eo_scramble_seq.argtypes = [ctypes.c_uint32, ctypes.c_int, u8p]
        L.eo_scramble_init.argtypes = [ctypes.c_uint32] * 3
        L.eo_scramble_init.restype = ctypes.c_uint32
        L.eo_crc16_reg.argtypes = [u8p, ctypes.c_int]
        L.eo_crc16_reg.restype = ctypes.c_uint32
        L.eo_encode_block.argtypes = [u8p, ctypes.c_int, u8p, u8p]
        L.eo_decode_block.argtypes = [i8p, ctypes.c_int, u8p, u8p]
        L.eo_decode_block.restype = ctypes.c_int
        L.eo_viterbi.argtypes = [i8p, ctypes.c_int, u8p]
        L.eo_chanfilt.argtypes = [f32p, ctypes.c_int, f32p, ctypes.c_int, ctypes.c_int, f32p, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, f32p, f32p]
        L.eo_chanfilt.restype = ctypes.c_int
        L.eo_timing.argtypes = [f32p, ctypes.c_int, ctypes.c_float, ctypes.c_float, f32p, f32p, i8p, u8p,
                                ctypes.c_int, f32p]
        L.eo_timing.restype = ctypes.c_int
        L.eo_timing_om.argtypes = [f32p, ctypes.c_int, f32p, ctypes.c_float, ctypes.c_float, f32p, f32p, i8p, u8p,
                                   ctypes.c_int, f32p]
        L.eo_timing_om.restype = ctypes.c_int
        L.eo_om_quarters.argtypes = [f32p, ctypes.c_int, f32p]
        L.eo_om_group_partials.argtypes = [f32p, ctypes.c_long, ctypes.c_int, f32p]
        L.eo_om_grouped.argtypes = [f32p, ctypes.c_long, ctypes.c_int, ctypes.c_int, f32p, f32p]
        L.eo_sync.argtypes = [u8p, ctypes.c_int, i32p, i32p, ctypes.c_int]
        L.eo_sync.restype = ctypes.c_int
        L.eo_sync_from.argtypes = [u8p, ctypes.c_int, ctypes.c_int, i32p, i32p, ctypes.c_int, i32p]
        L.eo_sync_from.restype = ctypes.c_int
        L.eo_timing_stream.argtypes = [f32p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_float,
                                       ctypes.c_float, f32p, f32p, i8p, u8p, ctypes.c_int, f32p]
        L.eo_timing_stream.restype = ctypes.c_int
        L.eo_decide.argtypes = [f32p, ctypes.c_int, u8p]
        _bound = True
    return L


# ------------------------------------------------------------------------------ design

def rrc(t, alpha=0.35):
    t = np.asarray(t, np.float64)
    out = np.empty_like(t)
    z = np.abs(t) < 1e-9
    out[z] = 1.0 - alpha + 4 * alpha / np.pi
    s = np.abs(np.abs(4 * alpha * t) - 1.0) < 1e-9
    out[s] = (alpha / np.sqrt(2)) * ((1 + 2 / np.pi) * np.sin(np.pi / (4 * alpha))
                                     + (1 - 2 / np.pi) * np.cos(np.pi / (4 * alpha)))
    o = ~(z | s)
    tt = t[o]
    out[o] = (np.sin(np.pi * tt * (1 - alpha)) + 4 * alpha * tt * np.cos(np.pi * tt * (1 + alpha))) / \
        (np.pi * tt * (1 - (4 * alpha * tt) ** 2))
    return out


def design(fs=FS_NOMINAL):
    """Receiver constants for input rate fs: stage-1 decimator taps, RRC polyphase prototype, loop
    constants.  The plan (spec of tetraear.signal.etsi.rate_design): stage 1 decimates by q1 to
    fs1 = fs / q1 >= 180 kHz (q1 <= 13), stage 2 resamples by the reduced fraction up/down =
    72 kHz / fs1 through an 8-symbol RRC prototype of 32 down + 1 taps (4 down taps per symbol)
    scaled by 240 kHz / fs1; of the candidates with <= 4096 taps and < 254 taps per output, the
    smallest down wins, then the largest q1."""
    import math
    fs_i = int(round(fs))
    if abs(fs - fs_i) > 1e-6 or fs_i < 72000:
        raise ValueError("ETSI receiver needs an integer rate >= 72 kHz")
    cands = []
    q1 = 1
    while q1 <= 13 and (q1 == 1 or fs_i / q1 >= 180000.0):
        g = math.gcd(72000 * q1, fs_i)
        up, down = 72000 * q1 // g, fs_i // g
        Lp = 32 * down + 1
        if Lp <= 4096 and (Lp - 1) // up + 2 < 254:
            cands.append((down, -q1, up))
        q1 += 1
    if not cands:
        raise ValueError("no ETSI channel-filter plan for this rate")
    down, q1, up = min(cands)
    q1 = -q1
    L1 = 1 if q1 == 1 else min(64, 2 * int(round(2.4 * q1)))
    h1 = (_design.firwin(L1, 60e3, fs=fs, window=("kaiser", 6.0)) if q1 > 1 else np.ones(1)).astype(np.float32)
    Lp = 32 * down + 1
    hp = (rrc((np.arange(Lp) - (Lp - 1) / 2) / (4.0 * down), 0.35) * (240000.0 * q1 / fs)).astype(np.float32)
    return dict(q1=q1, L1=L1, h1=h1, Lp=Lp, hp=hp, up=up, down=down, gain=np.float32(1.5),
                soft_scale=np.float32(64.0))


def scramble_seq(init, n=432):
    out = np.empty(n, np.uint8)
    lib().eo_scramble_seq(init, n, out)
    return out


def scramble_init(mcc, mnc, cc):
    return int(lib().eo_scramble_init(mcc, mnc, cc))


def crc16_reg(bits):
    b = np.ascontiguousarray(np.asarray(bits) & 1, np.uint8)
    return int(lib().eo_crc16_reg(b, len(b)))


# ------------------------------------------------------------------------------ transmitter

def encode_block(type1, kind, scr):
    K = KIND_PARAMS[kind][0]
    out = np.empty(K, np.uint8)
    lib().eo_encode_block(np.ascontiguousarray(type1, np.uint8), kind, np.ascontiguousarray(scr[:K], np.uint8), out)
    return out


def make_burst(btype, rng, cell_scr, payloads=None):
    """One 510-bit continuous-downlink burst; returns (bits, [(kind, type1), ...])."""
    bb = rng.integers(0, 2, 30).astype(np.uint8)
    head, tail, h2 = Q_BITS[10:22], Q_BITS[0:10], np.zeros(2, np.uint8)
    jobs = []

    def payload(kind):
        n1 = KIND_PARAMS[kind][3]
        return rng.integers(0, 2, n1).astype(np.uint8) if payloads is None else payloads.pop(0)

    if btype == BURST_SB:
        t_b = payload(2)
        t_h = payload(1)
        sb1 = encode_block(t_b, 2, scramble_seq(3, 120))
        bk2 = encode_block(t_h, 1, cell_scr)
        bits = np.concatenate([head, h2, F_BITS, sb1, Y_BITS, bb, bk2, h2, tail])
        jobs = [(2, t_b), (1, t_h)]
    elif btype == BURST_NDB_N:
        t_f = payload(0)
        blk = encode_block(t_f, 0, cell_scr)
        bits = np.concatenate([head, h2, blk[:216], bb[:14], N_BITS, bb[14:], blk[216:], h2, tail])
        jobs = [(0, t_f)]
    else:
        t1, t2 = payload(1), payload(1)
        b1 = encode_block(t1, 1, cell_scr)
        b2 = encode_block(t2, 1, cell_scr)
        bits = np.concatenate([head, h2, b1, bb[:14], P_BITS, bb[14:], b2, h2, tail])
        jobs = [(1, t1), (1, t2)]
    assert len(bits) == 510
    return bits, jobs


def burst_stream(rng, nbursts, cell_scr, kinds=None):
    bits, jobs = [], []
    for i in range(nbursts):
        bt = kinds[i % len(kinds)] if kinds is not None else int(rng.choice([0, 0, 1, 2]))
        b, j = make_burst(bt, rng, cell_scr)
        bits.append(b)
        jobs.append((bt, j))
    return np.concatenate(bits), jobs


def modulate(bits, n, fs=FS_NOMINAL, t0=0.0, phase0=0.0, cfo=0.0, snr_db=None, rng=None, amp=0.5, span=6):
    """pi/4-DQPSK (Table 5.1) with RRC(0.35) pulses sampled at fs; sample n is at symbol time
    t0 + n*18000/fs (symbols counted from the first dibit)."""
    d = np.asarray(bits, np.int64).reshape(-1, 2)
    step = np.where(d[:, 0] == 0, np.where(d[:, 1] == 0, 1, 3), np.where(d[:, 1] == 0, -1, -3))  # x pi/4
    ph = phase0 + np.pi / 4 * np.cumsum(step)
    sym = np.exp(1j * ph)
    t = t0 + np.arange(n) * (SYMBOL_RATE / fs)
    k0 = np.floor(t).astype(np.int64)
    x = np.zeros(n, np.complex128)
    for dd in range(-span, span + 1):
        k = k0 + dd
        ok = (k >= 0) & (k < len(sym))
        x[ok] += sym[k[ok]] * rrc(t[ok] - k[ok])
    x *= amp
    if cfo:
        x *= np.exp(2j * np.pi * cfo * np.arange(n) / fs)
    if snr_db is not None:   # Es/N0: N0 = (P * Ts) / 10^(snr/10), per-sample variance N0 * fs
        p = np.mean(np.abs(x) ** 2)
        sigma = np.sqrt(p * (fs / SYMBOL_RATE) / 10 ** (snr_db / 10) / 2)
        x += sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x.astype(np.complex64)


def bsch_cell_init(type1):
    """Scrambling init of the cell a decoded BSCH announces: extended colour code = MCC (type-1 bits
    31..40) | MNC (41..54) | colour code (4..9) (EN 300 392-2 §21.4.4.2 MAC-SYNC, §18.4.2.1
    D-MLE-SYNC), init = (ecc << 2) | 3 (§8.2.5.2)."""
    t = [int(v) & 1 for v in type1]
    cc = mm = 0
    for v in t[4:10]:
        cc = (cc << 1) | v
    for v in t[31:55]:
        mm = (mm << 1) | v
    return (((mm << 6) | cc) << 2) | 3


# ------------------------------------------------------------------------------ receiver

class Receiver:
    def __init__(self, fs=FS_NOMINAL):
        self.fs = fs
        self.d = design(fs)

    def chanfilt(self, x):
        d = self.d
        x = np.ascontiguousarray(np.asarray(x, np.complex64)).view(np.float32)
        N = len(x) // 2
        M1 = max(0, (N - d["L1"]) // d["q1"] + 1)
        x240 = np.zeros(2 * max(M1, 1), np.float32)
        y = np.zeros(2 * max(M1 * d["up"] // d["down"] + 2, 1), np.float32)
        M2 = lib().eo_chanfilt(x, N, d["h1"], d["L1"], d["q1"], d["hp"], d["Lp"], d["up"], d["down"], x240, y)
        return y[:2 * M2].view(np.complex64).copy()

    def timing(self, y, om=None):
        """Timing + decision on one chunk y; om: its Oerder-Meyr class sums A[4] (om_grouped), or
        None for the fused demod's quarter order (om_quarters)."""
        d = self.d
        yv = np.ascontiguousarray(np.asarray(y, np.complex64)).view(np.float32)
        M2 = len(yv) // 2
        smax = M2 // 4 + 2
        sym = np.zeros(2 * smax, np.float32)
        dscr = np.zeros(2 * smax, np.float32)
        soft = np.zeros(2 * smax, np.int8)
        hard = np.zeros(smax, np.uint8)
        diag = np.zeros(4, np.float32)
        if om is None:
            S = lib().eo_timing(yv, M2, d["gain"], d["soft_scale"], sym, dscr, soft, hard, smax, diag)
        else:
            S = lib().eo_timing_om(yv, M2, np.ascontiguousarray(om, np.float32), d["gain"], d["soft_scale"], sym,
                                   dscr, soft, hard, smax, diag)
        return (sym[:2 * S].view(np.complex64).copy(), soft[:2 * max(S - 1, 0)].copy(),
                hard[:max(S - 1, 0)].copy(), diag)

    def demod(self, x):
        return self.timing(self.chanfilt(x))

    def timing_stream(self, y, yoff, trk):
        """eo_timing_stream: the timing stage on one streaming window (trk: a TRACK record, updated)."""
        d = self.d
        yv = np.ascontiguousarray(np.asarray(y, np.complex64)).view(np.float32)
        M2 = len(yv) // 2
        smax = M2 // 4 + 3
        sym = np.zeros(2 * smax, np.float32)
        dscr = np.zeros(2 * smax, np.float32)
        soft = np.zeros(2 * smax, np.int8)
        hard = np.zeros(smax, np.uint8)
        diag = np.zeros(4, np.float32)
        S = lib().eo_timing_stream(yv, M2, int(yoff), trk.ctypes.data, d["gain"], d["soft_scale"], sym, dscr, soft,
                                   hard, smax, diag)
        return (sym[:2 * S].view(np.complex64).copy(), soft[:2 * max(S - 1, 0)].copy(),
                hard[:max(S - 1, 0)].copy(), diag)

    @staticmethod
    def om_quarters(y):
        """Oerder-Meyr class sums of one chunk in the fused demod's order (eo_om_quarters)."""
        yv = np.ascontiguousarray(np.asarray(y, np.complex64)).view(np.float32)
        A = np.zeros(4, np.float32)
        lib().eo_om_quarters(yv, len(yv) // 2, A)
        return A

    @staticmethod
    def om_group_partials(row, U):
        """The wideband resampler's per-group class partials of a carrier row: [ceil(n / U), 4]."""
        rv = np.ascontiguousarray(np.asarray(row, np.complex64)).view(np.float32)
        n = len(rv) // 2
        P = np.zeros(4 * (-(-n // U)), np.float32)
        lib().eo_om_group_partials(rv, n, U, P)
        return P.reshape(-1, 4)

    @staticmethod
    def om_grouped(row, s, M2, U, P=None):
        """Oerder-Meyr class sums of the chunk row[s, s + M2) in the wideband grouped order
        (eo_om_grouped) from the group partials P (computed from the row if None)."""
        rv = np.ascontiguousarray(np.asarray(row, np.complex64)).view(np.float32)
        if P is None:
            P = Receiver.om_group_partials(row, U)
        A = np.zeros(4, np.float32)
        lib().eo_om_grouped(rv, s, M2, U, np.ascontiguousarray(P, np.float32).reshape(-1), A)
        return A

    @staticmethod
    def decide(symbols):
        """Table 5.1 differential decision on given symbols (eo_decide): uint8 [n-1]."""
        x = np.ascontiguousarray(np.asarray(symbols, np.complex64)).view(np.float32)
        n = len(x) // 2
        out = np.zeros(max(n - 1, 0), np.uint8)
        if n >= 2:
            lib().eo_decide(x, n, out)
        return out

    @staticmethod
    def hard_bits(hard):
        h = np.asarray(hard, np.uint8)
        return np.stack([(h >> 1) & 1, h & 1], axis=1).reshape(-1).astype(np.uint8)

    def sync(self, hard, maxb=8):
        bits = np.ascontiguousarray(self.hard_bits(hard))
        starts = np.zeros(maxb, np.int32)
        kinds = np.zeros(maxb, np.int32)
        n = lib().eo_sync(bits, len(bits), starts, kinds, maxb)
        return list(zip(starts[:n].tolist(), kinds[:n].tolist()))

    @staticmethod
    def decode_block(soft5, kind, scr):
        n1 = KIND_PARAMS[kind][3]
        out = np.zeros(288, np.uint8)
        ok = lib().eo_decode_block(np.ascontiguousarray(soft5, np.int8), kind,
                                   np.ascontiguousarray(scr[:KIND_PARAMS[kind][0]], np.uint8), out)
        return out[:n1].copy(), bool(ok)

    def lower_mac(self, softbits, hard, cell_init):
        """Bursts -> decoded blocks: [(start, burst_kind, [(kind, type1, crc_ok), ...])]."""
        cell = scramble_seq(cell_init, 432)
        bsch = scramble_seq(3, 120)
        out = []
        for s, bk in self.sync(hard):
            sb = np.asarray(softbits, np.int8)
            blocks = []
            if bk == BURST_NDB_N:
                blocks.append((0, np.concatenate([sb[s + 14:s + 230], sb[s + 282:s + 498]]), cell))
            elif bk == BURST_NDB_P:
                blocks.append((1, sb[s + 14:s + 230], cell))
                blocks.append((1, sb[s + 282:s + 498], cell))
            else:
                blocks.append((2, sb[s + 94:s + 214], bsch))
                blocks.append((1, sb[s + 282:s + 498], cell))
            dec = [(k,) + self.decode_block(v, k, scr) for k, v, scr in blocks]
            out.append((s, bk, dec))
        return out

    def sync_from(self, hard, start, maxb=MAXB):
        """eo_sync_from over a row's dibits from bit `start`: ([(start, kind)], first position not examined)."""
        bits = np.ascontiguousarray(self.hard_bits(hard))
        starts = np.zeros(maxb, np.int32)
        kinds = np.zeros(maxb, np.int32)
        stop = np.zeros(1, np.int32)
        n = lib().eo_sync_from(bits, len(bits), int(start), starts, kinds, maxb, stop)
        return list(zip(starts[:n].tolist(), kinds[:n].tolist())), int(stop[0])

    def decode_bursts(self, softbits, bursts, cell_init):
        cell = scramble_seq(cell_init, 432)
        bsch = scramble_seq(3, 120)
        sb = np.asarray(softbits, np.int8)
        out = []
        for s, bk in bursts:
            if bk == BURST_NDB_N:
                blocks = [(0, np.concatenate([sb[s + 14:s + 230], sb[s + 282:s + 498]]), cell)]
            elif bk == BURST_NDB_P:
                blocks = [(1, sb[s + 14:s + 230], cell), (1, sb[s + 282:s + 498], cell)]
            else:
                blocks = [(2, sb[s + 94:s + 214], bsch), (1, sb[s + 282:s + 498], cell)]
            out.append((s, bk, [(k,) + self.decode_block(v, k, scr) for k, v, scr in blocks]))
        return out

    def lower_mac_acquire(self, softbits, hard, cell_init):
        """Cell acquisition: the chunk's BSCH blocks first (colour code 0); the last CRC-good one
        sets the cell, with which every SCH block of the chunk is then decoded.  Returns
        (lower_mac result, cell init after the chunk)."""
        sb = np.asarray(softbits, np.int8)
        bsch = scramble_seq(3, 120)
        init = int(cell_init)
        for s, bk in self.sync(hard):
            if bk == BURST_SB:
                t, ok = self.decode_block(sb[s + 94:s + 214], 2, bsch)
                if ok:
                    init = bsch_cell_init(t)
        return self.lower_mac(softbits, hard, init), init


# ------------------------------------------------------------------------------ streaming receiver

def stream_lengths(d, n):
    """(M1, M2) of the first n samples of a stream (tetra_etsi_lengths)."""
    m1 = (n - d["L1"]) // d["q1"] + 1 if n >= d["L1"] else 0
    num = d["up"] * m1 - 1 - (d["Lp"] - 1)
    return m1, (num // d["down"] + 1 if num >= 0 else 0)


class Stream:
    """CPU restatement of the streaming receiver (tetra_etsi_stream_window + tetra_demod_etsi_stream +
    tetra_lmac_etsi_stream) for one channel: consecutive chunks of one continuous capture decode as
    one symbol stream -- the channel filter over a window that re-reads the previous chunk's last
    samples (aligned so the polyphase phases equal a run over the whole capture), the timing loop
    (base, delta, last symbol) carried, and the lower MAC's greedy burst scan resumed at the bit it
    stopped at with the unconsumed dibits of the previous chunk in front of the new ones.

    The window of a chunk: with P = q1 down input samples per `up` outputs (doubled when odd, so
    windows hold whole sample pairs; then 2 up outputs), s = P floor((y_done - MARGIN) / (outputs per
    P)) (0 for the first chunk), window = capture[s, x_total), yoff = y_done - up s / (q1 down)."""

    def __init__(self, fs=FS_NOMINAL, cell_init=None):
        self.rx = Receiver(fs)
        d = self.rx.d
        # windows start at multiples of P input samples: q1 down carry `up` outputs; an even P keeps
        # the window an even number of samples (the kernels read sample pairs)
        self.Pb, self.up = d["q1"] * d["down"], d["up"]
        self.P = self.Pb * (2 if self.Pb % 2 else 1)
        self.buf = np.zeros(0, np.complex64)
        self.x_total = self.y_done = 0
        self.trk = np.zeros(1, TRACK)
        self.tail_hard = np.zeros(0, np.uint8)
        self.tail_soft = np.zeros(0, np.int8)
        self.phase = 0
        self.acquire = cell_init is None
        # before a BSCH is decoded: colour code 0 (init 3), what every receiver descrambles with
        self.cell = scramble_init(0, 0, 0) if cell_init is None else int(cell_init)

    def window(self, n):
        """(s, W, yoff, y_start) of the next chunk of n samples (global sample / y indices)."""
        ups = self.up * self.P // self.Pb   # outputs per P input samples
        s = self.P * ((self.y_done - MARGIN) // ups) if self.y_done > 0 else 0
        s = max(s, 0)
        y_start = self.up * s // self.Pb
        return s, self.x_total + n - s, self.y_done - y_start, y_start

    def push(self, x):
        """One chunk (complex64, even length) -> dict(y, symbols, soft, hard, bursts, stop, ...)."""
        x = np.asarray(x, np.complex64)
        s, W, yoff, y_start = self.window(len(x))
        self.buf = np.concatenate([self.buf, x])
        self.x_total += len(x)
        y = self.rx.chanfilt(self.buf[s:self.x_total])
        _, m_hi = stream_lengths(self.rx.d, self.x_total)
        assert len(y) == max(m_hi - y_start, 0), (len(y), m_hi, y_start)
        sym, soft, hard, diag = self.rx.timing_stream(y, yoff, self.trk[0:1])
        self.y_done = max(m_hi, self.y_done)
        # the lower MAC: the tail dibits, then the new ones; scan from the carried phase
        T = len(self.tail_hard)
        row_h = np.concatenate([self.tail_hard, hard])
        row_s = np.concatenate([self.tail_soft, soft])
        if self.acquire:   # BSCH first (colour code 0): the last CRC-good one sets the cell
            bursts, stop = self.rx.sync_from(row_h, self.phase)
            for b0, bk in bursts:
                if bk == BURST_SB:
                    t1, ok = self.rx.decode_block(row_s[b0 + 94:b0 + 214], 2, scramble_seq(3, 120))
                    if ok:
                        self.cell = bsch_cell_init(t1)
        bursts, stop = self.rx.sync_from(row_h, self.phase)
        dec = self.rx.decode_bursts(row_s, bursts, self.cell)
        d0 = stop // 2
        th, ts, ph = row_h[d0:], row_s[2 * d0:], stop & 1
        if len(th) > RESERVE:   # (only past MAXB bursts in one row) keep the last RESERVE dibits
            th, ts, ph = th[-RESERVE:], ts[-2 * RESERVE:], 0
        self.tail_hard, self.tail_soft, self.phase = th.copy(), ts.copy(), ph
        return dict(y=y, yoff=yoff, window=(s, W), symbols=sym, soft=soft, hard=hard, diag=diag,
                    bursts=[(b - 2 * T, k, dd) for b, k, dd in dec], cell=self.cell, stop=stop - 2 * T,
                    track=self.trk.copy())
