"""Wideband channeliser on the GPU (BASELINE.json configs[2]).

The reference receives one carrier per capture: the BladeRF is tuned to it and 2.4 MSps IQ goes
to SignalProcessor.process (/root/reference/tetraear/ui/modern.py:1886-1887, 2029).  The north
star's "polyphase FIR channeliser" instead takes a 20 MSps capture holding 800 carriers at 25 kHz
spacing and splits it on the device: a polyphase filter bank (libtetra_hip.so k_pfb_analysis2: fold
+ 800-point FFT fused, two blocks per iteration; D = M / 2 by default, so every carrier comes out at
50 kHz), then per carrier an RRC(0.35) matched-filter resampler to 72 kHz (k_pfb_resamp_fix), which
is exactly the sample stream the ETSI timing stage takes (4 samples per symbol, tetra_etsi_timing),
followed by the ETSI lower MAC.  This module designs the filters and moves arrays;
oracle/wideband.py is the float64 specification the tests hold it to.
"""
import collections
import ctypes
import functools
import os

import numpy as np
from scipy import signal as _design

from tetraear import _hip
from tetraear.signal.etsi import etsi_plan, rrc

FS_WB = 20e6
M_WB = 800
M2_CHUNK = 3932     # 72 kHz samples per timing chunk (as a 128 Ki chunk at 2.4 MSps)
# samples consecutive timing chunks share: a whole burst (255 symbols = 1020 samples at 72 kHz) plus
# 15 symbols, so a burst that starts in one chunk ends in it too (TETRA_WB_OVERLAP=0: chunks tile the
# row, the round-1..6 form that loses the burst across every seam -- A/B only)
OV_CHUNK = int(os.environ.get("TETRA_WB_OVERLAP", "1080"))
BURST_SAMPLES = 1020   # one 255-symbol slot at 72 kHz
# Two filter-bank designs (the carrier's output rate fs / D and what it implies):
#   oversample 2 (default): D = M / 2 -> 50 kHz carriers.  A carrier's band aliases onto itself from
#     37.5 kHz, so the prototype is 5 branches long (cut-off 25 kHz, Kaiser 8: 0.003 dB ripple over
#     +-12.5 kHz, 74 dB down from 37.5 kHz); resampler 50 -> 72 kHz = 36 / 25 with 828 RRC taps (23 per
#     output).  Half the blocks of oversample 4: half the FFTs, half the filter-bank output Y.
#   oversample 4 (round 1-3): D = M / 4 -> 100 kHz carriers, 2 branches (cut-off 2 spacings, 72 dB
#     down from 87.5 kHz), resampler 18 / 25 with 810 taps (45 per output).
DESIGNS = {2: dict(P=5, cut=25e3, beta=8.0, up=36, down=25, Lg=828),
           4: dict(P=2, cut=None, beta=7.0, up=18, down=25, Lg=810)}
OVERSAMPLE = int(os.environ.get("TETRA_WB_OVERSAMPLE", "2"))   # 4: the round-3 design (A/B)
# the default design's constants (module attributes the tests and the bench read)
P_WB, UP, DOWN, LG = (DESIGNS[OVERSAMPLE][k] for k in ("P", "up", "down", "Lg"))


@functools.lru_cache(maxsize=8)
def wb_design(fs=FS_WB, M=M_WB, oversample=None):
    """Prototype lowpass h [M P] (unity DC gain, flat over +-12.5 kHz, and down >= 72 dB from the
    first band that aliases onto a carrier at fs / D) and the resampler RRC g [Lg] at up * fs / D."""
    ov = OVERSAMPLE if oversample is None else oversample
    d = DESIGNS[ov]
    D = M // ov
    if abs(fs / D * d["up"] / d["down"] - 72000.0) > 1e-6:
        raise ValueError(f"the channeliser is built for fs / (M / {ov}) = {72000.0 * d['down'] / d['up']:.0f} Hz carriers")
    cut = d["cut"] if d["cut"] is not None else 2.0 * fs / M
    h = _design.firwin(M * d["P"], cut, fs=fs, window=("kaiser", d["beta"])).astype(np.float32)
    sps = fs / D * d["up"] / 18000.0
    g = rrc((np.arange(d["Lg"]) - (d["Lg"] - 1) / 2.0) / sps).astype(np.float32)
    return h, g


class WbPlan:
    """tetra_wb_plan plus the tap arrays it points at."""

    def __init__(self, fs=FS_WB, M=M_WB, oversample=None):
        ov = OVERSAMPLE if oversample is None else oversample
        d = DESIGNS[ov]
        self.h, self.g = wb_design(fs, M, ov)
        p = _hip.WbPlan()
        p.M, p.D, p.P, p.up, p.down, p.Lg, p.fs = M, M // ov, d["P"], d["up"], d["down"], d["Lg"], fs
        p.h = self.h.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        p.g = self.g.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        self.c = p
        self.M, self.D, self.fs, self.oversample = M, M // ov, fs, ov

    def lengths(self, Nw):
        nb, n72 = ctypes.c_int64(), ctypes.c_int64()
        _hip.lib().tetra_wb_lengths(self.c, Nw, ctypes.byref(nb), ctypes.byref(n72))
        return nb.value, n72.value


@functools.lru_cache(maxsize=8)
def wb_plan(fs=FS_WB, M=M_WB, oversample=None):
    return WbPlan(fs, M, oversample)


Chunks = collections.namedtuple("Chunks", "nchunk stride length rowlen")


def chunking(plan, Nw, m2=M2_CHUNK, ov=None):
    """Each carrier's 72 kHz row (rowlen samples kept) is cut into nchunk timing chunks: chunk c is
    row[c m2, min(c m2 + length, rowlen)), length = m2 + ov, so consecutive chunks share ov samples
    and the last one runs to the row's end (tetra_etsi_timing_chunks).  ov = 0: nchunk = n72 // m2
    chunks tiling the first nchunk m2 samples (tetra_etsi_timing_om's layout)."""
    ov = OV_CHUNK if ov is None else ov
    _, n72 = plan.lengths(Nw)
    if ov == 0:
        nchunk = n72 // m2
        if nchunk < 1:
            raise ValueError(f"{Nw} wideband samples give {n72} samples per carrier, less than one chunk of {m2}")
        return Chunks(nchunk, m2, m2, nchunk * m2)
    if ov < 0 or ov % 4 or n72 < 16:
        raise ValueError(f"overlap {ov} (a multiple of 4 >= 0) over {n72} samples per carrier")
    nchunk = max(1, -(-(n72 - ov) // m2))
    return Chunks(nchunk, m2, min(m2 + ov, n72), n72)


def merge_chunks(nburst, bursts, nblock, blocks, M, nchunk, stride, tol=64):
    """The lower MAC's bursts per (carrier, chunk) -> each burst once.  A burst in the ov samples two
    chunks share is found by both; its position in the carrier row (chunk start + 2 x start bit, to
    within the timing phase) tells the copies apart from the next burst (>= BURST_SAMPLES later).
    Returns (keep [C, MAXB] bool: the first copy of every burst, in row order; keep_blocks [C, MAXJ]
    bool: the blocks of kept bursts).  nburst [C], bursts [C][MAXB][2], nblock [C], blocks
    [C][MAXJ][4] as tetra_lmac_etsi leaves them (host arrays)."""
    nburst, bursts = np.asarray(nburst), np.asarray(bursts)
    nblock, blocks = np.asarray(nblock), np.asarray(blocks)
    C, maxb = bursts.shape[:2]
    valid = np.arange(maxb)[None, :] < nburst[:, None]
    ch = np.broadcast_to(np.arange(C)[:, None], (C, maxb))
    pos = (ch % nchunk) * stride + 2 * bursts[..., 0].astype(np.int64)
    car = ch // nchunk
    ci, ji = np.nonzero(valid)
    order = np.lexsort((ci, pos[ci, ji], car[ci, ji]))   # by carrier, row position, then chunk
    ci, ji = ci[order], ji[order]
    pc, cc = pos[ci, ji], car[ci, ji]
    first = np.ones(len(ci), bool)
    first[1:] = (cc[1:] != cc[:-1]) | (pc[1:] - pc[:-1] > tol)
    keep = np.zeros((C, maxb), bool)
    keep[ci[first], ji[first]] = True
    maxj = blocks.shape[1]
    jv = np.arange(maxj)[None, :] < nblock[:, None]
    bi = np.clip(blocks[..., 2], 0, maxb - 1)
    keep_blocks = jv & keep[np.arange(C)[:, None], bi]
    return keep, keep_blocks


def grouped_om(plan, m2=M2_CHUNK):
    """The wideband timing takes its Oerder-Meyr class sums from the resampler's group partials
    (tetra_channelize_om + tetra_etsi_timing_om) where the plan's output groups hold whole classes
    (up a multiple of 4: the D = M / 2 design) and TETRA_WB_OM is not 0."""
    return (plan.c.up % 4 == 0 and plan.c.up <= 64 and m2 % 4 == 0 and m2 >= 16
            and os.environ.get("TETRA_WB_OM", "1") != "0")


class WidebandReceiver:
    """Channeliser + per-carrier ETSI demod (timing, decision) for host or device arrays."""

    def __init__(self, fs=FS_WB, M=M_WB, m2=M2_CHUNK, oversample=None):
        self.plan = wb_plan(fs, M, oversample)
        self.etsi = etsi_plan(2.4e6)   # timing-loop constants (the channel-filter taps are not used)
        self.m2 = m2

    def channelize(self, x, n_keep=None):
        """x [Nw] complex64 -> y [M][n_keep] complex64 at 72 kHz."""
        c = _hip.ctx()
        x = np.ascontiguousarray(x, np.complex64)
        _, n72 = self.plan.lengths(len(x))
        n_keep = n72 if n_keep is None else n_keep
        y = np.empty((self.plan.M, n_keep), np.complex64)
        if n_keep == 0:   # a capture shorter than one 72 kHz output (the oracle's [M, 0])
            return y
        c.check(c.lib.tetra_channelize(c.handle, self.plan.c, _hip.ptr(x), len(x), _hip.ptr(y), n_keep), "channelize")
        return y

    def channelize_om(self, x, n_keep=None):
        """channelize plus the resampler's Oerder-Meyr group partials: (y [M][n_keep] complex64,
        om [M][ceil(n_keep / up)][4] float32) -- D = M / 2 plan only (tetra_channelize_om)."""
        c = _hip.ctx()
        x = np.ascontiguousarray(x, np.complex64)
        _, n72 = self.plan.lengths(len(x))
        n_keep = n72 if n_keep is None else n_keep
        y = np.empty((self.plan.M, n_keep), np.complex64)
        om = np.empty((self.plan.M, -(-n_keep // self.plan.c.up), 4), np.float32)
        if n_keep == 0:
            return y, om
        c.check(c.lib.tetra_channelize_om(c.handle, self.plan.c, _hip.ptr(x), len(x), _hip.ptr(y), n_keep,
                                          _hip.ptr(om)), "channelize_om")
        return y, om

    def grouped_om(self):
        """Whether demod forms the timing's Oerder-Meyr sums in the resampler (the D = M / 2 plan;
        TETRA_WB_OM=0 keeps the timing's own pass over y, for A/B)."""
        return grouped_om(self.plan, self.m2)

    def demod(self, x):
        """x [Nw] -> (hard, soft_bits, sym, nsym) per (carrier, chunk) of chunking(): [M, nchunk,
        smax] uint8, [M, nchunk, 2 smax] int8, [M, nchunk, smax] complex64, [M, nchunk] int32."""
        ck = chunking(self.plan, len(x), self.m2)
        om = None
        if self.grouped_om():
            y, om = self.channelize_om(x, ck.rowlen)
        else:
            y = self.channelize(x, ck.rowlen)
        c = _hip.ctx()
        M = self.plan.M
        C = M * ck.nchunk
        sm = ck.length // 4 + 2
        sym = np.empty((C, sm), np.complex64)
        soft = np.empty((C, 2 * sm), np.int8)
        hard = np.empty((C, sm), np.uint8)
        ns = np.empty(C, np.int32)
        c.check(c.lib.tetra_etsi_timing_chunks(c.handle, self.etsi, _hip.ptr(y), M, ck.rowlen, ck.nchunk, ck.stride,
                                               ck.length, _hip.ptr(om) if om is not None else None,
                                               om.shape[1] if om is not None else 0, self.plan.c.up, _hip.ptr(sym),
                                               _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), sm, None),
                "etsi_timing_chunks")
        return (hard.reshape(M, ck.nchunk, sm), soft.reshape(M, ck.nchunk, 2 * sm), sym.reshape(M, ck.nchunk, sm),
                ns.reshape(M, ck.nchunk))


    def decode(self, x, cells):
        """x [Nw] -> per carrier the frames decoded from it, each burst once (merge_chunks), in row
        order: demod, then the ETSI lower MAC on every (carrier, chunk) with carrier k's scrambling
        init cells[k].  A frame is the lower MAC's dict (core/etsi.py) plus "chunk" and "sample" (its
        start in the carrier's 72 kHz row, to within the timing phase)."""
        from tetraear.core.etsi import EtsiLowerMac
        hard, soft, _, ns = self.demod(x)
        M, nchunk, sm = hard.shape
        C = M * nchunk
        nb = np.zeros(C, np.int32)
        bursts = np.zeros((C, _hip.ETSI_MAXB, 2), np.int32)
        nk = np.zeros(C, np.int32)
        blocks = np.zeros((C, _hip.ETSI_MAXJ, 4), np.int32)
        t1 = np.zeros((C, _hip.ETSI_MAXJ, 268), np.uint8)
        c = _hip.ctx()
        cc = np.ascontiguousarray(np.repeat(np.asarray(cells, np.uint32), nchunk))
        c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(cc), C), "tetra_etsi_set_cells")
        c.check(c.lib.tetra_lmac_etsi(c.handle, _hip.ptr(soft.reshape(C, -1)), _hip.ptr(hard.reshape(C, -1)),
                                      _hip.ptr(ns.reshape(-1)), C, sm, _hip.ptr(nb), _hip.ptr(bursts), _hip.ptr(nk),
                                      _hip.ptr(blocks), _hip.ptr(t1)), "tetra_lmac_etsi")
        keep, _ = merge_chunks(nb, bursts, nk, blocks, M, nchunk, self.m2)
        frames = EtsiLowerMac._frames(C, nb, bursts, nk, blocks, t1)
        out = [[] for _ in range(M)]
        for ch in range(C):
            for b, f in enumerate(frames[ch]):
                if keep[ch, b]:
                    f["chunk"] = ch % nchunk
                    f["sample"] = (ch % nchunk) * self.m2 + 2 * f["position"]
                    out[ch // nchunk].append(f)
        for fr in out:
            fr.sort(key=lambda f: f["sample"])
        return out


class WidebandStream:
    """Consecutive pieces of one continuous wideband capture decoded as one stream (the C3 form of the
    ETSI receiver's streaming, signal/etsi.py EtsiStream): each call channelises the new samples
    behind a tail of the previous ones and WidebandReceiver.decode's frames are kept once per carrier
    by their position in the carrier's whole 72 kHz stream, so a burst across the seam between two
    pieces is decoded too.  The tail starts a whole number of resampler periods (D x down input
    samples -> up outputs) into the buffer, so its outputs are the previous buffer's at the same
    stream positions, bit for bit, and it holds the last CARRY_Y outputs' input: every burst that the
    buffer's end cut is whole in the next one.  The period also holds the filter bank's mixer term
    ((-1)^(k j) at D = M / 2, (-i)^(k j) at M / 4: whole cycles of it), else odd carriers would
    come out negated."""
    CARRY_Y = 2 * BURST_SAMPLES

    def __init__(self, cells, fs=FS_WB, M=M_WB, m2=M2_CHUNK, oversample=None, tol=64):
        self.rx = WidebandReceiver(fs, M, m2, oversample)
        self.cells = np.ascontiguousarray(cells, np.uint32)
        p = self.rx.plan
        blocks = int(np.lcm(p.c.down, p.oversample))   # filter-bank blocks per period
        self.per, self.ups, self.M, self.tol = p.D * blocks, p.c.up * blocks // p.c.down, p.M, tol
        self.reset()

    def reset(self):
        self.tail = np.zeros(0, np.complex64)
        self.y0 = 0                                    # stream position of the buffer's first output
        self.last = np.full(self.M, -(1 << 62), np.int64)   # stream position of each carrier's last frame

    def decode(self, x):
        """x: the next samples of the capture -> per carrier the frames first decoded now, each with
        "stream_sample" (its start in the carrier's 72 kHz stream)."""
        buf = np.concatenate([self.tail, np.asarray(x, np.complex64)])
        _, n72 = self.rx.plan.lengths(len(buf))
        out = [[] for _ in range(self.M)]
        if n72 >= 16:
            for k, fr in enumerate(self.rx.decode(buf, self.cells)):
                for f in fr:
                    a = self.y0 + f["sample"]
                    if a > self.last[k] + self.tol:
                        f["stream_sample"] = int(a)
                        out[k].append(f)
                        self.last[k] = a
        T = max(0, (n72 - self.CARRY_Y) // self.ups) * self.per   # the next buffer starts here
        self.tail = buf[T:]
        self.y0 += self.ups * (T // self.per)
        return out


def synth_wideband(Nw, seed=1, snr_db=30.0, cfo_max=300.0, fs=FS_WB, M=M_WB, oversample=None):
    """Synthetic capture (device-generated, copied to the host): x [Nw] complex64, cells [M],
    kinds [M][NB], payload [M][NB][2][268], t0 [M] (carrier k is FFT bin k, at +k fs/M)."""
    plan = wb_plan(fs, M, oversample)
    c = _hip.ctx()
    nbb = Nw // plan.D + 1
    nb = c.lib.tetra_synth_bursts_per_channel(nbb, fs / plan.D)
    x = np.empty(Nw, np.complex64)
    cells = np.empty(M, np.uint32)
    kinds = np.empty((M, nb), np.int32)
    payload = np.empty((M, nb, 2, 268), np.uint8)
    t0 = np.empty(M, np.float64)
    c.check(c.lib.tetra_synth_wideband(c.handle, plan.c, Nw, seed, snr_db, cfo_max, _hip.ptr(x), _hip.ptr(cells),
                                       _hip.ptr(kinds), _hip.ptr(payload), _hip.ptr(t0)), "synth_wideband")
    return x, cells, kinds, payload, t0


class BenchStep:
    """bench.py --chain wideband (C3): one step = the capture's waterfall rows (2048-pt Hann, hop
    2048), channelise the device-resident 20 MSps capture, timing + decision on every (carrier,
    chunk), lower MAC (sync, Viterbi, CRC) on all of them."""
    dtype = "f32 (DSP), int8/int32 (Viterbi)"

    def __init__(self, c, Nw, seed, device, snr_db=30.0, fs=FS_WB, M=M_WB):
        import torch
        self.c, self.Nw, self.fs = c, Nw, fs
        self.plan = wb_plan(fs, M)
        self.etsi = etsi_plan(2.4e6)
        self.ck = chunking(self.plan, Nw)
        self.nchunk, self.m2 = self.ck.nchunk, self.ck.stride
        self.C = M * self.nchunk
        self.sm = self.ck.length // 4 + 2
        nbb = Nw // self.plan.D + 1
        nb = c.lib.tetra_synth_bursts_per_channel(nbb, fs / self.plan.D)
        self.x = torch.empty((Nw, 2), dtype=torch.float32, device=device)
        cells = torch.empty(M, dtype=torch.int32, device=device)
        self.kinds = torch.empty((M, nb), dtype=torch.int32, device=device)
        self.payload = torch.empty((M, nb, 2, 268), dtype=torch.uint8, device=device)
        c.check(c.lib.tetra_synth_wideband(c.handle, self.plan.c, Nw, seed, snr_db, 300.0, _hip.ptr(self.x),
                                           _hip.ptr(cells), _hip.ptr(self.kinds), _hip.ptr(self.payload), None),
                "synth_wideband")
        c.synchronize()   # torch's ops below need not share the context's stream
        # every chunk of carrier k uses carrier k's scrambling code
        self.cells = cells.repeat_interleave(self.nchunk).contiguous()
        torch.cuda.current_stream(device).synchronize()
        c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(self.cells), self.C), "set_cells")
        self.y = torch.empty((M, self.ck.rowlen, 2), dtype=torch.float32, device=device)
        # the timing's Oerder-Meyr class sums from the resampler (grouped_om): its group partials
        self.om_grouped = grouped_om(self.plan, self.m2)
        self.ngrp = -(-self.ck.rowlen // self.plan.c.up)
        self.om = torch.empty((M, self.ngrp, 4), dtype=torch.float32, device=device) if self.om_grouped else None
        self.sym = torch.empty((self.C, self.sm, 2), dtype=torch.float32, device=device)
        self.soft = torch.empty((self.C, 2 * self.sm), dtype=torch.int8, device=device)
        self.hard = torch.empty((self.C, self.sm), dtype=torch.uint8, device=device)
        self.nsym = torch.empty(self.C, dtype=torch.int32, device=device)
        self.nburst = torch.empty(self.C, dtype=torch.int32, device=device)
        self.bursts = torch.empty((self.C, _hip.ETSI_MAXB, 2), dtype=torch.int32, device=device)
        self.nblock = torch.empty(self.C, dtype=torch.int32, device=device)
        self.blocks = torch.empty((self.C, _hip.ETSI_MAXJ, 4), dtype=torch.int32, device=device)
        self.type1 = torch.empty((self.C, _hip.ETSI_MAXJ, 268), dtype=torch.uint8, device=device)
        self.nfr = Nw // 2048   # waterfall rows of the capture (2048-pt Hann frames, hop 2048)
        self.wf = torch.empty((self.nfr, 2048), dtype=torch.float32, device=device)
        self.pipelined = False
        self.mid = None

    def pipeline(self):
        """Software pipeline over consecutive captures: the channeliser of step k+2 on the front
        stream while the per-carrier timing of step k+1 runs on a middle stream and the waterfall rows
        and the lower MAC of step k on a back stream (each its own context).  The carrier samples y
        (with their Oerder-Meyr partials) and the timing's outputs are what crosses the streams:
        double-buffered, each stage waits only on the events that protect its buffers.  Every step
        still does the whole chain."""
        import torch
        dev = self.x.device
        self.back = _hip.Context()
        # the waterfall rows go on the back stream, beside the channeliser (the front stream, the longer
        # of the two): 0.436 against 0.446 ms per step, same box (profiles/r04_ab_wideband_streams.txt);
        # TETRA_WB_WF_BACK=0 keeps them on the front.  TETRA_WB_FRONT_PRIO=1 runs the channeliser on a
        # high-priority stream of its own (no gain)
        self.wf_back = os.environ.get("TETRA_WB_WF_BACK", "1") == "1"
        if os.environ.get("TETRA_WB_FRONT_PRIO") == "1":
            self.s_front = torch.cuda.Stream(device=dev, priority=-1)
            self.c.check(self.c.lib.tetra_set_stream(self.c.handle, ctypes.c_void_p(self.s_front.cuda_stream)),
                         "set_stream")
        else:
            self.s_front = torch.cuda.current_stream(dev)
        self.s_back = torch.cuda.Stream(device=dev)
        self.back.check(self.back.lib.tetra_set_stream(self.back.handle, ctypes.c_void_p(self.s_back.cuda_stream)),
                        "set_stream")
        self.back.check(self.back.lib.tetra_etsi_set_cells(self.back.handle, _hip.ptr(self.cells), self.C), "set_cells")
        self.ys = [self.y, torch.empty_like(self.y)]
        self.oms = [self.om, torch.empty_like(self.om) if self.om is not None else None]
        self.ev_front = [torch.cuda.Event() for _ in range(2)]
        self.ev_back = [torch.cuda.Event() for _ in range(2)]
        for e in self.ev_back:
            e.record(self.s_back)
        # three streams (default): the timing on a middle stream of its own, the lower MAC (and the
        # waterfall rows) on the back stream -- three captures in flight; the timing's outputs (symbols,
        # soft bits, dibits, counts) are then double-buffered too.  Same box: 0.386-0.387 ms per step
        # against 0.397-0.415 with two streams (profiles/r04_ab_wb_stages.txt).  TETRA_WB_STAGES=2: the
        # two-stream form (timing + lower MAC on the back stream)
        self.mid = None
        if os.environ.get("TETRA_WB_STAGES", "3") == "3":
            self.mid = _hip.Context()
            self.s_mid = torch.cuda.Stream(device=dev)
            self.mid.check(self.mid.lib.tetra_set_stream(self.mid.handle, ctypes.c_void_p(self.s_mid.cuda_stream)),
                           "set_stream")
            self.outs = [(self.sym, self.soft, self.hard, self.nsym)]
            self.outs.append(tuple(torch.empty_like(t) for t in self.outs[0]))
            self.ev_mid = [torch.cuda.Event() for _ in range(2)]
            for e in self.ev_mid:
                e.record(self.s_mid)
        self.k = 0
        self.pipelined = True
        return self

    def contexts(self):
        return [self.c] + ([self.back] if self.pipelined else []) + ([self.mid] if self.mid is not None else [])

    def _waterfall(self, c):
        c.check(c.lib.tetra_waterfall(c.handle, _hip.ptr(self.x), _hip.TETRA_CF32, 1, self.Nw, 2048, 2048, self.nfr,
                                      _hip.ptr(self.wf)), "waterfall")

    def _front(self, c, y, om):
        if not (self.pipelined and self.wf_back):
            self._waterfall(c)
        if om is not None:
            c.check(c.lib.tetra_channelize_om(c.handle, self.plan.c, _hip.ptr(self.x), self.Nw, _hip.ptr(y),
                                              self.ck.rowlen, _hip.ptr(om)), "channelize_om")
        else:
            c.check(c.lib.tetra_channelize(c.handle, self.plan.c, _hip.ptr(self.x), self.Nw, _hip.ptr(y),
                                           self.ck.rowlen), "channelize")

    def _timing(self, c, y, om):
        ck = self.ck
        c.check(c.lib.tetra_etsi_timing_chunks(c.handle, self.etsi, _hip.ptr(y), self.plan.M, ck.rowlen, ck.nchunk,
                                               ck.stride, ck.length, _hip.ptr(om), self.ngrp if om is not None else 0,
                                               self.plan.c.up, _hip.ptr(self.sym), _hip.ptr(self.soft),
                                               _hip.ptr(self.hard), _hip.ptr(self.nsym), self.sm, None),
                "etsi_timing_chunks")

    def _lmac(self, c):
        c.check(c.lib.tetra_lmac_etsi(c.handle, _hip.ptr(self.soft), _hip.ptr(self.hard), _hip.ptr(self.nsym), self.C,
                                      self.sm, _hip.ptr(self.nburst), _hip.ptr(self.bursts), _hip.ptr(self.nblock),
                                      _hip.ptr(self.blocks), _hip.ptr(self.type1)), "lmac_etsi")

    def _back(self, c, y, om):
        if self.pipelined and self.wf_back:
            self._waterfall(c)
        self._timing(c, y, om)
        self._lmac(c)

    def __call__(self):
        if not self.pipelined:
            self._front(self.c, self.y, self.om)
            self._back(self.c, self.y, self.om)
            return
        i = self.k & 1
        self.k += 1
        y, om = self.ys[i], self.oms[i]
        self.s_front.wait_event(self.ev_back[i] if self.mid is None else self.ev_mid[i])   # y[i], om[i] consumed
        self._front(self.c, y, om)
        self.ev_front[i].record(self.s_front)
        if self.mid is None:
            self.s_back.wait_event(self.ev_front[i])
            self._back(self.back, y, om)
            self.ev_back[i].record(self.s_back)
            return
        # three streams: timing of this capture on the middle one once its channeliser is done and the
        # lower MAC two captures back has consumed output buffer i; the lower MAC on the back one
        self.sym, self.soft, self.hard, self.nsym = self.outs[i]
        self.s_mid.wait_event(self.ev_front[i])
        self.s_mid.wait_event(self.ev_back[i])
        self._timing(self.mid, y, om)
        self.ev_mid[i].record(self.s_mid)
        self.s_back.wait_event(self.ev_mid[i])
        if self.wf_back:
            self._waterfall(self.back)
        self._lmac(self.back)
        self.ev_back[i].record(self.s_back)

    def stage_bytes(self):
        """Algorithmic bytes per wideband input sample of each timed stage (cf32 = 8 B):
        the fused analysis (M = 800) and the fold read x and write Y (M per D samples), the FFT reads and writes Y, the resampler reads
        Y and writes y (M carriers at 72 kHz), the timing stage reads y and writes per symbol an
        8 B symbol, 2 soft bits and a hard dibit -- the samples two chunks share twice (cover =
        the chunks' total length over the row's).  bench.py reports the slowest of them."""
        M, D, fs, ck = self.plan.M, self.plan.D, self.fs, self.ck
        yb = 8.0 * M * 72000.0 / fs
        cover = ((ck.nchunk - 1) * ck.length + ck.rowlen - (ck.nchunk - 1) * ck.stride) / ck.rowlen
        ana = "k_pfb_analysis2" if os.environ.get("TETRA_WB_ANALYSIS") == "2" else \
            ("k_pfb_analysis1" if self.plan.oversample == 2 else "k_pfb_analysis")
        return {"waterfall": (12.0 * self.nfr * 2048 / self.Nw, "k_waterfall"),
                "wb_analysis": (8.0 + 8.0 * M / D, ana),   # fused fold + FFT: x in, Y out
                "wb_fold": (8.0 + 8.0 * M / D, "k_pfb_fold"), "wb_fft": (2 * 8.0 * M / D, None),
                "wb_resamp": (8.0 * M / D + yb + (yb * 2.0 / self.plan.c.up if self.om_grouped else 0.0),
                              "k_pfb_resamp_fix"),
                "etsi_timing": (cover * (yb + 11.0 * M * 18000.0 / fs), "k_timing")}

    def config(self, world):
        return {"workload": f"C3: {self.Nw} samples of a {self.fs / 1e6:g} MSps capture per GPU, "
                            f"{self.plan.M} carriers x {self.nchunk} timing chunks of {self.ck.length} "
                            f"every {self.m2}",
                "wideband_samples_per_gpu": self.Nw, "sample_rate": self.fs, "carriers": self.plan.M,
                "timing_chunks_per_carrier": self.nchunk, "timing_chunk_overlap": self.ck.length - self.m2,
                "parallelism": f"capture-sharded x{world}",
                "filter_bank": f"D = M / {self.plan.oversample} ({self.fs / self.plan.D / 1e3:g} kHz carriers)",
                "pipeline": self.pipelined}

    def realtime_channels(self, value_msps):
        return value_msps * 1e6 / self.fs * self.plan.M   # carriers served at real time

    def workload_key(self):
        return f"C3: {self.Nw} samples"   # a substring of config()["workload"]

    def quality(self):
        """The last step's decoded work, each burst once (merge_chunks): bursts, blocks, CRC-good
        blocks, and decoded_frac = bursts / the slots on air (M rows of rowlen samples, 1020 per
        slot; a slot cut by the capture's start or end cannot be decoded, so ~0.97-0.99 is whole)."""
        nb, bursts = self.nburst.cpu().numpy(), self.bursts.cpu().numpy()
        nk, blocks = self.nblock.cpu().numpy(), self.blocks.cpu().numpy()
        keep, kb = merge_chunks(nb, bursts, nk, blocks, self.plan.M, self.nchunk, self.m2)
        slots = self.plan.M * self.ck.rowlen / BURST_SAMPLES
        return dict(blocks=int(kb.sum()), crc_ok=int((blocks[..., 1].astype(bool) & kb).sum()),
                    bursts=int(keep.sum()), decoded_frac=round(float(keep.sum()) / slots, 4),
                    per_chunk=dict(bursts=int(nb.sum()), blocks=int(nk.sum())))
