"""ETSI lower MAC on the GPU: burst sync, descrambling, deinterleaving, RCPC Viterbi, CRC-16.

The reference slices bursts at a fixed offset and checks a "simplified" CRC on raw bits
(/root/reference/tetraear/core/decoder.py:835-888, protocol.py:292-329); it never channel-decodes.
This module decodes what the north star asks for (EN 300 392-2 §8.2, §9.4.4):
  normal continuous downlink burst, training sequence n -> one SCH/F block (432 -> 268 bits)
                                    training sequence p -> two SCH/HD blocks (216 -> 124 bits)
  synchronisation burst -> BSCH (120 -> 60 bits, colour code 0) + SCH/HD on block 2
The work runs in tetra_lmac_etsi (k_lmac_etsi); this module packages results as frame dicts.
"""
import numpy as np

from tetraear import _hip

BLOCK_NAMES = {0: "SCH/F", 1: "SCH/HD", 2: "BSCH"}
BURST_NAMES = {0: "NDB (n)", 1: "NDB (p)", 2: "SB"}
KIND_N1 = {0: 268, 1: 124, 2: 60}


def scrambling_init(mcc, mnc, colour_code):
    """EN 300 392-2 §8.2.5.2: 30-bit extended colour code with two leading ones."""
    return ((((mcc & 0x3FF) << 20) | ((mnc & 0x3FFF) << 6) | (colour_code & 0x3F)) << 2) | 3


def cell_of(init):
    """(MCC, MNC, colour code) of a scrambling init."""
    ecc = int(init) >> 2
    return (ecc >> 20) & 0x3FF, (ecc >> 6) & 0x3FFF, ecc & 0x3F


UNKNOWN_CELL = scrambling_init(0, 0, 0)   # colour code 0: what a receiver descrambles with before the BSCH


def acquired_channels(nblock, blocks):
    """[C] bool: the channel's call decoded a CRC-good BSCH block (block kind 2), i.e. the cell
    k_cell_acquire keeps came from a SYNC PDU of this call."""
    nblock = np.asarray(nblock)
    blocks = np.asarray(blocks)
    live = np.arange(blocks.shape[1])[None, :] < nblock[:, None]
    return np.any(live & (blocks[:, :, 0] == 2) & (blocks[:, :, 1] != 0), axis=1)


class EtsiLowerMac:
    """Lower MAC of the ETSI chain.  With a cell (mcc, mnc, colour_code) every channel is
    descrambled with it.  Without one the receiver acquires the cell itself: each chunk's BSCH
    blocks are decoded first with colour code 0, and the SYNC PDU of the last CRC-good one gives the
    channel's MCC / MNC / colour code (tetra_lmac_etsi_acquire).  The acquired cell persists across
    calls per channel -- the state the reference parser keeps from a SYSINFO broadcast
    (/root/reference/tetraear/core/protocol.py:479-485) -- and is exposed as ``cells`` /
    ``mcc`` / ``mnc`` / ``colour_code``."""

    def __init__(self, mcc=None, mnc=None, colour_code=None):
        self.acquire = mcc is None and mnc is None and colour_code is None
        self.cell = None if self.acquire else scrambling_init(mcc or 0, mnc or 0, colour_code or 0)
        self.cell_state = None   # [C] scrambling inits of the acquired cells (acquisition mode)
        # [C] bool: a CRC-good BSCH has been decoded on the channel.  Kept apart from cell_state,
        # because an all-zero cell (MCC = MNC = CC = 0) has the init of UNKNOWN_CELL.
        self.acquired = None
        self.reset_stream()

    def reset_stream(self):
        """decode_stream / decode start a new capture: no carried dibits."""
        self._rows = None   # (soft rows [C, 2 stride], hard rows [C, stride], lead [C]): the carried tails

    @property
    def cells(self):
        """Per channel (MCC, MNC, colour code) acquired so far, None where no BSCH decoded yet."""
        if self.cell_state is None:
            return []
        return [cell_of(v) if a else None for v, a in zip(self.cell_state, self.acquired)]

    @property
    def mcc(self):
        c = self.cells[0] if self.cells else None
        return None if c is None else c[0]

    @property
    def mnc(self):
        c = self.cells[0] if self.cells else None
        return None if c is None else c[1]

    @property
    def colour_code(self):
        c = self.cells[0] if self.cells else None
        return None if c is None else c[2]

    def decode_batch(self, soft, hard, nsym, cells=None):
        """soft [C, 2*smax] int8, hard [C, smax] uint8, nsym [C] -> per channel a list of frames.
        ``cells`` ([C] scrambling inits) overrides the receiver's cell for this call."""
        soft = np.ascontiguousarray(soft, np.int8)
        hard = np.ascontiguousarray(hard, np.uint8)
        nsym = np.ascontiguousarray(nsym, np.int32)
        C, smax = hard.shape
        nb = np.zeros(C, np.int32)
        bursts = np.zeros((C, _hip.ETSI_MAXB, 2), np.int32)
        nk = np.zeros(C, np.int32)
        blocks = np.zeros((C, _hip.ETSI_MAXJ, 4), np.int32)
        t1 = np.zeros((C, _hip.ETSI_MAXJ, 268), np.uint8)
        c = _hip.ctx()
        if self.acquire and cells is None:
            if self.cell_state is None or len(self.cell_state) != C:
                self.cell_state = np.full(C, UNKNOWN_CELL, np.uint32)
                self.acquired = np.zeros(C, bool)
            if self.acquired is None or len(self.acquired) != C:   # cell_state handed in from outside
                self.acquired = np.zeros(C, bool)
            c.check(c.lib.tetra_lmac_etsi_acquire(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), C, smax,
                                                  _hip.ptr(self.cell_state), _hip.ptr(nb), _hip.ptr(bursts),
                                                  _hip.ptr(nk), _hip.ptr(blocks), _hip.ptr(t1)),
                    "tetra_lmac_etsi_acquire")
            self.acquired |= acquired_channels(nk, blocks)
        else:
            cells = np.full(C, self.cell if self.cell is not None else UNKNOWN_CELL, np.uint32) if cells is None \
                else np.ascontiguousarray(cells, np.uint32)
            c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(cells), C), "tetra_etsi_set_cells")
            c.check(c.lib.tetra_lmac_etsi(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), C, smax,
                                          _hip.ptr(nb), _hip.ptr(bursts), _hip.ptr(nk), _hip.ptr(blocks), _hip.ptr(t1)),
                    "tetra_lmac_etsi")
        return self._frames(C, nb, bursts, nk, blocks, t1)

    def _run_stream(self, c, C, nb, bursts, nk, blocks, t1, cells, stream):
        """tetra_lmac_etsi_stream over stream = (soft rows, hard rows, nsym, stride, lead), with the
        receiver's cell handling (acquisition state or configured cells) as decode_batch's."""
        if self.acquire and cells is None:
            if self.cell_state is None or len(self.cell_state) != C:
                self.cell_state = np.full(C, UNKNOWN_CELL, np.uint32)
                self.acquired = np.zeros(C, bool)
            if self.acquired is None or len(self.acquired) != C:   # cell_state handed in from outside
                self.acquired = np.zeros(C, bool)
            ci = _hip.ptr(self.cell_state)
        else:
            cells = np.full(C, self.cell if self.cell is not None else UNKNOWN_CELL, np.uint32) if cells is None \
                else np.ascontiguousarray(cells, np.uint32)
            c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(cells), C), "tetra_etsi_set_cells")
            ci = None
        srow, hrow, ns, stride, lead = stream
        c.check(c.lib.tetra_lmac_etsi_stream(c.handle, _hip.ptr(srow), _hip.ptr(hrow), _hip.ptr(ns), C, stride,
                                             _hip.ptr(lead), _hip.ptr(srow), _hip.ptr(hrow), ci, _hip.ptr(nb),
                                             _hip.ptr(bursts), _hip.ptr(nk), _hip.ptr(blocks), _hip.ptr(t1)),
                "tetra_lmac_etsi_stream")
        if ci is not None:
            self.acquired |= acquired_channels(nk, blocks)

    def decode_stream(self, soft, hard, nsym, cells=None):
        """decode_batch for consecutive chunks of C continuous streams (EtsiStream.demod rows):
        each channel's dibits the previous call left unconsumed -- from the first bit its burst scan
        did not examine -- go in front of this chunk's, and the scan resumes there
        (tetra_lmac_etsi_stream), so a burst across the seam is decoded whole.  Positions are
        relative to this chunk's first dibit (negative: the burst began in the carried tail)."""
        soft = np.ascontiguousarray(soft, np.int8)
        hard = np.ascontiguousarray(hard, np.uint8)
        nsym = np.ascontiguousarray(nsym, np.int32)
        C, smax = hard.shape
        R = _hip.ETSI_RESERVE
        if self._rows is None or self._rows[1].shape[0] != C or self._rows[1].shape[1] < R + smax:
            stride = R + max(smax, self._rows[1].shape[1] - R if self._rows is not None and
                             self._rows[1].shape[0] == C else 0)
            srow, hrow = np.zeros((C, 2 * stride), np.int8), np.zeros((C, stride), np.uint8)
            lead = np.full(C, 2 * R, np.int32)
            if self._rows is not None and self._rows[1].shape[0] == C:   # keep the carried tails
                srow[:, :2 * R], hrow[:, :R] = self._rows[0][:, :2 * R], self._rows[1][:, :R]
                lead = self._rows[2]
            self._rows = (srow, hrow, lead)
        srow, hrow, lead = self._rows
        stride = hrow.shape[1]
        hrow[:, R:R + smax] = hard
        srow[:, 2 * R:2 * R + 2 * smax] = soft
        nb = np.zeros(C, np.int32)
        bursts = np.zeros((C, _hip.ETSI_MAXB, 2), np.int32)
        nk = np.zeros(C, np.int32)
        blocks = np.zeros((C, _hip.ETSI_MAXJ, 4), np.int32)
        t1 = np.zeros((C, _hip.ETSI_MAXJ, 268), np.uint8)
        self._run_stream(_hip.ctx(), C, nb, bursts, nk, blocks, t1, cells, (srow, hrow, nsym, stride, lead))
        return self._frames(C, nb, bursts, nk, blocks, t1)

    @staticmethod
    def _frames(C, nb, bursts, nk, blocks, t1):
        out = []
        for ch in range(C):
            frames = []
            for b in range(int(nb[ch])):
                start, kind = int(bursts[ch, b, 0]), int(bursts[ch, b, 1])
                blks = []
                for j in range(int(nk[ch])):
                    if blocks[ch, j, 2] != b:
                        continue
                    k = int(blocks[ch, j, 0])
                    blks.append({"channel": BLOCK_NAMES[k], "crc_ok": bool(blocks[ch, j, 1]),
                                 "bits": t1[ch, j, :KIND_N1[k]].copy(), "block": int(blocks[ch, j, 3])})
                frames.append({"position": start, "burst": BURST_NAMES[kind], "burst_kind": kind,
                               "timeslot": (start // 510) % 4, "blocks": blks,
                               "crc_ok": all(x["crc_ok"] for x in blks)})
            out.append(frames)
        return out

    def decode(self, symbols, soft_bits=None, stream=True):
        """One chunk of hard dibit symbols (process() output in etsi mode carries soft_bits).
        ``stream`` (default): the chunk continues the stream of the previous calls (decode_stream;
        TetraDecoder(mode='etsi').decode behind SignalProcessor(mode='etsi').process, as the
        reference's capture loop calls them chunk after chunk); reset_stream() starts a new one.
        ``stream=False``: the chunk on its own (decode_batch)."""
        h = np.asarray(symbols, np.uint8)
        sb = soft_bits if soft_bits is not None else getattr(symbols, "soft_bits", None)
        if sb is None:   # hard decisions only: +-64 soft values
            bits = np.stack([(h >> 1) & 1, h & 1], axis=1).reshape(-1)
            sb = np.where(bits == 0, 64, -64).astype(np.int8)
        n = len(h)
        smax = n + 2
        hard = np.zeros((1, smax), np.uint8)
        hard[0, :n] = h
        soft = np.zeros((1, 2 * smax), np.int8)
        soft[0, :2 * n] = np.asarray(sb, np.int8)[:2 * n]
        if stream:
            return self.decode_stream(soft, hard, np.array([n + 1], np.int32))[0]
        return self.decode_batch(soft, hard, np.array([n + 1], np.int32))[0]
