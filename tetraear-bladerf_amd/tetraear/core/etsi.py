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


class EtsiLowerMac:
    def __init__(self, mcc=0, mnc=0, colour_code=0):
        self.cell = scrambling_init(mcc, mnc, colour_code)

    def decode_batch(self, soft, hard, nsym, cells=None):
        """soft [C, 2*smax] int8, hard [C, smax] uint8, nsym [C] -> per channel a list of frames."""
        soft = np.ascontiguousarray(soft, np.int8)
        hard = np.ascontiguousarray(hard, np.uint8)
        nsym = np.ascontiguousarray(nsym, np.int32)
        C, smax = hard.shape
        cells = np.full(C, self.cell, np.uint32) if cells is None else np.ascontiguousarray(cells, np.uint32)
        nb = np.zeros(C, np.int32)
        bursts = np.zeros((C, _hip.ETSI_MAXB, 2), np.int32)
        nk = np.zeros(C, np.int32)
        blocks = np.zeros((C, _hip.ETSI_MAXJ, 4), np.int32)
        t1 = np.zeros((C, _hip.ETSI_MAXJ, 268), np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(cells), C), "tetra_etsi_set_cells")
        c.check(c.lib.tetra_lmac_etsi(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), C, smax, _hip.ptr(nb),
                                      _hip.ptr(bursts), _hip.ptr(nk), _hip.ptr(blocks), _hip.ptr(t1)),
                "tetra_lmac_etsi")
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

    def decode(self, symbols, soft_bits=None):
        """One stream of hard dibit symbols (process() output in etsi mode carries soft_bits)."""
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
        return self.decode_batch(soft, hard, np.array([n + 1], np.int32))[0]
