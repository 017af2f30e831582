#!/usr/bin/env python3
"""Golden fixtures for TetraProtocolParser.parse_mac_pdu (TEST INFRASTRUCTURE).

Runs the REFERENCE (/root/reference/tetraear/core/protocol.py:349-596) in this container, with the
oracle's ``bitstring`` shim on sys.path (bitstring, requirements.txt:5, is not installed), over
seeded sequences of data-bit vectors, each sequence on ONE parser instance (the parse is stateful:
fragment buffer, MCC/MNC/colour code, frame counters).  Only inputs and outputs are stored:

    python tests/golden/make_golden_mac.py      # writes tests/golden/g4_mac.npz

Per call: the bits; None or the MacPDU fields (pdu_type value, encrypted, address or -1, length,
fill_bits, encryption_mode, data bytes, reassembled_data or none); the parser state after the call
(mcc / mnc / colour_code or -1, clear/encrypted frame counters, fragment buffer, fragment address).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("TETRA_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "oracle", "shim"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import logging  # noqa: E402

logging.disable(logging.CRITICAL)
from tetraear.core.protocol import TetraProtocolParser  # noqa: E402  (the reference)


def bits_of(v, n):
    return [(v >> (n - 1 - i)) & 1 for i in range(n)]


def vector(rng, kind=None):
    """One data-bit vector: a structured header of a random PDU type followed by random bits."""
    L = int(rng.choice([0, 3, 7, 8, 9, 20, 28, 34, 35, 40, 41, 60, 108, 124, 216, 230, 268, 432, 510]))
    b = list(rng.integers(0, 2, L))
    if L < 8:
        return b
    pdu = int(rng.integers(0, 4)) if kind is None else kind
    b[0], b[1] = pdu >> 1, pdu & 1
    if pdu == 2 and L >= 34 and rng.random() < 0.7:   # MAC-BROADCAST SYSINFO: MCC(10) MNC(14) CC(6)
        b[2] = b[3] = 0
        mcc = int(rng.choice([int(rng.integers(200, 800)), int(rng.integers(0, 200)), int(rng.integers(800, 1024))]))
        mnc = int(rng.choice([int(rng.integers(0, 1000)), int(rng.integers(1000, 16384))]))
        b[4:34] = bits_of(mcc, 10) + bits_of(mnc, 14) + bits_of(int(rng.integers(0, 64)), 6)
    elif pdu in (0, 3):   # length indicator near the strict-check boundary
        pos = 5 + (24 if pdu == 0 else 0)
        if L >= pos + 6:
            room = L - pos - 6
            ln = int(np.clip(rng.choice([room // 8, (room + 16) // 8, (room + 16) // 8 + 1, room // 8 - 1, 0,
                                         int(rng.integers(0, 64))]), 0, 63))
            b[pos:pos + 6] = bits_of(ln, 6)
    return b


def main():
    rng = np.random.default_rng(20261016)
    seqs = []
    # the reference's own unit-test inputs (tests/unit/test_tetra_protocol.py:101-115)
    seqs.append([[0] * 4, [0, 0] + [0, 1] * 50])
    # fragment chains: RESOURCE, FRAG..., END; END / FRAG with nothing before them
    for _ in range(12):
        chain = [vector(rng, 0)] + [vector(rng, 1) for _ in range(int(rng.integers(0, 3)))] + [vector(rng, 3)]
        seqs.append(chain)
    seqs.append([vector(rng, 3), vector(rng, 1), vector(rng, 3)])
    # random sequences
    for _ in range(40):
        seqs.append([vector(rng) for _ in range(int(rng.integers(1, 9)))])

    rec = {k: [] for k in ("seq", "bits_off", "none", "ptype", "enc", "addr", "length", "fill", "mode",
                           "data_off", "reasm", "reasm_off", "mcc", "mnc", "cc", "n_clear", "n_enc",
                           "frag_off", "frag_addr")}
    bits_all, data_all, reasm_all, frag_all = [], [], [], []
    for si, seq in enumerate(seqs):
        p = TetraProtocolParser()
        for v in seq:
            a = np.array(v, dtype=np.int64)
            r = p.parse_mac_pdu(a)
            rec["seq"].append(si)
            rec["bits_off"].append(len(bits_all))
            bits_all.extend(v)
            rec["none"].append(r is None)
            rec["ptype"].append(-1 if r is None else r.pdu_type.value)
            rec["enc"].append(-1 if r is None else int(bool(r.encrypted)))
            rec["addr"].append(-1 if r is None or r.address is None else int(r.address))
            rec["length"].append(-1 if r is None else int(r.length))
            rec["fill"].append(-1 if r is None else int(r.fill_bits))
            rec["mode"].append(-1 if r is None else int(r.encryption_mode))
            rec["data_off"].append(len(data_all))
            data_all.extend(b"" if r is None else r.data)
            rec["reasm"].append(r is not None and r.reassembled_data is not None)
            rec["reasm_off"].append(len(reasm_all))
            reasm_all.extend(b"" if r is None or r.reassembled_data is None else r.reassembled_data)
            rec["mcc"].append(-1 if p.mcc is None else p.mcc)
            rec["mnc"].append(-1 if p.mnc is None else p.mnc)
            rec["cc"].append(-1 if p.colour_code is None else p.colour_code)
            rec["n_clear"].append(p.stats["clear_mode_frames"])
            rec["n_enc"].append(p.stats["encrypted_frames"])
            rec["frag_off"].append(len(frag_all))
            frag_all.extend(bytes(p.fragment_buffer))
            fa = p.fragment_metadata.get("address") if p.fragment_metadata else None
            rec["frag_addr"].append(-2 if not p.fragment_metadata else (-1 if fa is None else fa))
    n = len(rec["seq"])
    for k in ("bits_off", "data_off", "reasm_off", "frag_off"):
        rec[k].append({"bits_off": len(bits_all), "data_off": len(data_all), "reasm_off": len(reasm_all),
                       "frag_off": len(frag_all)}[k])
    out = {k: np.asarray(v, dtype=np.int64) for k, v in rec.items()}
    out["bits"] = np.asarray(bits_all, dtype=np.uint8)
    out["data"] = np.frombuffer(bytes(data_all), dtype=np.uint8)
    out["reasm_data"] = np.frombuffer(bytes(reasm_all), dtype=np.uint8)
    out["frag"] = np.frombuffer(bytes(frag_all), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "g4_mac.npz"), **out)
    print(f"g4_mac.npz: {len(seqs)} sequences, {n} calls, {int(np.sum(out['none']))} None")


if __name__ == "__main__":
    main()
