"""The wave-parallel burst CRC of k_lmac (csrc/compat_lmac.hip: LinCrc, check_crc_wave) restated on
the CPU and checked against the oracle's bitwise _check_crc (oracle/compat.py: check_crc, which
restates /root/reference/tetraear/core/protocol.py:292-329 and is pinned to the reference's golden
vectors).  The kernel computes the forward and the reversed CRC-16 registers as XORs of per-position
table entries (t[d] = S^(d+1)(0x8000)) from init[n] = S^n(0xFFFF); this test pins that algebra on
random and edge-case bursts of every length the decoder uses."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import compat as oracle  # noqa: E402

N = 494


def _step(c):
    return (((c << 1) ^ 0x1021) if c & 0x8000 else (c << 1)) & 0xFFFF


def _tables():
    t, r = [], _step(0x8000)
    for _ in range(N):
        t.append(r)
        r = _step(r)
    init, s = [], 0xFFFF
    for _ in range(N + 1):
        init.append(s)
        s = _step(s)
    return np.array(t), np.array(init)


T, INIT = _tables()


def check_crc_linear(bits):
    """check_crc_wave's arithmetic (lane order does not matter: XOR / OR / + are associative)."""
    b = np.asarray(bits, dtype=np.int64) & 1
    L = len(b)
    if L < 16:
        return False
    n = L - 16
    ones = int(b.sum())
    idx = np.nonzero(b[:n])[0]
    c = int(INIT[n]) ^ int(np.bitwise_xor.reduce(T[n - 1 - idx], initial=0))
    r = int(INIT[n]) ^ int(np.bitwise_xor.reduce(T[idx], initial=0))
    rx = 0
    for k in range(16):
        rx = (rx << 1) | int(b[L - 16 + k])
    if ones == 0 or ones == L:
        return False
    return bin(c ^ rx).count("1") <= 2 or bin(r ^ rx).count("1") <= 2


def _crc_reg(bits):
    c = 0xFFFF
    for x in bits:
        c ^= (int(x) & 1) << 15
        c = _step(c)
    return c


def test_registers_match_bitwise():
    rng = np.random.default_rng(3)
    for L in (17, 32, 216, 300, 510):
        for _ in range(50):
            b = rng.integers(0, 2, L)
            n = L - 16
            idx = np.nonzero(b[:n])[0]
            assert _crc_reg(b[:n]) == int(INIT[n]) ^ int(np.bitwise_xor.reduce(T[n - 1 - idx], initial=0))
            assert _crc_reg(b[:n][::-1]) == int(INIT[n]) ^ int(np.bitwise_xor.reduce(T[idx], initial=0))


def test_check_crc_matches_oracle():
    rng = np.random.default_rng(4)
    cases = []
    for L in (15, 16, 17, 216, 510):
        cases += [np.zeros(L, np.uint8), np.ones(L, np.uint8)]
        cases += [rng.integers(0, 2, L).astype(np.uint8) for _ in range(200)]
    # bursts whose CRC field holds the forward / reversed register, with 0-3 bit errors in the CRC
    for L in (216, 510):
        for k in range(40):
            b = rng.integers(0, 2, L).astype(np.uint8)
            reg = _crc_reg(b[:L - 16]) if k % 2 == 0 else _crc_reg(b[:L - 16][::-1])
            b[L - 16:] = [(reg >> (15 - j)) & 1 for j in range(16)]
            for e in rng.choice(16, size=k % 4, replace=False):
                b[L - 16 + e] ^= 1
            cases.append(b)
    got = [check_crc_linear(b) for b in cases]
    want = [oracle.check_crc(b) for b in cases]
    assert got == want
    assert sum(want) >= 60   # the CRC-good side is exercised
