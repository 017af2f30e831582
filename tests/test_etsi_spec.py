"""The ETSI oracle against a second, independent restatement of the spec (oracle/etsi_spec.py, CPU).

oracle/etsi_oracle.c is what the GPU chain is bit-identical to.  Here it is checked against
etsi_spec.py, which restates EN 300 392-2 §8.2.3-§8.2.5 in another formulation (polynomial CRC,
polynomial-product mother code, the puncturing / interleaving index formulas, the scrambler
recurrence), and the Viterbi against the maximum-likelihood property.  Parity with the reference
stays unpinned for this chain (the reference has none); see DESIGN.md §3.
"""
import numpy as np
import pytest

import etsi as E
import etsi_spec as S


def test_crc_known_answers():
    m = np.array([(b >> (7 - k)) & 1 for b in b"123456789" for k in range(8)], np.uint8)
    assert S.crc16_value(m) == 0xD64E                       # CRC-16 with ones' complement, check value
    reg = E.crc16_reg(np.concatenate([m, S.crc_bits(m)]))    # the oracle's register over data + CRC
    assert reg == 0x1D0F                                    # the residue of a good block


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_crc_polynomial_vs_oracle_register(kind):
    rng = np.random.default_rng(kind)
    n1 = S.KINDS[kind]["n1"]
    for _ in range(50):
        m = rng.integers(0, 2, n1).astype(np.uint8)
        good = np.concatenate([m, S.crc_bits(m)])
        assert E.crc16_reg(good) == 0x1D0F
        bad = good.copy()
        bad[int(rng.integers(0, len(bad)))] ^= 1
        assert E.crc16_reg(bad) != 0x1D0F


def test_scrambler_recurrence_vs_oracle():
    rng = np.random.default_rng(3)
    for mcc, mnc, cc in [(0, 0, 0), (262, 1, 5), (1023, 16383, 63)] + \
            [tuple(int(v) for v in rng.integers(0, [1024, 16384, 64])) for _ in range(20)]:
        init = E.scramble_init(mcc, mnc, cc)
        assert init == ((((mcc << 20) | (mnc << 6) | cc) << 2) | 3)
        assert np.array_equal(E.scramble_seq(init, 432), S.scrambling_sequence(mcc, mnc, cc, 432)), (mcc, mnc, cc)
    # BSCH: colour code 0 (init 3)
    assert np.array_equal(E.scramble_seq(3, 120), S.scrambling_sequence(0, 0, 0, 120))


def test_index_formulas():
    # puncturing: the first type-3 bits take mother bits 1, 2, 5, 9, 10, 13, ... (P = (1, 2, 5), t = 3)
    assert [S.puncture_index(j) for j in range(1, 10)] == [1, 2, 5, 9, 10, 13, 17, 18, 21]
    for kind, p in S.KINDS.items():
        K, a = p["K"], p["a"]
        assert np.gcd(a, K) == 1                            # the interleaver is a permutation
        assert sorted((a * i) % K for i in range(1, K + 1)) == list(range(K))
        # rate 2/3 of the tail-terminated mother code: K type-3 bits from (n1 + 20) * 4 mother bits
        assert K == 3 * (p["n1"] + 20) // 2 == (p["n1"] + 20) * 4 * 3 // 8


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_encoder_vs_oracle(kind):
    """Type-1 -> type-5 (CRC, tail, mother code, puncturing, interleaving, scrambling): the oracle's
    encoder equals the independent restatement for random blocks and cells."""
    rng = np.random.default_rng(10 + kind)
    n1, K = S.KINDS[kind]["n1"], S.KINDS[kind]["K"]
    for _ in range(40):
        t1 = rng.integers(0, 2, n1).astype(np.uint8)
        init = (int(rng.integers(0, 2 ** 30)) << 2) | 3
        want = S.encode(t1, kind, init)
        got = E.encode_block(t1, kind, E.scramble_seq(init, K))
        assert np.array_equal(got, want)


def test_training_sequences_vs_spec_and_reference():
    """q / n / p / y / f of the oracle's bursts == the spec strings; n and p are the reference's own
    TS1 / TS2 (/root/reference/tetraear/core/decoder.py:196-199, recorded in tests/golden/_signals.py)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import _signals
    assert np.array_equal(E.N_BITS, S.bits_of(S.SEQ_N)) and np.array_equal(E.P_BITS, S.bits_of(S.SEQ_P))
    assert np.array_equal(E.Q_BITS, S.bits_of(S.SEQ_Q)) and np.array_equal(E.Y_BITS, S.bits_of(S.SEQ_Y))
    assert np.array_equal(E.F_BITS, S.bits_of(S.SEQ_F))
    assert np.array_equal(_signals.TS_N, S.bits_of(S.SEQ_N)) and np.array_equal(_signals.TS_P, S.bits_of(S.SEQ_P))


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_viterbi_maximum_likelihood(kind):
    """On noisy blocks the oracle's decoded path (type-2 bits, CRC and tail included) correlates
    with the received soft bits at least as well as the transmitted codeword: the decoder returns a
    maximum-likelihood codeword, scored by the independent encoder."""
    rng = np.random.default_rng(20 + kind)
    n1, K, a = S.KINDS[kind]["n1"], S.KINDS[kind]["K"], S.KINDS[kind]["a"]
    n2 = n1 + 20
    worse = 0
    for trial in range(30):
        t1 = rng.integers(0, 2, n1).astype(np.uint8)
        init = (int(rng.integers(0, 2 ** 30)) << 2) | 3
        c5 = S.encode(t1, kind, init)
        sigma = 40.0 if trial % 3 else 70.0                  # moderate and heavy noise
        soft = np.clip(np.rint(np.where(c5 == 0, 32.0, -32.0) + rng.normal(0, sigma, K)), -127, 127).astype(np.int8)
        # descramble + deinterleave + depuncture exactly as the spec orders them, then the oracle's trellis
        scr = S.scrambling_sequence_init(init, K)
        ms = np.zeros(4 * n2, np.int8)
        for i in range(1, K + 1):
            k = 1 + (a * i) % K
            v = int(soft[k - 1])
            ms[S.puncture_index(i) - 1] = -v if scr[k - 1] else v
        path = np.zeros(n2, np.uint8)
        E.lib().eo_viterbi(ms, n2, path)
        assert np.array_equal(path[-4:], np.zeros(4, np.uint8))            # tail-terminated
        m_dec = S.codeword_metric(soft, path, kind, init)
        m_tx = S.codeword_metric(soft, S.type2(t1), kind, init)
        assert m_dec >= m_tx, (trial, m_dec, m_tx)
        worse += m_dec > m_tx
    assert worse > 0   # the heavy-noise blocks do decode to other (more likely) codewords
