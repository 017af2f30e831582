"""Second, independent restatement of the ETSI EN 300 392-2 channel coding (TEST INFRASTRUCTURE).

Written directly from the formulas of SURVEY.md Appendix B (EN 300 392-2 §8.2.3-§8.2.5), in plain
numpy / Python, sharing no code and no formulation with oracle/etsi_oracle.c:

  * CRC (§8.2.3.1): polynomial arithmetic over GF(2) -- F(x) is the ones' complement of the
    remainder of x^16 M(x) + x^K (x^15 + ... + 1) divided by G(x) = x^16 + x^12 + x^5 + 1 (the oracle
    runs a shift register);
  * tail: four zero bits;
  * mother code (§8.2.3.1.1): polynomial products of the type-2 sequence with
    G1 = 1 + D + D^4, G2 = 1 + D^2 + D^3 + D^4, G3 = 1 + D + D^2 + D^4, G4 = 1 + D + D^3 + D^4,
    interleaved V(4(k-1) + i) = (u * Gi)(k) (the oracle XORs register taps);
  * rate-2/3 puncturing (§8.2.3.1.2): t = 3, P = (1, 2, 5), type-3 bit j = V(k) with
    k = 8 floor((j-1)/t) + P(j - t floor((j-1)/t));
  * block interleaving (§8.2.4.1): type-4 bit k = type-3 bit i with k = 1 + (a i mod K);
  * scrambling (§8.2.5): p(k) = sum_i c_i p(k - i) over the taps of
    c(x) = 1 + x + x^2 + x^4 + x^5 + x^7 + x^8 + x^10 + x^11 + x^12 + x^16 + x^22 + x^23 + x^26 + x^32,
    initialised p(-31) = p(-30) = 1, p(-(i-1)) = e(i) for the 30 bits e(1..30) of the extended colour
    code MCC(10) MNC(14) CC(6), MSB first (the oracle shifts a 32-bit register).

tests/test_etsi_spec.py checks the oracle (and through it the GPU, which is bit-identical to the
oracle) against this module, and uses it for the Viterbi maximum-likelihood property.  It is not a
reference pin -- the reference has no channel coding -- but a wrong constant or
index formula now has to be wrong twice, in two unrelated formulations, to go unnoticed.
"""
import numpy as np

G_CRC = [16, 12, 5, 0]                                  # exponents of G(x)
GENERATORS = ([1, 1, 0, 0, 1], [1, 0, 1, 1, 1], [1, 1, 1, 0, 1], [1, 1, 0, 1, 1])   # G1..G4, D^0..D^4
PUNCT_P = (None, 1, 2, 5)                               # P(1), P(2), P(3); t = 3
KINDS = {0: dict(n1=268, K=432, a=103), 1: dict(n1=124, K=216, a=101), 2: dict(n1=60, K=120, a=11)}
SCRAMBLER_TAPS = (1, 2, 4, 5, 7, 8, 10, 11, 12, 16, 22, 23, 26, 32)   # c_i = 1

# EN 300 392-2 §9.4.4.3 sequences, typed from the spec's tables
SEQ_N = "1101000011101001110100"           # normal training sequence n (9.4.4.3.2)
SEQ_P = "0111101001000011011100"           # normal training sequence p
SEQ_Q = "1011011100000110101101"           # extended training sequence q (9.4.4.3.3)
SEQ_Y = "11000001100111001110100111000001100111"   # synchronisation training sequence y (9.4.4.3.4)
SEQ_F = "1" * 8 + "0" * 64 + "1" * 8      # frequency correction field f (9.4.4.3.1)


def bits_of(s):
    return np.array([int(c) for c in s], np.uint8)


def poly_mod(num, den_exps):
    """Remainder of a GF(2) polynomial (coefficient array, index = exponent) by a divisor given as
    exponents."""
    r = np.array(num, np.uint8) % 2
    top = max(den_exps)
    for e in range(len(r) - 1, top - 1, -1):
        if r[e]:
            for d in den_exps:
                r[e - top + d] ^= 1
    return r[:top]


def crc_bits(m):
    """The 16 CRC bits appended to K1 type-1 bits m (transmitted first = highest power)."""
    m = np.asarray(m, np.uint8) & 1
    k = len(m)
    # M(x): m[0] is the coefficient of x^(k-1)
    a = np.zeros(k + 16, np.uint8)
    for i, v in enumerate(m):
        a[k - 1 - i + 16] = v                          # x^16 M(x)
    b = np.zeros(k + 16, np.uint8)
    b[k:k + 16] = 1                                    # x^k (x^15 + ... + 1)
    rem = poly_mod(a ^ b, G_CRC)
    f = 1 - rem                                        # ones' complement
    return np.array([f[15 - i] for i in range(16)], np.uint8)   # highest power first


def crc16_value(m):
    v = 0
    for b in crc_bits(m):
        v = (v << 1) | int(b)
    return v


def type2(type1):
    """type-1 bits + CRC + four tail bits."""
    t1 = np.asarray(type1, np.uint8) & 1
    return np.concatenate([t1, crc_bits(t1), np.zeros(4, np.uint8)])


def mother(u):
    """V(4(k-1) + i) for k = 1..len(u), i = 1..4: (u * Gi) mod 2, truncated to len(u) steps."""
    u = np.asarray(u, np.int64)
    out = np.zeros(4 * len(u), np.uint8)
    for i, g in enumerate(GENERATORS):
        c = np.convolve(u, np.array(g, np.int64))[:len(u)] % 2
        out[i::4] = c
    return out


def puncture_index(j):
    """Mother index k (1-based) of type-3 bit j (1-based), rate 2/3."""
    t = 3
    q = (j - 1) // t
    return 8 * q + PUNCT_P[j - t * q]


def type3(type1, kind):
    p = KINDS[kind]
    v = mother(type2(type1))
    return np.array([v[puncture_index(j) - 1] for j in range(1, p["K"] + 1)], np.uint8)


def interleave(b3, kind):
    p = KINDS[kind]
    K, a = p["K"], p["a"]
    b4 = np.zeros(K, np.uint8)
    for i in range(1, K + 1):
        b4[(a * i) % K] = b3[i - 1]                    # k = 1 + (a i mod K), 1-based
    return b4


def scrambling_sequence(mcc, mnc, cc, n):
    """p(1..n) by the recurrence, from the extended colour code e(1..30) = MCC MNC CC, MSB first."""
    e = [int(c) for c in format(mcc & 0x3FF, "010b") + format(mnc & 0x3FFF, "014b") + format(cc & 0x3F, "06b")]
    p = {-31: 1, -30: 1}
    for i in range(1, 31):
        p[-(i - 1)] = e[i - 1]
    for k in range(1, n + 1):
        p[k] = sum(p[k - i] for i in SCRAMBLER_TAPS) % 2
    return np.array([p[k] for k in range(1, n + 1)], np.uint8)


def scrambling_sequence_init(init, n):
    """The same from a scrambling init as the ABI passes it: ((MCC<<20 | MNC<<6 | CC) << 2) | 3."""
    ecc = (int(init) >> 2) & 0x3FFFFFFF
    return scrambling_sequence(ecc >> 20, (ecc >> 6) & 0x3FFF, ecc & 0x3F, n)


def encode(type1, kind, init):
    """type-1 -> type-5 bits of one block: CRC, tail, mother code, puncture, interleave, scramble."""
    b4 = interleave(type3(type1, kind), kind)
    return b4 ^ scrambling_sequence_init(init, KINDS[kind]["K"])


def codeword_metric(soft5, type2_bits, kind, init):
    """Correlation of a type-5 soft block (int8, > 0 = bit 0) with the codeword of a type-2
    sequence: sum soft * (1 - 2 c).  The maximum-likelihood path maximises it over all tail-
    terminated type-2 sequences."""
    p = KINDS[kind]
    v = mother(type2_bits)
    b3 = np.array([v[puncture_index(j) - 1] for j in range(1, p["K"] + 1)], np.uint8)
    c5 = interleave(b3, kind) ^ scrambling_sequence_init(init, p["K"])
    return int(np.sum(np.asarray(soft5, np.int64) * (1 - 2 * c5.astype(np.int64))))
