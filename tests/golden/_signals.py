"""Seeded synthetic IQ families used to build golden fixtures (TEST INFRASTRUCTURE).

Families: complex noise, a TETRA-like pi/4-DQPSK burst stream with RRC
alpha=0.35 pulses at 18 ksym/s sampled at ``fs`` (ETSI EN 300 392-2 Table 5.1 dibit mapping,
normal downlink bursts carrying training sequence n/p at bit 244), a DC tone plus noise (the
shape of the reference's own ``sample_iq_samples`` fixture, /root/reference/tests/conftest.py:53-67)
and a high-noise stress variant.  Returned as complex64 rounded to the SC16 grid
(round(x*32768)/32768, as /root/reference/tetraear/signal/capture.py:259-269 produces), so a
fixture can store the exact input as int16 pairs.
"""
import numpy as np

TS_N = np.array([1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0], np.uint8)
TS_P = np.array([0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0], np.uint8)
# dibit (b1 b2) -> phase step, ETSI Table 5.1
_STEP = {(0, 0): np.pi / 4, (0, 1): 3 * np.pi / 4, (1, 1): -3 * np.pi / 4, (1, 0): -np.pi / 4}


def rrc_taps(alpha, sps, span):
    t = (np.arange(-span * sps / 2, span * sps / 2 + 1e-9) / sps).astype(np.float64)
    return rrc(t, alpha)


def rrc(t, alpha):
    """Root-raised-cosine impulse response at time t (in symbol periods), unit symbol period."""
    t = np.asarray(t, np.float64)
    out = np.empty_like(t)
    eps = 1e-9
    z = np.abs(t) < eps
    out[z] = 1.0 - alpha + 4 * alpha / np.pi
    s = np.abs(np.abs(4 * alpha * t) - 1.0) < eps
    out[s] = (alpha / np.sqrt(2)) * ((1 + 2 / np.pi) * np.sin(np.pi / (4 * alpha))
                                     + (1 - 2 / np.pi) * np.cos(np.pi / (4 * alpha)))
    o = ~(z | s)
    tt = t[o]
    num = np.sin(np.pi * tt * (1 - alpha)) + 4 * alpha * tt * np.cos(np.pi * tt * (1 + alpha))
    den = np.pi * tt * (1 - (4 * alpha * tt) ** 2)
    out[o] = num / den
    return out


def burst_bits(rng, two_log_chan=False):
    """One 510-bit normal continuous downlink burst (layout EN 300 392-2 §9.4.4.2.5)."""
    b = rng.integers(0, 2, 510).astype(np.uint8)
    b[244:266] = TS_P if two_log_chan else TS_N
    return b


def bits_to_phase_steps(bits):
    d = bits.reshape(-1, 2)
    steps = np.where(d[:, 0] == 0, np.where(d[:, 1] == 0, np.pi / 4, 3 * np.pi / 4),
                     np.where(d[:, 1] == 0, -np.pi / 4, -3 * np.pi / 4))
    return steps


def tetra_iq(rng, n, fs, cfo=0.0, snr_db=None, alpha=0.35, span=8, amp=0.5):
    """pi/4-DQPSK burst stream sampled at fs (fractional samples/symbol allowed)."""
    sym_rate = 18000.0
    nsym = int(np.ceil(n / fs * sym_rate)) + span + 4
    nburst = nsym // 255 + 1
    bits = np.concatenate([burst_bits(rng, k % 2 == 1) for k in range(nburst)])[: 2 * nsym]
    ph = np.cumsum(bits_to_phase_steps(bits)) + rng.uniform(0, 2 * np.pi)
    sym = np.exp(1j * ph)
    t = np.arange(n) / fs * sym_rate + span / 2  # in symbol periods
    k0 = np.floor(t).astype(np.int64)
    x = np.zeros(n, np.complex128)
    for d in range(-span // 2, span // 2 + 1):
        k = k0 + d
        x += sym[k] * rrc(t - k, alpha)
    x *= amp / np.sqrt(np.mean(np.abs(x) ** 2))
    if cfo:
        x *= np.exp(2j * np.pi * cfo * np.arange(n) / fs)
    if snr_db is not None:
        p = np.mean(np.abs(x) ** 2)
        sigma = np.sqrt(p / (10 ** (snr_db / 10)) / 2)
        x += sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x, bits


def sc16_round(x):
    """Quantise to the SC16 grid; returns (complex64 samples, int16 [n,2])."""
    iq = np.stack([np.round(x.real * 32768), np.round(x.imag * 32768)], axis=-1)
    iq = np.clip(iq, -32768, 32767).astype(np.int16)
    return (iq[:, 0].astype(np.float32) / 32768 + 1j * (iq[:, 1].astype(np.float32) / 32768)).astype(
        np.complex64), iq


def family(name, rng, n, fs):
    if name == "noise":
        x = 0.25 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    elif name == "tetra":
        x, _ = tetra_iq(rng, n, fs, cfo=rng.uniform(-600, 600), snr_db=30)
    elif name == "tetra_clean":
        x, _ = tetra_iq(rng, n, fs)
    elif name == "tone":
        x = np.exp(1j * 2 * np.pi * 0 * np.arange(n) / fs) * 0.5 \
            + 0.05 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    elif name == "stress":
        x, _ = tetra_iq(rng, n, fs, cfo=rng.uniform(-600, 600), snr_db=6)
    else:
        raise ValueError(name)
    return sc16_round(x)


# ---------------------------------------------------------------- g5_scanner.npz input encodings
# A scanner case's input is stored as one of (so the fixture stays small and decodes exactly):
#   c_<i>  complex64 samples;
#   q_<i>  int16 [n, 2] on the SC16 grid (x = q / 32768 in float32, as sc16_round);
#   k_<i>  uint8 constellation indices with p_<i> complex64 [4] points and r_<i> = (repeat, offset):
#          x = repeat(p[k], repeat)[offset:] (a phase-step walk held for `repeat` samples per symbol).
def scanner_input(z, i):
    if f"c_{i}" in z.files:
        return z[f"c_{i}"]
    if f"q_{i}" in z.files:
        q = z[f"q_{i}"]
        return (q[:, 0].astype(np.float32) / 32768 + 1j * (q[:, 1].astype(np.float32) / 32768)).astype(np.complex64)
    rep, off = (int(v) for v in z[f"r_{i}"])
    return np.repeat(z[f"p_{i}"][z[f"k_{i}"]], rep)[off:]


# ---------------------------------------------------------------- compat form sweep
SWEEP_FAMILIES = ("tetra", "tetra_clean", "noise", "tone", "stress")
SWEEP_AFC = 2.4e6 / 2048   # the AFC bin of /root/reference/tetraear/ui/modern.py:1956-1974


def sweep_chunks(seed, n_chunks=40, n=131072, fs=2.4e6):
    """The GUI's call pattern (modern.py:1919,2029: one 131072-sample chunk per process() call, an AFC
    offset of k bins, |k| <= 10) as a seeded stream: default_rng(777000 + seed) draws, per chunk, a
    family, an offset and the family's samples, in that order.  Yields (chunk, family, offset,
    complex64 samples, int16 [n, 2] SC16 image)."""
    rng = np.random.default_rng(777000 + seed)
    for k in range(n_chunks):
        fam = SWEEP_FAMILIES[int(rng.integers(0, len(SWEEP_FAMILIES)))]
        fo = SWEEP_AFC * int(rng.integers(-10, 11))
        x, iq = family(fam, rng, n, fs)
        yield k, fam, fo, x, iq


def sweep_chunk(seed, chunk, n=131072, fs=2.4e6):
    """One chunk of sweep_chunks (the stream is regenerated up to it)."""
    for k, fam, fo, x, iq in sweep_chunks(seed, chunk + 1, n, fs):
        if k == chunk:
            return fam, fo, x, iq
