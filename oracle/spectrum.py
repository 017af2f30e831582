"""CPU oracle for the waterfall spectrum (TEST INFRASTRUCTURE -- only tests/, smoke() and
bench.py's cpu_baseline leg use it; the product path never does).

Definition (SURVEY.md §8d config C3 "2048-pt Hann waterfall"; the display it feeds is the
reference's live spectrum, /root/reference/tetraear/ui/modern.py:1928-1941, which computes one such
frame per chunk with these numpy calls in float64):

    P_f[k] = 20 log10( |fftshift(fft(x[f hop : f hop + nfft] * hanning(nfft)))[k]| / nfft + 1e-20 )

Parity is a tolerance (the GPU computes in fp32), written in tests/test_spectrum.py.  Pinned by
known answers, not by reference fixtures: the Hann window's coherent gain (a complex tone of
amplitude A exactly on bin k reads 20 log10(A (nfft - 1) / (2 nfft)) at shifted index k + nfft/2),
its first sidelobe pattern (the two neighbouring bins read A (nfft - 1) / (4 nfft)), and a direct
O(n^2) DFT of the windowed frame (tests/test_spectrum.py).
"""
import numpy as np

N_FFT = 2048


def frame_power(x, nfft=N_FFT):
    """One spectrum frame of x[:nfft] in dBFS, fftshifted (float64)."""
    x = np.asarray(x)[:nfft].astype(np.complex128)
    X = np.fft.fftshift(np.fft.fft(x * np.hanning(nfft)))
    return 20 * np.log10(np.abs(X) / nfft + 1e-20)


def frame_magnitude(x, nfft=N_FFT):
    """|X| / nfft of the same frame (the linear quantity the tolerance is written on)."""
    x = np.asarray(x)[:nfft].astype(np.complex128)
    return np.abs(np.fft.fftshift(np.fft.fft(x * np.hanning(nfft)))) / nfft


def waterfall(iq, hop=N_FFT, nframes=None, nfft=N_FFT, magnitude=False):
    """iq [C][N] (or [N]) -> [C][nframes][nfft] (or [nframes][nfft]) float64."""
    a = np.asarray(iq)
    one = a.ndim == 1
    a = a[None] if one else a
    N = a.shape[1]
    if nframes is None:
        nframes = (N - nfft) // hop + 1
    f = frame_magnitude if magnitude else frame_power
    out = np.stack([np.stack([f(a[c, i * hop:i * hop + nfft], nfft) for i in range(nframes)])
                    for c in range(a.shape[0])])
    return out[0] if one else out


def dft_power(x, nfft=N_FFT):
    """Direct float64 DFT of the windowed frame (pins frame_power's FFT call)."""
    n = np.arange(nfft)
    xw = np.asarray(x)[:nfft].astype(np.complex128) * np.hanning(nfft)
    X = np.exp(-2j * np.pi * np.outer(n, n) / nfft) @ xw
    return 20 * np.log10(np.abs(np.fft.fftshift(X)) / nfft + 1e-20)


# ------------------------------------------------------------------ signal-present / AFC gate
# the capture loop's gate in front of process() (/root/reference/tetraear/ui/
# modern.py:1952-2028), as that survey row describes it -- centre-band mean / max / argmax of the
# frame's dB row, the peak's frequency offset, the out-of-band noise mean, and the decision
# snr > 15 and peak > -70 and peak_above_avg > 3.  Restated from that description in float64 on
# frame_power; pinned by analytic known answers in tests/test_spectrum.py (tone on bin k -> offset
# k fs / 2048; each threshold flipped on its own), not by reference fixtures (parity unpinned: the
# round-1 refusal to record the reference's gate).

GATE_FIELDS = ("valid", "signal", "peak", "peak_bin", "peak_freq", "noise", "snr", "above", "present", "afc")


def gate_bins(fs, nfft=N_FFT, bandwidth=25000.0):
    """(start, end, noise_end, noise_start2) of the centre band and the two noise bands."""
    per_bin = fs / nfft
    nb = int(bandwidth / per_bin)
    centre = nfft // 2
    start, end = max(0, centre - nb // 2), min(nfft, centre + nb // 2)
    return start, end, max(0, start - 10), min(nfft, end + 10)


def gate(power, fs, nfft=N_FFT):
    """Gate decision on one fftshifted dB row: dict over GATE_FIELDS."""
    p = np.asarray(power, np.float64)
    start, end, n1, n2 = gate_bins(fs, nfft)
    out = dict.fromkeys(GATE_FIELDS, 0.0)
    if end <= start:
        return out
    band = p[start:end]
    sig, peak = float(np.mean(band)), float(np.max(band))
    k = start + int(np.argmax(band))
    freqs = np.fft.fftshift(np.fft.fftfreq(nfft, 1 / fs))
    noise_bins = np.concatenate([p[0:n1], p[n2:nfft]])
    noise = float(np.mean(noise_bins)) if len(noise_bins) else -100.0
    snr, above = sig - noise, peak - sig
    present = snr > 15 and peak > -70 and above > 3
    out.update(valid=1.0, signal=sig, peak=peak, peak_bin=float(k), peak_freq=float(freqs[k]), noise=noise, snr=snr,
               above=above, present=float(present), afc=float(freqs[k]) if present and peak > -70 else 0.0)
    return out


def gate_iq(x, fs, nfft=N_FFT):
    """The gate of a chunk: on the spectrum of its first nfft samples (no detection when shorter)."""
    x = np.asarray(x)
    if len(x) < nfft:
        return dict.fromkeys(GATE_FIELDS, 0.0)
    return gate(frame_power(x, nfft), fs, nfft)
