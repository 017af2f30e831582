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
