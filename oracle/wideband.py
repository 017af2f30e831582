"""CPU oracle for the wideband channeliser (TEST INFRASTRUCTURE -- only tests/, smoke() and
bench.py's cpu_baseline leg use it; the product path never does).

The reference has no channeliser (it tunes the SDR to one carrier per capture,
/root/reference/tetraear/ui/modern.py:1886-1887), so this float64 numpy restatement IS the
specification of tetraear-bladerf_amd/csrc/wideband.hip:

  analysis  u_j[r] = sum_p h[pM + r] x[n_j - pM - r],  n_j = L - 1 + jD   (L = MP, D = M/2 or M/4)
            Y_j[k] = sum_r u_j[r] exp(+2 pi i k r / M)
            v_k[j] = exp(-2 pi i k j D / M) Y_j[k] = (-i)^(k j 4D/M mod 4) Y_j[k]
  resample  y_k[n] = sum_{q<Q} g[(down n mod up) + up q] v_k[floor(down n / up) + Q - 1 - q]
  synthesis x[n]   = sum_j D h[n - jD] W_j[n mod M],  W_j[r] = sum_k s_k[j] exp(+2 pi i k r / M)

Parity: the GPU runs in fp32 with a rocFFT transform, so y is compared within a tolerance; the
timing stage downstream of y is bit-exact against oracle/etsi.py on the GPU's own y.
"""
import os

import numpy as np
from scipy import signal as _design

from etsi import rrc

FS_WB, M_WB = 20e6, 800
# the filter bank's two designs (tetraear.signal.wideband.DESIGNS restates them for the product):
#   oversample 2 -- D = M / 2, 50 kHz carriers, P = 5 branches (cut-off 25 kHz, Kaiser 8), resampler
#                   36 / 25 with 828 taps; the default
#   oversample 4 -- D = M / 4, 100 kHz carriers, P = 2 (cut-off 50 kHz, Kaiser 7), 18 / 25, 810 taps
OVERSAMPLE = {2: (5, 25e3, 8.0, 36, 25, 828), 4: (2, 50e3, 7.0, 18, 25, 810)}
DEFAULT_OVERSAMPLE = int(os.environ.get("TETRA_WB_OVERSAMPLE", "2"))


def design(fs=FS_WB, M=M_WB, oversample=None):
    ov = DEFAULT_OVERSAMPLE if oversample is None else oversample
    P, cut, beta, up, down, Lg = OVERSAMPLE[ov]
    D = M // ov
    h = _design.firwin(M * P, cut, fs=fs, window=("kaiser", beta)).astype(np.float32)
    sps = fs / D * up / 18000.0
    g = rrc((np.arange(Lg) - (Lg - 1) / 2.0) / sps).astype(np.float32)
    return dict(M=M, D=D, P=P, up=up, down=down, Lg=Lg, fs=fs, h=h, g=g)


def lengths(d, Nw):
    L = d["M"] * d["P"]
    Q = d["Lg"] // d["up"]
    nblk = (Nw - L) // d["D"] + 1 if Nw >= L else 0
    n72 = (d["up"] * (nblk - Q) + d["up"] - 1) // d["down"] + 1 if nblk >= Q else 0
    return nblk, n72


def analysis(x, d):
    """v [M][nblk] complex128: the filter-bank outputs at fs / D."""
    M, D, P = d["M"], d["D"], d["P"]
    h = d["h"].astype(np.float64)
    x = np.asarray(x, np.complex128)
    nblk, _ = lengths(d, len(x))
    L = M * P
    r = np.arange(M)
    u = np.zeros((nblk, M), np.complex128)
    nj = L - 1 + D * np.arange(nblk)
    for p in range(P):
        u += h[p * M + r][None, :] * x[nj[:, None] - p * M - r[None, :]]
    Y = np.fft.ifft(u, axis=1) * M
    k = np.arange(M)
    q = (k[:, None] * (np.arange(nblk) * (4 * D // M))[None, :]) % 4   # e^{-2 pi i k j D / M}
    return (-1j) ** q * Y.T


def resample(v, d, n_keep=None):
    up, down, g = d["up"], d["down"], d["g"].astype(np.float64)
    Q = d["Lg"] // up
    nblk = v.shape[1]
    n72 = (up * (nblk - Q) + up - 1) // down + 1 if nblk >= Q else 0
    n = np.arange(n72 if n_keep is None else n_keep)
    rho = (down * n) % up
    top = (down * n) // up + Q - 1
    qq = np.arange(Q)
    taps = g[rho[:, None] + up * qq[None, :]]          # [n][Q]
    idx = top[:, None] - qq[None, :]                    # [n][Q]
    out = np.empty((v.shape[0], len(n)), np.complex128)
    for k0 in range(0, v.shape[0], 32):
        vv = v[k0:k0 + 32][:, idx]                      # [k][n][Q]
        out[k0:k0 + 32] = np.einsum("nq,knq->kn", taps, vv)
    return out


def channelize(x, d, n_keep=None):
    return resample(analysis(x, d), d, n_keep)


def synthesize(s, d, Nw):
    """s [M][nbb] carrier baseband at fs / D -> x [Nw] (noiseless)."""
    M, D, P = d["M"], d["D"], d["P"]
    h = d["h"].astype(np.float64)
    nbb = s.shape[1]
    W = np.fft.ifft(np.asarray(s, np.complex128), axis=0) * M     # [r][j]
    n = np.arange(Nw)
    x = np.zeros(Nw, np.complex128)
    L = M * P
    for j in range(nbb):
        lo, hi = j * D, min(Nw, j * D + L)
        if lo >= Nw:
            break
        nn = n[lo:hi]
        x[lo:hi] += D * h[nn - j * D] * W[nn % M, j]
    return x
