"""Recorded-IQ files for the GPU receiver.

The reference has no recorded-IQ format: capture.py:241-269 reads the BladeRF's interleaved int16
(I, Q) buffer and scales it by 1/32768.  These files keep that wire format on disk (``.sc16``) or
the scaled complex64 samples (``.cf32``), one channel per file or several channels interleaved
sample by sample, and are read memory-mapped in chunks -- the SC16 chunks go to the device as they
are (4 B per sample) and are scaled inside the channel filter (``tetra_demod_etsi_fmt`` with
``TETRA_SC16``), bit-identical to the complex64 path.
"""
import os

import numpy as np

FORMATS = {"sc16": (np.int16, 2), "cf32": (np.complex64, 1)}


def fmt_of(path, fmt=None):
    if fmt is None:
        fmt = os.path.splitext(path)[1].lstrip(".").lower()
    if fmt not in FORMATS:
        raise ValueError(f"unknown IQ format {fmt!r} (expected one of {sorted(FORMATS)})")
    return fmt


def write_iq(path, samples, fmt=None):
    """Write [N] or [N, channels] samples.  For sc16, complex input is rounded to the int16 grid
    (x * 32768, clipped) and int16 [.., 2] input is written as is."""
    fmt = fmt_of(path, fmt)
    x = np.asarray(samples)
    if fmt == "sc16":
        if x.dtype != np.int16:
            x = np.stack([np.round(x.real * 32768), np.round(x.imag * 32768)], axis=-1)
            x = np.clip(x, -32768, 32767).astype(np.int16)
    else:
        x = x.astype(np.complex64)
    np.ascontiguousarray(x).tofile(path)


def open_iq(path, channels=1, fmt=None):
    """Memory-map a recording: [N, channels, 2] int16 (sc16) or [N, channels] complex64 (cf32)."""
    fmt = fmt_of(path, fmt)
    dtype, per = FORMATS[fmt]
    item = np.dtype(dtype).itemsize * per * channels
    n = os.path.getsize(path) // item
    shape = (n, channels, 2) if fmt == "sc16" else (n, channels)
    return np.memmap(path, dtype=dtype, mode="r", shape=shape), fmt


def chunks(path, chunk=128 * 1024, channels=1, fmt=None):
    """Yield channel-major chunks ready for EtsiReceiver.demod_batch: int16 [channels, chunk, 2]
    for sc16, complex64 [channels, chunk] for cf32 (the last partial chunk is dropped, as the
    capture loop reads fixed 128 Ki chunks, modern.py:1919)."""
    m, fmt = open_iq(path, channels, fmt)
    for s in range(0, m.shape[0] - chunk + 1, chunk):
        block = np.asarray(m[s:s + chunk])
        yield np.ascontiguousarray(np.moveaxis(block, 1, 0))


def to_complex64(x):
    """SC16 [.., 2] -> complex64 exactly as capture.py:259-269 scales (x / 32768)."""
    x = np.asarray(x)
    if x.dtype == np.int16:
        return (x[..., 0].astype(np.float32) / 32768 + 1j * (x[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    return x.astype(np.complex64)
