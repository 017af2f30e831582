"""SignalProcessor.resample (/root/reference/tetraear/signal/processor.py:35-49) on the GPU against
scipy.signal.resample -- the reference's own call, so scipy is the oracle here (scipy 1.15.3,
complex path: fft, spectrum truncation / zero padding with the Nyquist split and join, ifft).

Tolerance: max |GPU - scipy| <= TOL x max |scipy| per call, TOL = 2e-6 for complex64 (both sides
compute in single precision, with different FFT factorisations) and 1e-12 for complex128.  Real
input runs the complex transform and keeps the real part (scipy's rfft path, up to rounding).
"""
import numpy as np
import pytest
from scipy import signal

TOL32, TOL64 = 2e-6, 1e-12

# (Nx, num) pairs: down/up, even/odd N = min(Nx, num), the N = 2 edge, the reference's own test
# (1000 samples 2.4 MSps -> 1.2 MSps), a GUI-sized chunk, prime lengths (Bluestein in rocFFT)
CASES = [(1000, 500), (1000, 1500), (1001, 500), (1000, 501), (999, 1998), (64, 2), (2, 64), (3, 7), (7, 3),
         (131072, 13107), (4099, 1031), (1031, 4099)]


def _x(n, dtype, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("Nx,num", CASES)
@pytest.mark.parametrize("dtype", [np.complex64, np.complex128])
def test_resample_matches_scipy(Nx, num, dtype):
    from tetraear.signal import SignalProcessor
    fs = 2.4e6
    p = SignalProcessor(fs)
    x = _x(Nx, dtype, Nx * 7 + num)
    target = fs * num / Nx
    assert int(Nx * target / fs) in (num, num - 1)
    num = int(Nx * target / fs)
    got = p.resample(x, target)
    want = signal.resample(x, num)
    assert got.dtype == want.dtype and got.shape == want.shape
    tol = TOL32 if dtype == np.complex64 else TOL64
    assert np.abs(got - want).max() <= tol * np.abs(want).max()


@pytest.mark.gpu
def test_resample_real_input_and_reference_test_shape():
    """The reference's unit test (tests/unit/test_signal_processor.py:27-35): length scales with
    the rate ratio; real input gives scipy's real-path result."""
    from tetraear.signal import SignalProcessor
    p = SignalProcessor(2.4e6)
    x = _x(1000, np.complex64, 1)
    y = p.resample(x, 1.2e6)
    assert len(y) == 500
    r = np.random.default_rng(2).standard_normal(1000)
    for n_out, rate in ((500, 1.2e6), (1500, 3.6e6)):
        got = p.resample(r, rate)
        want = signal.resample(r, n_out)
        assert got.dtype == want.dtype and np.abs(got - want).max() <= 1e-12 * np.abs(want).max()
