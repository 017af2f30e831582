"""Signal processing (demodulation).  Mirrors /root/reference/tetraear/signal/__init__.py:11-28.

SignalProcessor and the scanner's signal detector (TetraSignalDetector) are this build's, on the
GPU.  BladeRF capture (``capture``) and the frequency sweep (FrequencyScanner) are the reference's:
they resolve when the reference's package root is on sys.path after this one (tetraear/_overlay.py)
and raise ImportError naming the missing reference otherwise.
"""
from tetraear import _overlay

__path__ = _overlay.extend(__path__, __name__)


def __getattr__(name):
    if name == "SignalProcessor":
        from tetraear.signal.processor import SignalProcessor
        return SignalProcessor
    if name == "TetraSignalDetector":
        from tetraear.signal.scanner import TetraSignalDetector
        return TetraSignalDetector
    if name == "FrequencyScanner":
        from tetraear.signal.scanner import FrequencyScanner
        return FrequencyScanner
    if name in ("BladeRFCapture", "list_bladerf_devices"):
        if not _overlay.active():
            raise _overlay.ReferenceUnavailable(
                f"{name} is the reference's (tetraear/signal/capture.py): put the reference's package root on "
                f"sys.path after this build's, or set TETRAEAR_REFERENCE_ROOT")
        from tetraear.signal import capture
        return getattr(capture, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = ["SignalProcessor", "BladeRFCapture", "list_bladerf_devices", "TetraSignalDetector", "FrequencyScanner"]
