"""Signal processing (demodulation).  Mirrors /root/reference/tetraear/signal/__init__.py:11-28.

The scanner's signal detector (TetraSignalDetector) runs on the GPU (tetraear.signal.scanner).
BladeRF capture and the frequency sweep (FrequencyScanner) are hardware/UI components outside this
hot-path build; asking for them raises ImportError naming the reference module that provides them.
"""


def __getattr__(name):
    if name == "SignalProcessor":
        from tetraear.signal.processor import SignalProcessor
        return SignalProcessor
    if name == "TetraSignalDetector":
        from tetraear.signal.scanner import TetraSignalDetector
        return TetraSignalDetector
    if name in ("BladeRFCapture", "list_bladerf_devices", "FrequencyScanner"):
        raise ImportError(f"{name} is not part of the MI355X hot-path build; use the reference's "
                          f"tetraear.signal.{'capture' if 'BladeRF' in name or 'bladerf' in name else 'scanner'}")
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = ["SignalProcessor", "TetraSignalDetector"]
