"""tetraear (MI355X build): the demod + lower-MAC hot path of TetraEar-BladeRF on gfx950.

The package keeps the reference's ``tetraear.signal`` / ``tetraear.core`` module surface for the
hot path; numeric work runs in libtetra_hip.so (see include/tetra_hip.h).  With the reference's
package root on sys.path after this one (or in $TETRAEAR_REFERENCE_ROOT) the reference's other
modules resolve through this package too (tetraear/_overlay.py, INTEGRATION.md option A).
Lazy top-level names as /root/reference/tetraear/__init__.py:24-36 exports them.
"""
from tetraear import _overlay

__path__ = _overlay.extend(__path__, __name__)
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("TetraDecoder", "TEADecryptor", "TetraKeyManager", "TetraProtocolParser"):
        import tetraear.core as core
        return getattr(core, name)
    if name in ("SignalProcessor", "BladeRFCapture", "TetraSignalDetector"):
        import tetraear.signal as sig
        return getattr(sig, name)
    if name == "VoiceProcessor":
        from tetraear.audio import VoiceProcessor   # the reference's (overlay)
        return VoiceProcessor
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = ["TetraDecoder", "TEADecryptor", "TetraKeyManager", "TetraProtocolParser", "SignalProcessor",
           "BladeRFCapture", "TetraSignalDetector", "VoiceProcessor"]
