"""Core decoding (lower MAC).  Mirrors /root/reference/tetraear/core/__init__.py:11-34: the
decoder, parser and protocol types are this build's; the TEA crypto classes (TEADecryptor,
TetraKeyManager) are the reference's, resolved through the overlay (tetraear/_overlay.py) when its
package root is on sys.path after this one."""
from tetraear import _overlay

__path__ = _overlay.extend(__path__, __name__)

from tetraear.core.protocol import (  # noqa: E402
    TetraProtocolParser,
    TetraBurst,
    MacPDU,
    CallMetadata,
    BurstType,
    ChannelType,
    PDUType,
)
from tetraear.core.decoder import TetraDecoder  # noqa: E402


def __getattr__(name):
    if name in ("TEADecryptor", "TetraKeyManager"):
        if not _overlay.active():
            raise _overlay.ReferenceUnavailable(
                f"{name} is the reference's (tetraear/core/crypto.py): put the reference's package root on "
                f"sys.path after this build's, or set TETRAEAR_REFERENCE_ROOT")
        from tetraear.core import crypto
        return getattr(crypto, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = [
    "TetraDecoder",
    "TEADecryptor",
    "TetraKeyManager",
    "TetraProtocolParser",
    "TetraBurst",
    "MacPDU",
    "CallMetadata",
    "BurstType",
    "ChannelType",
    "PDUType",
]
