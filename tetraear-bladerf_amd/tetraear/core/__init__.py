"""Core decoding (lower MAC).  Mirrors /root/reference/tetraear/core/__init__.py:11-34 for the
hot-path names; the TEA crypto classes stay in the reference (out of scope)."""
from tetraear.core.protocol import (
    TetraProtocolParser,
    TetraBurst,
    MacPDU,
    CallMetadata,
    BurstType,
    ChannelType,
    PDUType,
)
from tetraear.core.decoder import TetraDecoder

__all__ = [
    "TetraDecoder",
    "TetraProtocolParser",
    "TetraBurst",
    "MacPDU",
    "CallMetadata",
    "BurstType",
    "ChannelType",
    "PDUType",
]
