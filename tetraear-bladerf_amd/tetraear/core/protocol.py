"""Burst-level protocol types and the lower-MAC half of TetraProtocolParser, on the GPU.

Mirrors the hot-path part of /root/reference/tetraear/core/protocol.py:
  enums and dataclasses (BurstType, ChannelType, PDUType, TetraBurst, MacPDU, CallMetadata)
                                                             protocol.py:34-139
  TetraProtocolParser.parse_burst and helpers, _check_crc, _calculate_crc16
                                                             protocol.py:142-347
Burst typing, slicing and the CRC run in libtetra_hip.so.  The upper-MAC parsers of the
reference (parse_mac_pdu, SDS, LIP, call metadata -- protocol.py:349-1300) are out of scope of
this hot-path build and stay the reference's Python; ``upper_mac`` hooks are where they attach
(INTEGRATION.md).
"""
import logging
from dataclasses import dataclass
from enum import Enum
from typing import Optional

import numpy as np

from tetraear import _hip

logger = logging.getLogger(__name__)


class BurstType(Enum):
    NormalUplink = 1
    NormalDownlink = 2
    ControlUplink = 3
    ControlDownlink = 4
    Synchronization = 5
    Linearization = 6


class ChannelType(Enum):
    TCH = "Traffic Channel"
    STCH = "Stealing Channel"
    SCH = "Signaling Channel"
    AACH = "Associated Control Channel"
    BSCH = "Broadcast Synchronization Channel"
    BNCH = "Broadcast Network Channel"


class PDUType(Enum):
    MAC_RESOURCE = 0
    MAC_FRAG = 1
    MAC_END = 2
    MAC_BROADCAST = 3
    MAC_SUPPL = 4
    MAC_U_SIGNAL = 5
    MAC_DATA = 6
    MAC_U_BLK = 7


@dataclass
class TetraBurst:
    """One 255-symbol burst (protocol.py:66-76)."""
    burst_type: BurstType
    slot_number: int
    frame_number: int
    training_sequence: np.ndarray
    data_bits: np.ndarray
    crc_ok: bool
    scrambling_code: int = 0
    colour_code: int = 0


@dataclass
class MacPDU:
    pdu_type: PDUType
    encrypted: bool
    address: Optional[int]
    length: int
    data: bytes
    fill_bits: int = 0
    encryption_mode: int = 0
    reassembled_data: Optional[bytes] = None


@dataclass
class CallMetadata:
    call_type: str
    talkgroup_id: Optional[int]
    source_ssi: Optional[int]
    dest_ssi: Optional[int]
    channel_allocated: Optional[int]
    call_identifier: Optional[int] = None
    call_priority: int = 0
    mcc: Optional[int] = None
    mnc: Optional[int] = None
    duplex_mode: str = "simplex"
    encryption_enabled: bool = False
    encryption_algorithm: Optional[str] = None


def _bits_u8(bits):
    b = np.asarray(bits)
    return np.ascontiguousarray(np.where((b == 0) | (b == 1), b, 2), dtype=np.uint8)


def burst_from_bits(bits510, btype_value, crc_ok, slot_number, frame_number, colour_code):
    """Assemble a TetraBurst from the device's burst bits (protocol.py:267-290 slices)."""
    bits = bits510.astype(np.int64)
    if btype_value == BurstType.Synchronization.value:
        ts, data = bits[108:130], bits
    else:
        ts, data = bits[108:122], np.concatenate([bits[0:108], bits[122:230]])
    return TetraBurst(burst_type=BurstType(btype_value), slot_number=slot_number, frame_number=frame_number,
                      training_sequence=ts, data_bits=data, crc_ok=bool(crc_ok), colour_code=colour_code)


class TetraProtocolParser:
    """PHY/lower-MAC burst parser (protocol.py:142)."""

    SYMBOLS_PER_SLOT = 255
    SLOTS_PER_FRAME = 4
    FRAMES_PER_MULTIFRAME = 18
    MULTIFRAMES_PER_HYPERFRAME = 60
    TRAINING_SEQUENCES = {
        1: [0, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 0, 1, 1],
        2: [0, 0, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 0, 1],
        3: [0, 0, 0, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 0],
    }
    SYNC_CONTINUOUS_DOWNLINK = [1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0]
    SYNC_DISCONTINUOUS_DOWNLINK = [0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 0, 0, 1, 1]

    def __init__(self):
        self.current_frame_number = 0
        self.current_multiframe = 0
        self.current_hyperframe = 0
        self.mcc = None
        self.mnc = None
        self.la = None
        self.colour_code = None
        self.stats = {
            'total_bursts': 0, 'crc_pass': 0, 'crc_fail': 0, 'clear_mode_frames': 0,
            'encrypted_frames': 0, 'decrypted_frames': 0, 'voice_calls': 0,
            'data_messages': 0, 'control_messages': 0,
        }
        self.fragment_buffer = bytearray()
        self.fragment_metadata = {}

    def count_burst(self, crc_ok):
        self.stats['total_bursts'] += 1
        self.stats['crc_pass' if crc_ok else 'crc_fail'] += 1

    def parse_burst(self, symbols, slot_number: int = 0) -> Optional[TetraBurst]:
        """Burst type, training sequence, data bits and CRC of one slot (protocol.py:192-244)."""
        if len(symbols) < self.SYMBOLS_PER_SLOT:
            logger.warning(f"Insufficient symbols for burst: {len(symbols)} < {self.SYMBOLS_PER_SLOT}")
            return None
        s = np.ascontiguousarray(np.asarray(symbols)[:self.SYMBOLS_PER_SLOT], dtype=np.int64)
        btype = np.zeros(1, np.int32)
        ok = np.zeros(1, np.uint8)
        bits = np.empty((1, 510), np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_parse_bursts(c.handle, _hip.ptr(s), 1, _hip.ptr(btype), _hip.ptr(ok), _hip.ptr(bits)),
                "tetra_parse_bursts")
        self.count_burst(bool(ok[0]))
        return burst_from_bits(bits[0], int(btype[0]), bool(ok[0]), slot_number, self.current_frame_number,
                               self.colour_code or 0)

    def _match(self, bits, pattern, offset=0):
        b = _bits_u8(bits)
        cnt = np.zeros(1, np.int32)
        pat = np.ascontiguousarray(pattern, dtype=np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_match_count(c.handle, _hip.ptr(b), 1, len(b), _hip.ptr(pat), offset, _hip.ptr(cnt)),
                "tetra_match_count")
        return int(cnt[0])

    def _detect_burst_type(self, bits) -> BurstType:
        sync_pos = len(bits) // 2
        if self._check_sync_pattern(np.asarray(bits)[sync_pos:sync_pos + 22]):
            return BurstType.Synchronization
        return BurstType.NormalDownlink

    def _check_sync_pattern(self, bits) -> bool:
        """max(match_cont, match_disc) / 22 > 0.8 (protocol.py:256-265)."""
        if len(bits) < 22:
            return False
        m = max(self._match(bits, self.SYNC_CONTINUOUS_DOWNLINK), self._match(bits, self.SYNC_DISCONTINUOUS_DOWNLINK))
        return bool(m / 22 > 0.8)

    def _extract_training_sequence(self, bits, burst_type: BurstType):
        return bits[108:130] if burst_type == BurstType.Synchronization else bits[108:122]

    def _extract_data_bits(self, bits, burst_type: BurstType):
        if burst_type in (BurstType.NormalDownlink, BurstType.NormalUplink):
            return np.concatenate([bits[0:108], bits[122:230]])
        return bits

    def _check_crc(self, bits) -> bool:
        """Soft CRC check: <=2 bit errors, reversed-payload retry (protocol.py:292-329)."""
        b = _bits_u8(bits) & 1
        if len(b) == 0:
            return False
        ok = np.zeros(1, np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_check_crc(c.handle, _hip.ptr(np.ascontiguousarray(b)), 1, len(b), _hip.ptr(ok)),
                "tetra_check_crc")
        return bool(ok[0])

    def _calculate_crc16(self, bits) -> np.ndarray:
        """CRC-16/CCITT-FALSE, MSB-first bit list (protocol.py:331-347)."""
        b = np.ascontiguousarray(np.asarray(bits, dtype=np.int64) & 1, dtype=np.uint8)
        if len(b) == 0:
            return np.array([(0xFFFF >> i) & 1 for i in range(15, -1, -1)])
        crc = np.zeros(1, np.uint16)
        c = _hip.ctx()
        c.check(c.lib.tetra_crc16(c.handle, _hip.ptr(b), 1, len(b), 0, _hip.ptr(crc)), "tetra_crc16")
        v = int(crc[0])
        return np.array([(v >> i) & 1 for i in range(15, -1, -1)])

    # upper MAC (protocol.py:349-1300) is the reference's Python; attach it here
    def parse_mac_pdu(self, bits):
        return None

    def get_statistics(self):
        return dict(self.stats)
