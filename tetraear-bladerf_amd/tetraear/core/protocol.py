"""Burst-level protocol types and the lower-MAC half of TetraProtocolParser, on the GPU.

Mirrors the hot-path part of /root/reference/tetraear/core/protocol.py:
  enums and dataclasses (BurstType, ChannelType, PDUType, TetraBurst, MacPDU, CallMetadata)
                                                             protocol.py:34-139
  TetraProtocolParser.parse_burst and helpers, _check_crc, _calculate_crc16
                                                             protocol.py:142-347
  parse_mac_pdu (MAC PDU headers, fragment reassembly)          protocol.py:349-596
Burst typing, slicing, the CRC and the MAC PDU header fields run in libtetra_hip.so.  The rest of
the reference's upper MAC (call metadata, SDS, LIP, GSM 7-bit text -- protocol.py:597-1300) is out
of scope of this hot-path build and stays the reference's Python: with the reference's package
root on sys.path after this build's (tetraear/_overlay.py), ``parse_call_metadata``,
``parse_sds_message``, ``parse_sds_data``, ``parse_lip``, ``extract_voice_payload``,
``format_call_metadata`` and their helpers run the reference's own methods on this parser's state
(MCC / MNC / colour code, statistics), with this module's enums and dataclasses.
"""
import logging
from dataclasses import dataclass
from enum import Enum
from typing import Optional

import numpy as np

from tetraear import _hip, _overlay

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


def burst_data_bits(bits510, btype_value):
    """_extract_data_bits (protocol.py:277-290): all 510 bits of a synchronisation burst, else
    bits[0:108] + bits[122:230]."""
    if btype_value == BurstType.Synchronization.value:
        return bits510
    return np.concatenate([bits510[0:108], bits510[122:230]])


def burst_from_bits(bits510, btype_value, crc_ok, slot_number, frame_number, colour_code):
    """Assemble a TetraBurst from the device's burst bits (protocol.py:267-290 slices)."""
    bits = bits510.astype(np.int64)
    data = burst_data_bits(bits, btype_value)
    if btype_value == BurstType.Synchronization.value:
        ts = bits[108:130]
    else:
        ts = bits[108:122]
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

    def parse_mac_pdu(self, bits) -> Optional[MacPDU]:
        """MAC PDU of one slot's data bits (protocol.py:349-596): header fields and data bytes
        from the GPU (tetra_mac_headers), fragment buffer / SYSINFO state / statistics here."""
        if len(bits) < 8:   # protocol.py:360-361, without a launch
            return None
        return self.parse_mac_pdu_batch([bits])[0]

    def parse_mac_pdu_batch(self, frames) -> list:
        """parse_mac_pdu over many frames in order, one launch: [MacPDU or None].

        Frames are 0/1 integer bit vectors, as parse_burst's data_bits.  The reference raises a
        ValueError from int(..., 2) when a parsed header field holds anything else (bool arrays
        included: int('TrueFalse', 2)).  This build checks every frame of 8 or more bits: at the
        first bad frame, the frames before it are parsed (their fragment / SYSINFO / statistics
        state applied, as the reference's sequential calls would have left it) and then the
        ValueError is raised, so the batch returns nothing."""
        rows = [np.asarray(f).ravel() for f in frames]
        for i, r in enumerate(rows):
            if r.size >= 8 and (r.dtype == np.bool_ or not np.all((r == 0) | (r == 1))):
                self._mac_batch(rows[:i])
                raise ValueError(f"parse_mac_pdu: frame {i}: bits must be integer 0/1")
        return self._mac_batch(rows)

    def mac_fields(self, rows):
        """The stateless device half of parse_mac_pdu for many 0/1 rows: (fields [F, MAC_FIELDS],
        packed data bytes [F, stride/8]) from one tetra_mac_headers launch."""
        F = len(rows)
        stride = max(8, max(r.size for r in rows))
        bits = np.zeros((F, stride), np.uint8)
        nbits = np.zeros(F, np.int32)
        for i, r in enumerate(rows):
            bits[i, :r.size] = r
            nbits[i] = r.size
        dstride = (stride + 7) // 8
        fields = np.zeros((F, _hip.MAC_FIELDS), np.int32)
        data = np.zeros((F, dstride), np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_mac_headers(c.handle, _hip.ptr(bits), _hip.ptr(nbits), F, stride, _hip.ptr(fields),
                                        _hip.ptr(data), dstride), "tetra_mac_headers")
        return fields, data

    def _mac_batch(self, rows):
        if not rows:
            return []
        fields, data = self.mac_fields(rows)
        return [self.mac_state(fields[i], data[i]) for i in range(len(rows))]

    def mac_state(self, r, data):
        """The stateful half of parse_mac_pdu for one frame's device fields, applied in frame order."""
        status = int(r[_hip.MAC_STATUS])
        if r[_hip.MAC_SYSINFO]:   # set before the sanity check (protocol.py:483-485)
            self.mcc, self.mnc, self.colour_code = int(r[_hip.MAC_MCC]), int(r[_hip.MAC_MNC]), int(r[_hip.MAC_CC])
            if status == 2:
                logger.debug(f"Invalid MCC {self.mcc} / MNC {self.mnc} in SYNC - not real TETRA")
            else:
                logger.info(f"Valid TETRA SYNC: MCC={self.mcc} MNC={self.mnc}")
        if status != 0:
            return None
        ptype = PDUType(int(r[_hip.MAC_PTYPE]))
        mode = int(r[_hip.MAC_MODE])
        encrypted = mode > 0
        address = int(r[_hip.MAC_ADDR]) if ptype == PDUType.MAC_RESOURCE else None
        length = int(r[_hip.MAC_LENGTH])
        data_bytes = bytes(data[:(int(r[_hip.MAC_DATA_BITS]) + 7) // 8])
        if ptype == PDUType.MAC_RESOURCE:                                   # protocol.py:446-449
            self.fragment_buffer = bytearray(data_bytes)
            self.fragment_metadata = {'address': address, 'encrypted': encrypted, 'mode': mode}
        elif ptype in (PDUType.MAC_FRAG, PDUType.MAC_END):                  # :463-469, :538-544
            self.fragment_buffer.extend(data_bytes)
            if self.fragment_metadata:
                encrypted = self.fragment_metadata.get('encrypted', False)
                address = self.fragment_metadata.get('address')
        self.stats['encrypted_frames' if encrypted else 'clear_mode_frames'] += 1   # :546-549
        pdu = MacPDU(pdu_type=ptype, encrypted=encrypted, address=address, length=length, data=data_bytes,
                     fill_bits=int(r[_hip.MAC_FILL]), encryption_mode=mode)
        if ptype == PDUType.MAC_END:                                        # :573-583
            if self.fragment_buffer:
                pdu.reassembled_data = bytes(self.fragment_buffer)
                if self.fragment_metadata:
                    if not pdu.address:
                        pdu.address = self.fragment_metadata.get('address')
                    pdu.encrypted = self.fragment_metadata.get('encrypted', False)
                self.fragment_buffer = bytearray()
                self.fragment_metadata = {}
        elif ptype == PDUType.MAC_RESOURCE:                                 # :585-594
            pdu.reassembled_data = bytes(data_bytes)
        return pdu

    def get_statistics(self):
        """The counters plus clear / encrypted shares and the CRC success rate, in percent
        (protocol.py:1261-1275)."""
        frames = self.stats['clear_mode_frames'] + self.stats['encrypted_frames']
        clear = self.stats['clear_mode_frames'] / frames * 100 if frames > 0 else 0
        enc = self.stats['encrypted_frames'] / frames * 100 if frames > 0 else 0
        return {**self.stats, 'clear_mode_percentage': clear, 'encrypted_percentage': enc,
                'crc_success_rate': self.stats['crc_pass'] / max(1, self.stats['total_bursts']) * 100}

    # ------------------------------------------------------------ upper MAC: the reference's
    def _reference(self):
        mod = _overlay.reference_module("core/protocol", patch={
            "BurstType": BurstType, "ChannelType": ChannelType, "PDUType": PDUType, "TetraBurst": TetraBurst,
            "MacPDU": MacPDU, "CallMetadata": CallMetadata})
        return mod.TetraProtocolParser

    def __getattr__(self, name):
        """Members of the reference parser this build does not define (the upper MAC's helpers,
        protocol.py:623-1260), bound to this parser; only reached when normal lookup fails, so the
        hot-path methods above are never the reference's."""
        if name.startswith("__") or not _overlay.active():
            raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")
        ref = self._reference()
        if not hasattr(ref, name):
            raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")
        return _overlay.bind(self, ref, name)

    def parse_call_metadata(self, mac_pdu):
        """Talkgroup / SSI / channel of a MAC PDU (protocol.py:597-621), the reference's."""
        return _overlay.bind(self, self._reference(), "parse_call_metadata")(mac_pdu)

    def parse_sds_message(self, mac_pdu):
        """SDS text of a MAC PDU (protocol.py:786-800), the reference's."""
        return _overlay.bind(self, self._reference(), "parse_sds_message")(mac_pdu)

    def parse_sds_data(self, data):
        """SDS payload bytes to text (protocol.py:802-1018), the reference's."""
        return _overlay.bind(self, self._reference(), "parse_sds_data")(data)

    def parse_lip(self, data):
        """Location Information Protocol payload (protocol.py:1020-1112), the reference's."""
        return _overlay.bind(self, self._reference(), "parse_lip")(data)

    def extract_voice_payload(self, mac_pdu):
        """Voice frame bytes of a traffic MAC PDU (protocol.py:1239-1259), the reference's."""
        return _overlay.bind(self, self._reference(), "extract_voice_payload")(mac_pdu)

    def format_call_metadata(self, metadata):
        """Display string of a CallMetadata (protocol.py:1277-1300), the reference's."""
        return _overlay.bind(self, self._reference(), "format_call_metadata")(metadata)
