"""MI355X TetraDecoder -- the reference's lower-MAC surface, computed by libtetra_hip.so.

Mirrors the hot-path methods of /root/reference/tetraear/core/decoder.py:
  symbols_to_bits  :140-169     find_sync  :171-295     decode :835-888     decode_frame :890-992
Correlation, the greedy sync scan, burst slicing, burst typing and CRC run on the GPU
(tetra_lmac_compat / tetra_find_sync / tetra_symbols_to_bits).  The Python here keeps the
reference's float decisions (threshold comparisons, the adaptive re-search rule) and builds the
frame dicts, through decode_frame's MAC PDU stage (decoder.py:994-1053: parse_mac_pdu on the GPU,
the drop rule, mac_pdu, the encryption fields).  Call metadata, SDS and decryption
(decoder.py:1055-1117) are not part of this hot-path build: they stay the reference's Python and
attach through ``upper_mac``, which runs them -- the reference's parser methods and _decrypt_frame --
whenever the reference's package root is on sys.path after this build's (tetraear/_overlay.py).
Then the other members of the reference's TetraDecoder (common_keys, _decrypt_frame,
format_frame_info, ...) resolve too; the hot-path methods here never delegate.

``mode="etsi"`` (or ``TETRAEAR_DEMOD=etsi`` for callers that construct ``TetraDecoder()``
unchanged) decodes ETSI channel coding (cell acquisition from the BSCH, descramble, deinterleave,
RCPC Viterbi, CRC-16) on the soft bits of the ETSI demodulator instead; see tetraear.core.etsi.
Its frames carry the reference's frame-dict keys, built from the decoded type-1 bits.
"""
import ctypes
import functools
import logging
from typing import Optional

import numpy as np

from tetraear import _hip, _overlay
from tetraear.core.protocol import TetraProtocolParser, burst_data_bits, burst_from_bits

logger = logging.getLogger(__name__)

TS1 = np.array([1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0])
TS2 = np.array([0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0])
FRAME_TYPE_NAMES = {0: "MAC-RESOURCE", 1: "MAC-FRAG", 2: "MAC-BROADCAST", 3: "MAC-END/RES"}
FRAME_TYPE_DESC = {0: "Resource allocation", 1: "Fragment", 2: "Broadcast info", 3: "End/Reserved"}
ENC_MODES = {1: ("TEA1", "Class 2 (SCK)"), 2: ("TEA2", "Class 3 (DCK)"), 3: ("TEA3", "Reserved")}


def count_threshold(thr):
    """Least match count c with c/22 >= thr -- the float test of decoder.py:240-245."""
    for c in range(23):
        if c / 22 >= thr:
            return c
    return 23


def _find_sync_outcome(thr, best):
    """(count threshold used, max_corr) of find_sync(thr) when the stream's best count is `best`.

    With no hit every position is visited, so max_corr is best/22 and the adaptive re-search
    (decoder.py:263-281) is a greedy scan at the adaptive threshold."""
    k = count_threshold(thr)
    if best >= k:
        return k, None
    mc = best / 22
    if mc > 0.75 and mc >= (thr - 0.15):
        ad = max(0.75, mc - 0.02)
        if ad < thr:
            ka = count_threshold(ad)
            if best >= ka:
                return ka, mc
    return None, mc


@functools.lru_cache(maxsize=1)
def cascade_table():
    """decode()'s 0.90 -> 0.85 -> 0.80 -> adaptive cascade (decoder.py:845-857) as a function of
    the stream's best correlation count: the count threshold its sync positions use, or -1."""
    tab = np.full(23, -1, np.int8)
    for best in range(23):
        k, mc = _find_sync_outcome(0.90, best)
        if k is None:
            k, mc = _find_sync_outcome(0.85, best)
        if k is None:
            k, mc = _find_sync_outcome(0.80, best)
            if k is None and mc >= 0.75:
                k, _ = _find_sync_outcome(max(0.75, mc - 0.02), best)
        tab[best] = -1 if k is None else k
    return tab


def _bits_u8(bits):
    b = np.asarray(bits)
    return np.ascontiguousarray(np.where((b == 0) | (b == 1), b, 2), dtype=np.uint8)


class TetraDecoder:
    """Decodes TETRA frames from demodulated symbols (decoder.py:16)."""

    def __init__(self, key_manager=None, auto_decrypt: bool = True, mode=None):
        self.SYNC_PATTERN = [0, 1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0,
                             1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0]
        self.FRAME_LENGTH = 510
        self.key_manager = key_manager
        self.auto_decrypt = auto_decrypt
        self.protocol_parser = TetraProtocolParser()
        self.sync_patterns = {'TS1': TS1.copy(), 'TS2': TS2.copy()}
        self.user_keys = []
        from tetraear.signal.processor import demod_mode
        self.mode = demod_mode(mode)
        self._etsi = None

    # ------------------------------------------------------------------ keys and the reference's rest
    def set_keys(self, keys):
        """User keys for the decryption's brute force (decoder.py:101-138).  Each hex string (spaces,
        ':' and '-' ignored) becomes ('TEA1', key) for 10 bytes, or the same 16 bytes as TEA2, TEA3
        and TEA4; a 32-byte key contributes its first 16 bytes that way.  Other lengths and strings
        that do not parse are logged and skipped."""
        self.user_keys = []
        for text in keys:
            try:
                raw = bytes.fromhex(text.replace(' ', '').replace(':', '').replace('-', ''))
                if len(raw) == 10:
                    self.user_keys.append(('TEA1', raw))
                elif len(raw) in (16, 32):
                    if len(raw) == 32:
                        logger.warning("256-bit key provided; using first 128 bits for TEA2/TEA3/TEA4 attempts")
                    self.user_keys += [(alg, raw[:16]) for alg in ('TEA2', 'TEA3', 'TEA4')]
                else:
                    logger.warning(f"Invalid key length: {len(raw)} bytes (expected 10 or 16)")
            except Exception as e:
                logger.error(f"Failed to parse key '{text}': {e}")
        logger.info(f"Loaded {len(self.user_keys)} user-provided encryption keys")

    def _reference(self):
        return _overlay.reference_module("core/decoder").TetraDecoder

    def __getattr__(self, name):
        """Members of the reference's TetraDecoder this build does not define -- the common-key
        table (decoder.py:36-99), _decrypt_frame (:576-834), format_frame_info and
        _get_frame_type_name (:1121-1200) -- bound to this decoder, when the reference is on the
        path.  Only reached when normal lookup fails: the hot-path methods are never the reference's."""
        if name.startswith("__") or not _overlay.active():
            raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")
        ref = self._reference()
        if name == "common_keys":   # built on first use by the reference's own setup, user keys kept
            users = self.__dict__.get("user_keys", [])
            _overlay.bind(self, ref, "_setup_common_keys")()
            self.user_keys = users
            return self.__dict__["common_keys"]
        if not hasattr(ref, name):
            raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")
        return _overlay.bind(self, ref, name)

    # ------------------------------------------------------------------ bits
    def symbols_to_bits(self, symbols):
        """Dibits MSB-first; 8-PSK neighbour map when max(symbols) > 3 (decoder.py:140-169)."""
        s = np.asarray(symbols)
        if len(s) == 0:
            return np.array([]), np.array([])
        s = np.ascontiguousarray(s, dtype=np.int64)
        bits = np.empty(2 * len(s), np.int64)
        mapped = np.empty(len(s), np.int64)
        c = _hip.ctx()
        c.check(c.lib.tetra_symbols_to_bits(c.handle, _hip.ptr(s), len(s), _hip.ptr(bits), _hip.ptr(mapped)),
                "tetra_symbols_to_bits")
        return bits, mapped

    # ------------------------------------------------------------------ sync
    def _greedy(self, b, k, maxpos):
        pos = np.zeros(max(1, maxpos), np.int64)
        n, mc = ctypes.c_int32(0), ctypes.c_int32(0)
        c = _hip.ctx()
        c.check(c.lib.tetra_find_sync(c.handle, _hip.ptr(b), len(b), k, _hip.ptr(pos), len(pos), n, mc),
                "tetra_find_sync")
        return [int(p) for p in pos[:min(n.value, len(pos))]], mc.value

    def find_sync(self, bits, threshold=0.85, return_max_corr=False):
        """22-bit TS1/TS2 correlation with greedy +250 skip and adaptive re-search (decoder.py:171-295)."""
        self.sync_patterns = {'TS1': TS1.copy(), 'TS2': TS2.copy()}
        if len(bits) < 22:
            return ([], 0.0) if return_max_corr else []
        b = _bits_u8(bits)
        maxpos = (len(b) - 21) // 250 + 2
        sync, maxc = self._greedy(b, count_threshold(threshold), maxpos)
        max_corr = maxc / 22
        if not sync and max_corr > 0.75 and max_corr >= (threshold - 0.15):
            adaptive = max(0.75, max_corr - 0.02)
            if adaptive < threshold:
                sync, _ = self._greedy(b, count_threshold(adaptive), maxpos)
                logger.debug(f"Found {len(sync)} syncs at adaptive threshold {adaptive:.4f} "
                             f"(max: {max_corr:.4f}, original: {threshold:.4f})")
        return (sync, max_corr) if return_max_corr else sync

    # ------------------------------------------------------------------ frames
    def decode(self, symbols):
        """Sync cascade, slot slicing and burst parsing of one symbol stream (decoder.py:835-888)."""
        if self.mode == "etsi":
            return self._etsi_frames(self._etsi_rx().decode(symbols))
        return self.decode_batch([symbols])[0]

    def decode_batch(self, streams):
        """decode() over many independent symbol streams with one device pass per stage: sync,
        slicing, burst typing and CRC in one tetra_lmac_compat launch, then the MAC PDU headers of
        every slot in one tetra_mac_headers launch.  The parser state (statistics, fragment buffer,
        SYSINFO) is applied in stream and frame order, as consecutive decode() calls would."""
        streams = [np.asarray(s) for s in streams]
        C = len(streams)
        stride = max([len(s) for s in streams] + [1])
        sym = np.zeros((C, stride), np.int64)
        ns = np.zeros(C, np.int32)
        for i, s in enumerate(streams):
            sym[i, :len(s)] = s
            ns[i] = len(s)
        nsync = np.zeros(C, np.int32)
        rec = np.zeros((C, _hip.MAX_SYNC, _hip.F_FIELDS), np.int32)
        fbits = np.zeros((C, _hip.MAX_SYNC, 510), np.uint8)
        bbits = np.zeros((C, _hip.MAX_SYNC, 510), np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_lmac_compat(c.handle, _hip.ptr(sym), _hip.ptr(ns), C, stride, _hip.ptr(cascade_table()),
                                        _hip.ptr(nsync), _hip.ptr(rec), _hip.ptr(fbits), _hip.ptr(bbits)),
                "tetra_lmac_compat")
        slots = []   # (stream, record, frame bits, burst bits) of every slot decode_frame parses
        for i in range(C):
            for f in range(int(nsync[i])):
                r = rec[i, f]
                if r[_hip.F_VALID] and int(r[_hip.F_NBITS]) >= self.FRAME_LENGTH:
                    slots.append((i, r, fbits[i, f, :int(r[_hip.F_NBITS])], bbits[i, f]))
        # parse_mac_pdu(burst.data_bits) of every slot (decoder.py:996): device header fields
        rows = [burst_data_bits(bb, int(r[_hip.F_BTYPE])) for _, r, _, bb in slots]
        fields, data = self.protocol_parser.mac_fields(rows) if rows else (None, None)
        out = [[] for _ in range(C)]
        for k, (i, r, fb, bb) in enumerate(slots):
            number = int(r[_hip.F_NUMBER])
            frame = self._frame_dict(fb.astype(np.int64), 0, number)
            crc_ok = bool(r[_hip.F_CRC])
            self.protocol_parser.count_burst(crc_ok)
            burst = burst_from_bits(bb, int(r[_hip.F_BTYPE]), crc_ok, number % 4,
                                    self.protocol_parser.current_frame_number, self.protocol_parser.colour_code or 0)
            frame['burst_crc'] = crc_ok
            pdu = self.protocol_parser.mac_state(fields[k], data[k])
            frame = self._mac_stage(frame, burst, pdu)
            if frame:
                out[i].append(frame)
                logger.info(f"Decoded frame {frame['number']} (type: {frame['type']})")
        return out

    def _frame_dict(self, frame_bits, start_pos, frame_number):
        """The lower-MAC frame dict of decode_frame (decoder.py:898-972)."""
        pdu = int(frame_bits[0]) * 2 + int(frame_bits[1])
        enc = int(frame_bits[2]) * 2 + int(frame_bits[3])
        info = {'description': FRAME_TYPE_DESC.get(pdu, f'Raw type {pdu}')}
        alg = None
        if enc in ENC_MODES:
            alg, info['encryption_mode'] = ENC_MODES[enc]
        return {
            'type': pdu,
            'type_name': FRAME_TYPE_NAMES.get(pdu, f"Type {pdu}"),
            'number': frame_number,
            'timeslot': frame_number % 4,
            'bits': frame_bits,
            'header': "".join("1" if v else "0" for v in frame_bits[:32]),
            'position': start_pos,
            'encrypted': enc > 0,
            'encryption_algorithm': alg,
            'key_id': '0',
            'additional_info': info,
        }

    def _mac_stage(self, frame, burst, pdu):
        """decode_frame's MAC PDU stage (decoder.py:994-1100) on the parsed PDU of the slot.

        No PDU and a failed CRC drops the frame (decoder.py:1093-1095).  A PDU adds
        frame['mac_pdu'] and settles 'encrypted' / 'encryption_algorithm': from the PDU's mode when
        it is encrypted (decoder.py:1008-1035), otherwise by the data-entropy rule -- more than 8
        bytes with a distinct-byte ratio above 0.7 count as encrypted (decoder.py:1036-1053).
        Then upper_mac (call metadata / SDS, decoder.py:1055-1091) runs on the kept frame."""
        if pdu is None:
            return self.upper_mac(frame, burst, None) if burst.crc_ok else None
        frame['mac_pdu'] = {'type': pdu.pdu_type.name, 'encrypted': pdu.encrypted, 'address': pdu.address,
                            'length': pdu.length, 'data': pdu.data}
        if pdu.encrypted:
            frame['encrypted'] = True
            mode = getattr(pdu, 'encryption_mode', 0)
            if mode in ENC_MODES:
                frame['encryption_algorithm'], frame['additional_info']['encryption_mode'] = ENC_MODES[mode]
            elif not frame['encryption_algorithm']:
                frame['encryption_algorithm'] = 'TEA1'
        else:
            n = len(pdu.data)
            if n > 0 and len(set(pdu.data)) / max(n, 1) > 0.7 and n > 8:
                frame['encrypted'] = True
            else:
                frame['encrypted'] = False
                frame['encryption_algorithm'] = None
        return self.upper_mac(frame, burst, pdu)

    def decode_frame(self, bits, start_pos, symbols=None, frame_number=0):
        """Frame header, burst parse and MAC PDU stage of one 510-bit slot (decoder.py:890-1100)."""
        if len(bits) < self.FRAME_LENGTH:
            return None
        fb = np.asarray(bits)
        frame = self._frame_dict(fb, start_pos, frame_number)
        try:
            if symbols is None:   # rebuild 0-3 symbols from bit pairs (decoder.py:977-983)
                b = fb.astype(np.int64)
                if len(b) % 2:
                    raise IndexError("index out of range")
                symbols = (b[0::2] << 1) | b[1::2]
            burst = self.protocol_parser.parse_burst(np.asarray(symbols), slot_number=frame_number % 4)
            if burst:
                frame['burst_crc'] = burst.crc_ok
                return self._mac_stage(frame, burst, self.protocol_parser.parse_mac_pdu(burst.data_bits))
        except Exception as e:   # the reference logs and keeps the frame (decoder.py:1102-1103)
            logger.debug(f"Protocol parsing error: {e}")
        return frame

    def upper_mac(self, frame, burst, mac_pdu=None):
        """The reference's call metadata, SDS and decryption (decoder.py:1055-1117), called with every
        frame the MAC PDU stage keeps and its MacPDU (None when the slot has none).

        With the reference on the path (tetraear/_overlay.py) this runs them: the parser's
        parse_call_metadata / parse_sds_data and this decoder's _decrypt_frame are the reference's own
        methods, and the frame gains the reference's upper-MAC keys -- call_metadata, sds_message,
        decoded_text, is_reassembled, additional_info's talkgroup / source_ssi / mcc / mnc / sds_text,
        and the decryption's fields -- with the reference's frame selection: an exception in the
        metadata / SDS step drops a frame whose CRC failed (decoder.py:1097-1100).  Without the
        reference it returns the frame unchanged: this build's frames then carry the lower-MAC and
        MAC PDU fields only (upper MAC out of scope; tests/test_oracle_golden.py declares
        exactly the keys above as the gap).  A subclass may override it."""
        if not _overlay.active():
            return frame
        info = frame['additional_info']
        if mac_pdu is not None:
            try:
                meta = self.protocol_parser.parse_call_metadata(mac_pdu)
                if meta:
                    frame['call_metadata'] = {
                        'call_type': meta.call_type, 'talkgroup_id': meta.talkgroup_id, 'source_ssi': meta.source_ssi,
                        'dest_ssi': meta.dest_ssi, 'channel': meta.channel_allocated,
                        'call_identifier': meta.call_identifier, 'priority': meta.call_priority, 'mcc': meta.mcc,
                        'mnc': meta.mnc, 'encryption': meta.encryption_enabled,
                        'encryption_alg': meta.encryption_algorithm}
                    for key, v in (('talkgroup', meta.talkgroup_id), ('source_ssi', meta.source_ssi),
                                   ('mcc', meta.mcc), ('mnc', meta.mnc)):
                        if v:
                            info[key] = v
                payload = mac_pdu.reassembled_data if mac_pdu.reassembled_data else mac_pdu.data
                if not mac_pdu.encrypted and len(payload) > 0:
                    text = self.protocol_parser.parse_sds_data(payload)
                    if text and not text.startswith("[BIN]"):
                        frame['sds_message'] = frame['decoded_text'] = text
                        info['sds_text'] = text[:50]
                        if mac_pdu.reassembled_data:
                            frame['is_reassembled'] = True
                            info['description'] += " (Reassembled)"
            except Exception as e:
                logger.debug(f"MAC PDU parsing error: {e}")
                if not burst.crc_ok:
                    return None
        if frame.get('encrypted') and (self.key_manager or self.auto_decrypt):
            frame = self._decrypt_frame(frame)
            if frame.get('decrypted') and 'decrypted_bytes' in frame:
                try:
                    text = self.protocol_parser.parse_sds_data(bytes.fromhex(frame['decrypted_bytes']))
                    if text:
                        frame['sds_message'] = frame['decoded_text'] = text
                        info['sds_text'] = text[:50]
                except Exception:
                    pass
        return frame

    def _etsi_frames(self, raw):
        """ETSI bursts as the reference's frame dicts (decoder.py:960-972 keys + the MAC PDU stage),
        built from the channel-decoded type-1 bits.  Every logical channel block carries its own MAC
        PDU (EN 300 392-2 §21.4), so the MAC stage runs once per CRC-good SCH/F or SCH/HD block, in
        burst and block order: the BSCH is skipped (its MAC-SYNC PDU has another layout, and the
        cell it carries is already EtsiLowerMac's acquisition) and CRC-failed blocks are not parsed
        (their bits are not the transmitted ones).  Per burst: frame number start // 510,
        burst_crc = every block's CRC-16, the frame header and type from the first MAC block, and the
        compat drop rule (no PDU and a failed CRC drops the burst).  The burst's first PDU goes
        through the compat MAC stage ('mac_pdu', 'encrypted', 'encryption_algorithm'); all of them
        are on 'mac_pdus'.  The ETSI details stay on the frame: 'blocks', 'burst', 'burst_kind'."""
        from tetraear.core.protocol import BurstType, TetraBurst
        rows, owner = [], []   # one row per CRC-good SCH/F / SCH/HD block, in order
        for i, f in enumerate(raw):
            for b in f["blocks"]:
                if b["channel"] != "BSCH" and b["crc_ok"]:
                    rows.append(np.asarray(b["bits"], np.uint8))
                    owner.append(i)
        fields, data = self.protocol_parser.mac_fields(rows) if rows else (None, None)
        pdus = [[] for _ in raw]
        out = []
        k = 0
        for i, f in enumerate(raw):
            mac_blocks = [b for b in f["blocks"] if b["channel"] != "BSCH"] or f["blocks"]
            if not mac_blocks:
                continue
            bits = np.asarray(mac_blocks[0]["bits"]).astype(np.int64)
            number = f["position"] // 510
            frame = self._frame_dict(bits, f["position"], number)
            crc_ok = bool(f["crc_ok"])
            self.protocol_parser.count_burst(crc_ok)
            frame.update(burst_crc=crc_ok, blocks=f["blocks"], burst=f["burst"], burst_kind=f["burst_kind"])
            while k < len(owner) and owner[k] == i:   # the MAC state advances in block order
                pdu = self.protocol_parser.mac_state(fields[k], data[k])
                if pdu is not None:
                    pdus[i].append(pdu)
                k += 1
            burst = TetraBurst(burst_type=BurstType.Synchronization if f["burst_kind"] == 2 else BurstType.NormalDownlink,
                               slot_number=number % 4, frame_number=self.protocol_parser.current_frame_number,
                               training_sequence=np.zeros(0, np.int64),
                               data_bits=np.concatenate([np.asarray(b["bits"]) for b in f["blocks"]]).astype(np.int64),
                               crc_ok=crc_ok, colour_code=self._etsi.colour_code or 0)
            frame = self._mac_stage(frame, burst, pdus[i][0] if pdus[i] else None)
            if frame:
                frame['mac_pdus'] = [{'type': p.pdu_type.name, 'encrypted': p.encrypted, 'address': p.address,
                                      'length': p.length, 'data': p.data} for p in pdus[i]]
                out.append(frame)
        return out

    def _etsi_rx(self):
        if self._etsi is None:
            from tetraear.core.etsi import EtsiLowerMac
            self._etsi = EtsiLowerMac()
        return self._etsi
