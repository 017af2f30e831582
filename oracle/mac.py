"""CPU restatement of TetraProtocolParser.parse_mac_pdu (TEST INFRASTRUCTURE ONLY -- the checker).

Follows /root/reference/tetraear/core/protocol.py:349-596 statement by statement, for 0/1 bit
vectors: the header fields, the strict length checks, the SYSINFO MCC/MNC/colour-code state, and
the fragment buffer (MAC-RESOURCE starts it, MAC-FRAG appends, MAC-END appends, finalises, clears).
Pinned by tests/golden/g4_mac.npz (make_golden_mac.py runs the reference itself).  Only tests/
may import it; the product parses headers on the GPU (tetra_mac_headers).
"""


def _uint(bits):
    """int(''.join(str(b) for b in bits), 2) for 0/1 bits (protocol.py:412,420,483-485)."""
    v = 0
    for b in bits:
        v = (v << 1) | int(b)
    return v


def _tobytes(bits):
    """BitArray(bits).tobytes(): MSB-first, the last byte zero-padded (protocol.py:442)."""
    out = bytearray()
    for i in range(0, len(bits), 8):
        chunk = [int(bool(b)) for b in bits[i:i + 8]]
        chunk += [0] * (8 - len(chunk))
        out.append(_uint(chunk))
    return bytes(out)


class MacParser:
    """The state parse_mac_pdu reads and writes (protocol.py:164-190)."""

    def __init__(self):
        self.mcc = self.mnc = self.colour_code = None
        self.n_clear = self.n_enc = 0
        self.fragment_buffer = bytearray()
        self.fragment_metadata = {}

    def parse(self, bits):
        """protocol.py:349-596; returns None or a dict of the MacPDU fields (pdu_type as the
        PDUType enum value)."""
        bits = [int(b) for b in bits]
        n = len(bits)
        if n < 8:                                                   # :360-361
            return None
        pti = (bits[0] << 1) | bits[1]                              # :369
        ptype = {0: 0, 1: 1, 2: 3}.get(pti, 2)                      # :372-382 (MAC_END = 2)
        mode = (bits[2] << 1) | bits[3]                             # :389
        encrypted = mode > 0
        address, length, data, fill = None, 0, b"", 0
        if ptype == 0:                                              # MAC-RESOURCE :399-449
            fill = bits[4]
            pos = 5
            if n < pos + 24:
                return None
            address = _uint(bits[pos:pos + 24])
            pos += 24
            if n < pos + 6:
                return None
            length = _uint(bits[pos:pos + 6])
            pos += 6
            dl = length * 8
            if dl > n - pos + 16:                                   # :433-434
                return None
            data = _tobytes(bits[pos:pos + dl] if dl > 0 and n >= pos + dl else bits[pos:])
            self.fragment_buffer = bytearray(data)
            self.fragment_metadata = {"address": address, "encrypted": encrypted, "mode": mode}
        elif ptype == 1:                                            # MAC-FRAG :451-469
            fill = bits[4]
            data = _tobytes(bits[5:])
            self.fragment_buffer.extend(data)
            if self.fragment_metadata:
                encrypted = self.fragment_metadata.get("encrypted", False)
                address = self.fragment_metadata.get("address")
        elif ptype == 3:                                            # MAC-BROADCAST :471-504
            btype = (bits[2] << 1) | bits[3]
            pos = 4
            if btype == 0:
                if n < pos + 30:
                    return None
                self.mcc = _uint(bits[pos:pos + 10])
                self.mnc = _uint(bits[pos + 10:pos + 24])
                self.colour_code = _uint(bits[pos + 24:pos + 30])
                if self.mcc < 200 or self.mcc > 799 or self.mnc > 999:   # :489-494
                    return None
            data = _tobytes(bits[pos:])
        else:                                                       # MAC-END :506-544
            fill = bits[4]
            pos = 5
            if n < pos + 6:
                return None
            length = _uint(bits[pos:pos + 6])
            pos += 6
            dl = length * 8
            if dl > n - pos + 16:
                return None
            data = _tobytes(bits[pos:pos + dl] if dl > 0 and n >= pos + dl else bits[pos:])
            self.fragment_buffer.extend(data)
            if self.fragment_metadata:
                encrypted = self.fragment_metadata.get("encrypted", False)
                address = self.fragment_metadata.get("address")
        if encrypted:                                               # :546-549
            self.n_enc += 1
        else:
            self.n_clear += 1
        pdu = dict(pdu_type=ptype, encrypted=encrypted, address=address, length=length, data=data,
                   fill_bits=fill, encryption_mode=mode, reassembled_data=None)
        if ptype == 2:                                              # :573-583
            if self.fragment_buffer:
                pdu["reassembled_data"] = bytes(self.fragment_buffer)
                if self.fragment_metadata:
                    if not pdu["address"]:
                        pdu["address"] = self.fragment_metadata.get("address")
                    pdu["encrypted"] = self.fragment_metadata.get("encrypted", False)
                self.fragment_buffer = bytearray()
                self.fragment_metadata = {}
        elif ptype == 0:                                            # :585-594
            pdu["reassembled_data"] = bytes(data)
        return pdu
