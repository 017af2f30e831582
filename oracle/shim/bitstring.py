"""Minimal stand-in for the third-party ``bitstring`` package (TEST INFRASTRUCTURE ONLY).

The reference lists ``bitstring>=4.0.0`` (/root/reference/requirements.txt:5) but it is not
installed in this image and there is no network.  The reference's hot path touches only a
tiny part of its API (/root/reference/tetraear/core/decoder.py:898-909,
/root/reference/tetraear/core/protocol.py:442-534,743-752,1037-1072):

* ``BitArray(iterable_of_truthy)`` and ``BitArray(bytes)``
* slicing -> ``BitArray``; ``.uint``; ``.int`` (two's complement); ``.bin``; ``.tobytes()``
  (zero-padded to a whole byte, as bitstring 4 does).

This module is put on ``sys.path`` ONLY by ``tests/golden/make_golden.py`` when it imports the
reference to record golden vectors.  Nothing in the product imports it.
"""


class BitArray:
    __slots__ = ("_b",)

    def __init__(self, auto=None):
        if auto is None:
            self._b = []
        elif isinstance(auto, BitArray):
            self._b = list(auto._b)
        elif isinstance(auto, (bytes, bytearray, memoryview)):
            out = []
            for byte in bytes(auto):
                out.extend((byte >> (7 - k)) & 1 for k in range(8))
            self._b = out
        else:
            self._b = [1 if v else 0 for v in auto]

    def __len__(self):
        return len(self._b)

    def __iter__(self):
        return iter(bool(v) for v in self._b)

    def __getitem__(self, key):
        if isinstance(key, slice):
            out = BitArray()
            out._b = self._b[key]
            return out
        return bool(self._b[key])

    @property
    def uint(self):
        if not self._b:
            raise ValueError("empty bitstring has no uint value")
        v = 0
        for b in self._b:
            v = (v << 1) | b
        return v

    @property
    def int(self):
        u = self.uint
        n = len(self._b)
        return u - (1 << n) if self._b[0] else u

    @property
    def bin(self):
        return "".join("1" if b else "0" for b in self._b)

    def tobytes(self):
        bits = self._b + [0] * ((-len(self._b)) % 8)
        out = bytearray()
        for i in range(0, len(bits), 8):
            v = 0
            for b in bits[i:i + 8]:
                v = (v << 1) | b
            out.append(v)
        return bytes(out)

    @property
    def bytes(self):
        return self.tobytes()
