"""Child process of tests/test_dropin_overlay.py (TEST INFRASTRUCTURE; runs only where the reference
is present, i.e. in the build container).

    python tests/overlay_probe.py reference OUT.json   # sys.path: the reference (+ bitstring shim)
    python tests/overlay_probe.py overlay OUT.json     # sys.path: this build, then the reference

`reference` decodes the g2 golden symbol streams with the reference's own TetraDecoder.decode() and
writes every kept frame dict (all keys, upper MAC included), plus set_keys / parse_sds_data results.

`overlay` runs on this build's package with the reference behind it (tetraear/_overlay.py) and
writes: which file each module modern.py:193-201 imports resolves to, where the hot-path methods
live, the same set_keys / parse_sds_data results, and the g2 frames through this build's MAC PDU
stage and upper_mac.  There is no GPU here, so the device half of decode() (sync, slicing, burst
CRC, MAC PDU header fields) is taken from the CPU oracle -- itself pinned to these fixtures
(test_oracle_golden.py) -- and fed to TetraDecoder._mac_stage exactly as decode_batch feeds the
device's results; everything from the MAC PDU on is the build's code and the reference's upper MAC.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

KEYS = ["00112233445566778899", "AA BB CC DD EE FF 00 11 22 33 44 55 66 77 88 99", "0a:0b:0c:0d:0e:0f:10:11:12:13",
        "zz", "1234", "ff" * 32]
SDS = [b"", b"\x01", b"\x01\x02Hello world", b"\x02\x05\x00TEST MESSAGE 42", bytes(range(40)), b"\xff" * 12,
       b"\x0a\x00\x48\x45\x4c\x4c\x4f\x20\x57\x4f\x52\x4c\x44", b"\x03" + bytes(range(65, 91))]


def jsonable(v):
    if isinstance(v, (bytes, bytearray)):
        return {"bytes": bytes(v).hex()}
    if isinstance(v, np.ndarray):
        return [int(x) for x in v.tolist()]
    if isinstance(v, dict):
        return {str(k): jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [jsonable(x) for x in v]
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.bool_):
        return bool(v)
    return v


def streams():
    z = np.load(os.path.join(HERE, "golden", "g2_decode.npz"))
    n = len([k for k in z.files if k.endswith("_sym")])
    return [z[f"s{i}_sym"] for i in range(n)]


def common(TetraDecoder, TetraProtocolParser, out):
    d = TetraDecoder(auto_decrypt=False)
    d.set_keys(KEYS)
    out["user_keys"] = [[a, k.hex()] for a, k in d.user_keys]
    p = TetraProtocolParser()
    out["sds"] = [p.parse_sds_data(b) for b in SDS]
    out["sds_stats"] = dict(p.stats)


def reference(path):
    sys.path[:0] = [os.environ["TETRA_REFERENCE"], os.path.join(REPO, "oracle", "shim")]
    from tetraear.core.decoder import TetraDecoder
    from tetraear.core.protocol import TetraProtocolParser
    out = {}
    common(TetraDecoder, TetraProtocolParser, out)
    for ad in (False, True):
        res = []
        for sym in streams():
            dec = TetraDecoder(auto_decrypt=ad)
            res.append([jsonable(f) for f in dec.decode(sym)])
        out[f"frames_{ad}"] = res
    json.dump(out, open(path, "w"))


def overlay(path):
    sys.path[:0] = [os.path.join(REPO, "tetraear-bladerf_amd")]
    sys.path.append(os.environ["TETRA_REFERENCE"])
    sys.path.append(os.path.join(REPO, "oracle", "shim"))
    import importlib
    out = {"modules": {}}
    for m in ("tetraear.signal.capture", "tetraear.signal.processor", "tetraear.core.decoder", "tetraear.core.crypto",
              "tetraear.core.mcc_mnc", "tetraear.core.validator", "tetraear.core.location", "tetraear.signal.scanner",
              "tetraear.audio.voice", "tetraear.core.protocol"):
        out["modules"][m] = os.path.realpath(importlib.import_module(m).__file__)
    # the names modern.py:193-201 imports
    from tetraear.signal.capture import BladeRFCapture, list_bladerf_devices  # noqa: F401
    from tetraear.signal.processor import SignalProcessor
    from tetraear.core.decoder import TetraDecoder
    from tetraear.core.crypto import TetraKeyManager  # noqa: F401
    from tetraear.core.mcc_mnc import get_location_info  # noqa: F401
    from tetraear.core.validator import TetraSignalValidator  # noqa: F401
    from tetraear.core.location import LocationParser  # noqa: F401
    from tetraear.signal.scanner import FrequencyScanner, TetraSignalDetector
    from tetraear.audio.voice import VoiceProcessor  # noqa: F401
    from tetraear.core import TetraProtocolParser, TEADecryptor, MacPDU, PDUType, TetraBurst, BurstType  # noqa: F401
    import tetraear
    out["top_level"] = [n for n in tetraear.__all__ if getattr(tetraear, n, None) is not None]
    hot = {"SignalProcessor": (SignalProcessor, ["process", "process_batch", "filter_signal", "demodulate_dqpsk",
                                                 "extract_symbols", "frequency_shift", "resample"]),
           "TetraDecoder": (TetraDecoder, ["decode", "decode_frame", "find_sync", "symbols_to_bits", "set_keys",
                                           "upper_mac"]),
           "TetraProtocolParser": (TetraProtocolParser, ["parse_burst", "_check_crc", "_calculate_crc16",
                                                         "parse_mac_pdu", "get_statistics"])}
    out["hot"] = {f"{c}.{m}": os.path.realpath(sys.modules[getattr(cls, m).__module__].__file__)
                  for c, (cls, ms) in hot.items() for m in ms}
    out["scanner_detector"] = type(FrequencyScanner(None).detector) is TetraSignalDetector
    common(TetraDecoder, TetraProtocolParser, out)
    d = TetraDecoder(auto_decrypt=True)
    out["common_keys"] = sorted(d.common_keys)
    out["bound"] = [type(d._decrypt_frame).__name__, d.format_frame_info.__func__.__module__]
    # g2 through the build's MAC PDU stage + upper MAC, the device half from the oracle
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import compat as O
    from mac import MacParser
    for ad in (False, True):
        res = []
        for sym in streams():
            dec = TetraDecoder(auto_decrypt=ad, mode="compat")
            bits, _ = O.symbols_to_bits(sym)
            mp = MacParser()
            pp = dec.protocol_parser

            def to_pdu(pd):
                pp.mcc, pp.mnc, pp.colour_code = mp.mcc, mp.mnc, mp.colour_code
                return None if pd is None else MacPDU(
                    pdu_type=PDUType(pd["pdu_type"]), encrypted=pd["encrypted"], address=pd["address"],
                    length=pd["length"], data=bytes(pd["data"]), fill_bits=pd["fill_bits"],
                    encryption_mode=pd["encryption_mode"], reassembled_data=pd["reassembled_data"])

            # the decryption re-parses decrypted payloads (decoder.py:760-766) through the parser's
            # hot-path methods, which are device calls: the same CPU stand-ins, on the one MAC state
            pp.parse_mac_pdu = lambda b: to_pdu(mp.parse(b))
            pp._check_crc = lambda b: bool(O.check_crc(np.asarray(b)))
            kept = []
            for f in O.decode_frames(sym):
                if f["nbits"] < 510:
                    continue
                fb = np.asarray(bits[f["start"]:f["start"] + 510]).astype(np.int64)
                frame = dec._frame_dict(fb, 0, f["number"])
                crc = bool(f["crc_ok"])
                dec.protocol_parser.count_burst(crc)
                burst = TetraBurst(burst_type=BurstType(f["burst_type"]), slot_number=f["number"] % 4, frame_number=0,
                                   training_sequence=np.asarray(f["ts"]), data_bits=np.asarray(f["data"]), crc_ok=crc)
                frame["burst_crc"] = crc
                frame = dec._mac_stage(frame, burst, to_pdu(mp.parse(f["data"])))
                if frame:
                    kept.append(jsonable(frame))
            res.append(kept)
        out[f"frames_{ad}"] = res
    json.dump(out, open(path, "w"))


if __name__ == "__main__":
    {"reference": reference, "overlay": overlay}[sys.argv[1]](sys.argv[2])
