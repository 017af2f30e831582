"""ctypes binding of libtetra_hip.so (include/tetra_hip.h).

This is the only way the Python surface reaches compute: every numeric method of
SignalProcessor / TetraDecoder / TetraProtocolParser calls an entry point here.  There is no CPU
fallback: if the library or a gfx950 device is missing, ``ctx()`` raises ``TetraHipError``.
"""
import ctypes
import os
import threading

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TETRA_HIP_LIB", os.path.join(os.path.dirname(_PKG), "lib", "libtetra_hip.so"))

TETRA_CF32, TETRA_CF64, TETRA_SC16 = 0, 1, 2
TETRA_F32, TETRA_F64 = 3, 4   # real samples: tetra_demod_dqpsk only
MAX_SYNC = 16
F_POS, F_START, F_VALID, F_NBITS, F_NUMBER, F_BTYPE, F_CRC, F_HDR, F_FIELDS = range(9)
(MAC_STATUS, MAC_PTYPE, MAC_MODE, MAC_FILL, MAC_ADDR, MAC_LENGTH, MAC_DATA_BITS, MAC_SYSINFO, MAC_MCC, MAC_MNC,
 MAC_CC) = range(11)
MAC_FIELDS = 12


class TetraHipError(RuntimeError):
    pass


class CompatPlan(ctypes.Structure):
    """Mirror of struct tetra_compat_plan (include/tetra_hip.h)."""
    _fields_ = [
        ("q", ctypes.c_int32), ("dec_f64", ctypes.c_int32), ("filt", ctypes.c_int32),
        ("ntaps", ctypes.c_int32), ("sps", ctypes.c_int32), ("phase_step", ctypes.c_int32),
        ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32), ("fs_dec", ctypes.c_double),
        ("sos_f32", ctypes.c_float * 24), ("zi_f32", ctypes.c_float * 8),
        ("sos_f64", ctypes.c_double * 24), ("zi_f64", ctypes.c_double * 8),
        ("b", ctypes.c_double * 8), ("a", ctypes.c_double * 8), ("lzi", ctypes.c_double * 8),
        ("thr", ctypes.c_double * 4),
    ]


COMPAT_SEQUENTIAL, COMPAT_BLOCKED = 1, 2   # tetra_compat_plan.flags: 0 = sequential (scipy-exact), 2 = latency mode
FORM_DEC_BLOCKED, FORM_LF_BLOCKED, FORM_POW_PREPASS = 1, 2, 4   # tetra_compat_forms bits
ETSI_FORCE_GENERIC = 1   # tetra_etsi_plan.flags: run a canonical plan on the generic-rate kernel


class EtsiPlan(ctypes.Structure):
    """Mirror of struct tetra_etsi_plan (include/tetra_hip.h)."""
    _fields_ = [
        ("q1", ctypes.c_int32), ("L1", ctypes.c_int32), ("Lp", ctypes.c_int32), ("up", ctypes.c_int32),
        ("down", ctypes.c_int32), ("gain", ctypes.c_float), ("soft_scale", ctypes.c_float),
        ("flags", ctypes.c_int32), ("h1", ctypes.c_float * 64), ("hp", ctypes.c_float * 4096),
    ]


class WbPlan(ctypes.Structure):
    """Mirror of struct tetra_wb_plan (include/tetra_hip.h); h and g point at arrays the owner keeps."""
    _fields_ = [
        ("M", ctypes.c_int32), ("D", ctypes.c_int32), ("P", ctypes.c_int32), ("up", ctypes.c_int32),
        ("down", ctypes.c_int32), ("Lg", ctypes.c_int32), ("fs", ctypes.c_double),
        ("h", ctypes.POINTER(ctypes.c_float)), ("g", ctypes.POINTER(ctypes.c_float)),
    ]


ETSI_MAXB, ETSI_MAXJ = 8, 16
ETSI_RESERVE, ETSI_MARGIN = 256, 8   # streaming rows: dibits ahead of a chunk's; window re-computed outputs
# struct tetra_etsi_track (include/tetra_hip.h): one channel's carried timing loop
ETSI_TRACK = __import__("numpy").dtype([("base", "<f4"), ("delta", "<f4"), ("prev_re", "<f4"), ("prev_im", "<f4"),
                                       ("acquired", "<i4"), ("reserved", "<i4", (3,))])

_lib = None
_lib_lock = threading.Lock()
_tls = threading.local()

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i32 = ctypes.c_int
_i32p = ctypes.POINTER(ctypes.c_int32)
_dp = ctypes.POINTER(ctypes.c_double)


def _bind(L):
    sig = {
        "tetra_abi_version": (_i32, []),
        "tetra_create": (_vp, [_i32]),
        "tetra_destroy": (None, [_vp]),
        "tetra_last_error": (ctypes.c_char_p, [_vp]),
        "tetra_get_stream": (_vp, [_vp]),
        "tetra_set_stream": (_i32, [_vp, _vp]),
        "tetra_synchronize": (_i32, [_vp]),
        "tetra_device_arch": (_i32, [_vp, ctypes.c_char_p, _sz]),
        "tetra_profile": (_i32, [_vp, _i32]),
        "tetra_profile_read": (_i32, [_vp, ctypes.c_char_p, _sz, _vp, _vp, _i32, _i32p]),
        "tetra_compat_symbols": (ctypes.c_int64, [ctypes.POINTER(CompatPlan), _sz]),
        "tetra_compat_blocked_table": (_i32, [ctypes.POINTER(CompatPlan), _i32, _vp]),
        "tetra_compat_forms": (_i32, [ctypes.POINTER(CompatPlan), _sz, _sz, _i32p]),
        "tetra_demod_compat": (_i32, [_vp, ctypes.POINTER(CompatPlan), _vp, _i32, _sz, _sz, _vp, _vp, _vp, _vp, _vp,
                                      _sz, _i32p]),
        "tetra_decimate": (_i32, [_vp, ctypes.POINTER(CompatPlan), _vp, _i32, _sz, _sz, _vp]),
        "tetra_frequency_shift": (_i32, [_vp, _vp, _i32, _sz, _sz, _vp, ctypes.c_double, _vp]),
        "tetra_filtfilt": (_i32, [_vp, ctypes.POINTER(CompatPlan), _vp, _i32, _sz, _sz, _vp]),
        "tetra_extract_symbols": (_i32, [_vp, _vp, _i32, _sz, _sz, _i32, _i32, _vp, _vp, _vp, _sz]),
        "tetra_demod_dqpsk": (_i32, [_vp, _vp, _i32, _sz, _sz, _vp, _vp]),
        "tetra_lmac_compat": (_i32, [_vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp]),
        "tetra_symbols_to_bits": (_i32, [_vp, _vp, _sz, _vp, _vp]),
        "tetra_find_sync": (_i32, [_vp, _vp, _sz, _i32, _vp, _i32, _i32p, _i32p]),
        "tetra_match_count": (_i32, [_vp, _vp, _sz, _sz, _vp, _sz, _vp]),
        "tetra_parse_bursts": (_i32, [_vp, _vp, _sz, _vp, _vp, _vp]),
        "tetra_crc16": (_i32, [_vp, _vp, _sz, _sz, _i32, _vp]),
        "tetra_check_crc": (_i32, [_vp, _vp, _sz, _sz, _vp]),
        "tetra_mac_headers": (_i32, [_vp, _vp, _vp, _sz, _sz, _vp, _vp, _sz]),
        "tetra_etsi_lengths": (_i32, [ctypes.POINTER(EtsiPlan), _sz, _vp, _vp, _vp]),
        "tetra_etsi_chanfilt": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _sz, _sz, _vp]),
        "tetra_etsi_timing": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _sz, _sz, _vp, _vp, _vp, _vp, _sz, _vp]),
        "tetra_etsi_timing_om": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _sz, _sz, _vp, _sz, _sz, ctypes.c_int, _vp,
                                        _vp, _vp, _vp, _sz, _vp]),
        "tetra_etsi_timing_chunks": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _sz, _sz, _sz, _sz, _sz, _vp, _sz,
                                            ctypes.c_int, _vp, _vp, _vp, _vp, _sz, _vp]),
        "tetra_demod_etsi":(_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _sz, _sz, _vp, _vp, _vp, _vp, _sz, _vp]),
        "tetra_etsi_chanfilt_fmt": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _i32, _sz, _sz, _vp]),
        "tetra_demod_etsi_fmt": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _i32, _sz, _sz, _vp, _vp, _vp, _vp, _sz,
                                        _vp]),
        "tetra_etsi_set_cells": (_i32, [_vp, _vp, _sz]),
        "tetra_etsi_decide": (_i32, [_vp, _vp, _i32, _sz, _vp]),
        "tetra_etsi_kernel_info": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _i32, _sz, _i32, ctypes.c_char_p, _sz, _vp]),
        "tetra_lmac_etsi": (_i32, [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp]),
        "tetra_lmac_etsi_acquire": (_i32, [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
        "tetra_etsi_stream_window": (_i32, [ctypes.POINTER(EtsiPlan), ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            _vp, _vp, _vp, _vp]),
        "tetra_demod_etsi_stream": (_i32, [_vp, ctypes.POINTER(EtsiPlan), _vp, _i32, _sz, _sz, _sz, ctypes.c_int,
                                           _vp, _vp, _vp, _vp, _vp, _sz, _sz, _vp]),
        "tetra_lmac_etsi_stream": (_i32, [_vp, _vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
        "tetra_etsi_mix": (_i32, [_vp, _vp, _sz, _sz, _sz, _vp, ctypes.c_double, ctypes.c_int64, _vp]),
        "tetra_etsi_decode_blocks": (_i32, [_vp, _vp, _sz, _i32, _vp, _vp, _vp]),
        "tetra_etsi_encode_blocks": (_i32, [_vp, _vp, _sz, _i32, _vp, _vp]),
        "tetra_wb_lengths": (_i32, [ctypes.POINTER(WbPlan), _sz, _vp, _vp]),
        "tetra_read_floor": (_i32, [_vp, _vp, _sz, _sz, _sz]),
        "tetra_mark": (_i32, [_vp, _i32]),
        "tetra_resample": (_i32, [_vp, _vp, _i32, _sz, _sz, _sz, _vp]),
        "tetra_waterfall": (_i32, [_vp, _vp, _i32, _sz, _sz, _sz, _sz, _sz, _vp]),
        "tetra_afc_gate": (_i32, [_vp, _vp, _i32, _sz, _sz, ctypes.c_double, _vp, _vp, _vp, _vp]),
        "tetra_scan_detect": (_i32, [_vp, _vp, _i32, _sz, _sz, _i32, ctypes.c_uint32, _vp]),
        "tetra_channelize": (_i32, [_vp, ctypes.POINTER(WbPlan), _vp, _sz, _vp, _sz]),
        "tetra_channelize_om": (_i32, [_vp, ctypes.POINTER(WbPlan), _vp, _sz, _vp, _sz, _vp]),
        "tetra_synth_wideband": (_i32, [_vp, ctypes.POINTER(WbPlan), _sz, ctypes.c_uint64, ctypes.c_float,
                                        ctypes.c_float, _vp, _vp, _vp, _vp, _vp]),
        "tetra_synth_bursts_per_channel": (_i32, [_sz, ctypes.c_double]),
        "tetra_synth_etsi": (_i32, [_vp, _sz, _sz, ctypes.c_double, ctypes.c_uint64, ctypes.c_float, ctypes.c_float,
                                    _vp, _vp, _vp, _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load libtetra_hip.so (raises TetraHipError when it is missing -- no fallback)."""
    global _lib
    if _lib is None:
        with _lib_lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise TetraHipError(f"libtetra_hip.so not found at {LIB_PATH}: build it with "
                                        f"`make -C tetraear-bladerf_amd` (no CPU fallback exists)")
                # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same SONAME as
                # /opt/rocm's).  Whichever loads first serves both, and torch only initialises on
                # its own build, so let torch load it before this library binds to it.
                try:
                    import torch  # noqa: F401
                except ImportError:
                    pass
                _lib = _bind(ctypes.CDLL(LIB_PATH))
    return _lib


class Context:
    """One HIP context (device + stream) per host thread, as the C ABI requires."""

    def __init__(self, device=None):
        if device is None:
            device = int(os.environ.get("TETRA_HIP_DEVICE", "0"))
        self.lib = lib()
        self.handle = self.lib.tetra_create(device)
        if not self.handle:
            raise TetraHipError("tetra_create failed: " + (self.lib.tetra_last_error(None) or b"").decode())
        self.device = device

    def check(self, rc, what=""):
        if rc != 0:
            msg = (self.lib.tetra_last_error(self.handle) or b"").decode()
            raise TetraHipError(f"{what} failed (rc={rc}): {msg}")

    def arch(self):
        buf = ctypes.create_string_buffer(64)
        self.check(self.lib.tetra_device_arch(self.handle, buf, 64), "tetra_device_arch")
        return buf.value.decode()

    def synchronize(self):
        self.check(self.lib.tetra_synchronize(self.handle), "tetra_synchronize")

    def __del__(self):
        try:
            if self.handle:
                self.lib.tetra_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def ctx():
    """The calling thread's default context.  It runs on the null stream, so its work is ordered with
    torch's default stream: device tensors torch just made are complete before its kernels read them,
    and torch's ops see its results (a context of its own -- Context() -- keeps a non-blocking stream
    of its own, for callers that order their streams themselves, as bench.py and the pipelines do)."""
    c = getattr(_tls, "ctx", None)
    if c is None:
        c = Context()
        c.check(c.lib.tetra_set_stream(c.handle, None), "tetra_set_stream")
        _tls.ctx = c
    return c


def ptr(a):
    """Address of a C-contiguous numpy array (or a torch tensor's data_ptr)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libtetra_hip must be C-contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)
