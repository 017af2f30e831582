#!/usr/bin/env python3
"""Where the fused ETSI demod's time goes (GPU box): fused demod vs its components vs HBM floors.
usage: python tools/probe_demod.py [C] [N]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))
import torch  # noqa: E402

from tetraear import _hip  # noqa: E402
from tetraear.signal.etsi import BenchStep, lengths  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    c.check(c.lib.tetra_set_stream(c.handle, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "stream")
    s = BenchStep(c, C, N, 2.4e6, seed=1, device=dev)
    _, M2, sm = lengths(s.plan, N)
    y = torch.empty((C, M2, 2), dtype=torch.float32, device=dev)
    gb = C * N * 8 / 1e9
    res = {}
    res["fused_demod"] = timeit(lambda: s._demod(c, s.sym, s.soft, s.hard, s.nsym))
    res["chanfilt_only(y->HBM)"] = timeit(lambda: c.check(c.lib.tetra_etsi_chanfilt(
        c.handle, s.plan, _hip.ptr(s.iq), C, N, _hip.ptr(y)), "chanfilt"))
    res["timing_only"] = timeit(lambda: c.check(c.lib.tetra_etsi_timing(
        c.handle, s.plan, _hip.ptr(y), C, M2, _hip.ptr(s.sym), _hip.ptr(s.soft), _hip.ptr(s.hard), _hip.ptr(s.nsym),
        sm, None), "timing"))
    def cf_then_timing():
        c.check(c.lib.tetra_etsi_chanfilt(c.handle, s.plan, _hip.ptr(s.iq), C, N, _hip.ptr(y)), "chanfilt")
        c.check(c.lib.tetra_etsi_timing(c.handle, s.plan, _hip.ptr(y), C, M2, _hip.ptr(s.sym), _hip.ptr(s.soft),
                                        _hip.ptr(s.hard), _hip.ptr(s.nsym), sm, None), "timing")
    res["chanfilt+timing(serial)"] = timeit(cf_then_timing)
    res["fused_demod(again)"] = timeit(lambda: s._demod(c, s.sym, s.soft, s.hard, s.nsym))
    res["lmac"] = timeit(lambda: s._lmac(c, s.soft, s.hard, s.nsym))
    flat = s.iq.view(-1, 4)
    res["read_floor(sum)"] = timeit(lambda: flat.sum(dim=0))
    out = torch.empty_like(flat)
    res["copy_floor(copy_)"] = timeit(lambda: out.copy_(flat))
    for lds in (0, 40 * 1024, 72 * 1024):
        res[f"hip_read_floor(lds={lds // 1024}K)"] = timeit(lambda: c.check(c.lib.tetra_read_floor(
            c.handle, _hip.ptr(s.iq), C, N * 8, lds), "read_floor"))
    res["fused_demod(3rd)"] = timeit(lambda: s._demod(c, s.sym, s.soft, s.hard, s.nsym))
    for k, v in res.items():
        extra = f"  {gb / v:.2f} TB/s of input" if "lmac" not in k and "timing" not in k else ""
        print(f"{k:24s} {v:8.4f} ms{extra}", flush=True)


if __name__ == "__main__":
    main()
