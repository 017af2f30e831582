"""Timing-only (wrong y): k_pfb_resamp_fix with each packed FMA replaced by a packed add of the row (no tap
read from LDS, the same count of VALU ops) -- prices the tap reads and the moves that pair them.  Applies to
csrc/wideband.hip (tools/ab.sh build NAME tools/ab_patches/resamp_no_taps.py wideband)."""
import sys

s = sys.stdin.read()
old = """                        const float w = tapL[use.idx[i][o]];
                        acc[o] = __builtin_elementwise_fma(pf2{w, w}, vv, acc[o]);   // = fmaf per component"""
new = """                        acc[o] = acc[o] + vv;"""
assert old in s, "resamp_no_taps: the FMA lines moved"
sys.stdout.write(s.replace(old, new))
