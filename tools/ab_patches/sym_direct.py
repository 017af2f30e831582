# Fused demod tail: the tracking loop stores each block's symbols straight to global memory (one
# 512-B store per block, off the loop's chain) instead of staging them in LDS for the final copy-out,
# which then moves only the soft bits and hard dibits (3 B instead of 11 B per symbol).
import sys
s = sys.stdin.read()
def sub(a, b):
    global s
    assert s.count(a) == 1, (a, s.count(a))
    s = s.replace(a, b)
sub("const TrackOut o = timing_track<true>(ly, M2, to.gain, to.soft_scale, stage ? stage->sym : to.sym + so, scr,",
    "const TrackOut o = timing_track<true>(ly, M2, to.gain, to.soft_scale, to.sym + so, scr,")
sub("    copy_out(reinterpret_cast<uint8_t *>(to.sym + so), reinterpret_cast<const uint8_t *>(stage->sym), 8 * o.S, tid);\n", "")
sys.stdout.write(s)
