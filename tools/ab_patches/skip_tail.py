# the fused per-wave demod without its timing tail (tracking, decisions, output copy): timing only
import sys
s = sys.stdin.read()
a = "        timing_tail(reinterpret_cast<const float2 *>(yb), reinterpret_cast<float2 *>(R), to, M2, ch, tid, tro, prog,"
assert a in s
sys.stdout.write(s.replace(a, "        if (M2 < 0) timing_tail(reinterpret_cast<const float2 *>(yb), reinterpret_cast<float2 *>(R), to, M2, ch, tid, tro, prog,"))
