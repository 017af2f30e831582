# timing only: the Gardner update's IEEE division E / W replaced by a multiply (prices the division
# on the tracking chain; delta is then garbage, clamped to +-1.5)
import sys
s = sys.stdin.read()
a = "            if (W > 0.0f) delta = delta - gain * (E / W);"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "            if (W > 0.0f) delta = delta - gain * (E * W);   // timing variant"))
