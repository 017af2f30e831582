# timing only: the fused tail's interpolation window reads from LDS replaced by register values
# (prices the LDS round trip + cubic on the tracking chain)
import sys
s = sys.stdin.read()
a = "            interp_pair(y, 0, t, a, b);\n"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "            a = make_float2(t, -t); b = make_float2(off, t * t);   // timing variant\n"))
