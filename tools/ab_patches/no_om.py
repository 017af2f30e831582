# the fused per-wave tail without the Oerder-Meyr sums (timing only)
import sys
s = sys.stdin.read()
a = "    if (om && M2 >= 16) om[tid] = om_part(ly, M2, tid >> 6, tid & 63);"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "    if (om && M2 >= 16) om[tid] = 1.0f + (float)(tid & 3);   // timing variant"))
