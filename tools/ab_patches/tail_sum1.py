# timing only: the block's two 64-lane sums cut to one DPP level (prices wave_sum2 on the chain)
import sys
s = sys.stdin.read()
a = "            wave_sum2(E, W);\n            if (W > 0.0f) delta"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "            E = E + dppf<0xB1>(E);\n            W = W + dppf<0xB1>(W);   // timing variant\n            if (W > 0.0f) delta"))
