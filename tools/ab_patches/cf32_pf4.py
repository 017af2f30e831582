# cf32 k_chanfilt_r with four input tiles in flight per wave instead of three (bit-identical)
import sys
s = sys.stdin.read()
a = "template <> struct RCfg<float4> { static constexpr int bps = 8, pf = 3, nb = 1, wlr = WLR; };"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, a.replace("pf = 3", "pf = 4")))
