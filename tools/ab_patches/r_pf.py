# k_chanfilt_r's SC16 prefetch depth from env RPF (timing)
import os
import sys
s = sys.stdin.read()
a = "struct RCfg<uint4> { static constexpr int bps = 4, pf = 4; }"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "struct RCfg<uint4> { static constexpr int bps = 4, pf = %d; }" % int(os.environ["RPF"])))
