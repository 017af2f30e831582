# first-round workgroups 256..511 start STAGGER_US microseconds late (s_memrealtime, 100 MHz), so
# the two workgroups a CU holds run out of phase (timing experiment; outputs unchanged).
# STAGGER_MODE=uniform: block b < 512 waits (b / 512) * STAGGER_US instead.
import os
import sys
s = sys.stdin.read()
k = s.index("void k_chanfilt_r(")
a = "    const int ch = blockIdx.x, tid = threadIdx.x, lane = tid & 63;\n"
i = s.index(a, k) + len(a)
us = int(os.environ["STAGGER_US"])
if os.environ.get("STAGGER_MODE", "half") == "half":
    cond, ticks = "blockIdx.x >= 256 && blockIdx.x < 512", f"{100 * us}ull"
else:
    cond, ticks = "blockIdx.x < 512", f"(unsigned long long)(blockIdx.x * {100 * us}ull / 512)"
ins = (f"    if ({cond}) {{\n"
       "        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();\n"
       f"        while (__builtin_amdgcn_s_memrealtime() - t0 < {ticks}) __builtin_amdgcn_s_sleep(8);\n"
       "    }\n")
sys.stdout.write(s[:i] + ins + s[i:])
