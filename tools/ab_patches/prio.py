# k_chanfilt_r's waves at wave priority PRIO (env) from their start, so that the lower-MAC waves of
# the previous batch (priority 0) running beside them in the bench's pipeline fill issue gaps only
import os
import sys
s = sys.stdin.read()
k = s.index("void k_chanfilt_r(")
a = "    const int ch = blockIdx.x, tid = threadIdx.x, lane = tid & 63;\n"
i = s.index(a, k) + len(a)
sys.stdout.write(s[:i] + f"    __builtin_amdgcn_s_setprio({int(os.environ['PRIO'])});\n" + s[i:])
