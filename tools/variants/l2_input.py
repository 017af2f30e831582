# k_chanfilt_w reading only 16 distinct channels' input (ch & 15: L2/MALL-resident after the first
# round) -- the kernel's compute/latency-bound time without the HBM stream (timing only)
import sys
s = sys.stdin.read()
a = "    const float4 *xp = iq + (size_t)ch * (N / 2) + 5L * K0;"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "    const float4 *xp = iq + (size_t)(ch & 15) * (N / 2) + 5L * K0;"))
