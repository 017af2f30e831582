# k_chanfilt_r reading only 16 distinct channels' input (L2/MALL-resident): its compute-bound time (timing only)
import sys
s = sys.stdin.read()
a = "    const uint8_t *xp = reinterpret_cast<const uint8_t *>(iq) + ((size_t)ch * N + s0) * BPS;"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "    const uint8_t *xp = reinterpret_cast<const uint8_t *>(iq) + ((size_t)(ch & 15) * N + s0) * BPS;"))
