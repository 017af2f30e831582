# k_chanfilt_r with each lane loading its own 10-sample block from memory (five 8-B loads, no LDS
# image, no halo copy) instead of the shared image
import sys
s = sys.stdin.read()
a = "constexpr bool R_DIRECT = false;"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, "constexpr bool R_DIRECT = true;"))
