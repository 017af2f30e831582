# timing only: the banked decimator passes load every batch from the row's first window (L2 hits,
# no HBM stream; outputs wrong) -- prices the input stream of k_sos_fwd_bank / k_sos_bwd_bank
import sys
s = sys.stdin.read()
a = "        for (int k = 0; k < NW; ++k) v[k] = *reinterpret_cast<const f4u *>(src + 16 * k);"
b = "            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const float4 *>(sw - t0 - 16 * k);"
assert s.count(a) == 1 and s.count(b) == 1
s = s.replace(a, "        for (int k = 0; k < NW; ++k) v[k] = *reinterpret_cast<const f4u *>(xw + 16 * k);   // timing variant")
s = s.replace(b, "            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const float4 *>(sw - 16 * k);   // timing variant")
sys.stdout.write(s)
