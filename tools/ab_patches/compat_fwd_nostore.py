# timing only: k_sos_fwd_bank computes its outputs but does not store the scratch row (prices the
# full-rate fp32 scratch write; the reverse pass then reads stale scratch)
import sys
s = sys.stdin.read()
a = "                if (own) *reinterpret_cast<float4 *>(sp + (t0 + u - 18 + 4 * sec)) = float4{w[0], w[1], w[2], w[3]};"
assert s.count(a) == 1
sys.stdout.write(s.replace(a, '                asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));   // timing variant'))
