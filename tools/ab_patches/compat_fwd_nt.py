# bit-identical variant: k_sos_fwd_bank's scratch stores with the nontemporal hint
import sys
s = sys.stdin.read()
a = "                if (own) *reinterpret_cast<float4 *>(sp + (t0 + u - 18 + 4 * sec)) = float4{w[0], w[1], w[2], w[3]};"
assert s.count(a) == 1
b = ("                if (own) {   // nt variant\n"
     "                    typedef float f4v __attribute__((ext_vector_type(4)));\n"
     "                    __builtin_nontemporal_store(f4v{w[0], w[1], w[2], w[3]}, reinterpret_cast<f4v *>(sp + (t0 + u - 18 + 4 * sec)));\n"
     "                }")
sys.stdout.write(s.replace(a, b))
