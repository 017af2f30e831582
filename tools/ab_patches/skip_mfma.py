# the per-wave demod's stage-2 bursts without their 39-step MFMA chain (operand reads and stores kept): timing only
import sys
s = sys.stdin.read()
a = "            for (int s2 = 13 * s3; s2 < 13 * s3 + 13; ++s2)\n                c = __builtin_amdgcn_mfma_f32_16x16x4f32(at[s2], bv[s2], c, 0, 0, 0);"
assert a in s
sys.stdout.write(s.replace(a, "            for (int s2 = 13 * s3; s2 < 13 * s3 + 13; ++s2)\n                c[s2 & 3] += bv[s2] * at[s2];"))
