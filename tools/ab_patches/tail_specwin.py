# candidate (bit-identical): the fused tail's Gardner loop reads the NEXT block's interpolation window
# from LDS right after this block's interpolation, at the position the current delta predicts
# (8 samples around it), so the LDS round trip overlaps the block's reductions and division.  The
# window's integer position moves by floor(off') - floor(off), normally the same for every lane:
# when it is, 0 or +-1 selects the samples from the prefetched registers (a scalar branch), anything else reads
# as before.  The cubic itself is interp_pair's, operation for operation.
import sys
s = sys.stdin.read()
a = "    float2 pre[4], pre2[4];   // RING: the next block's 256 samples in flight (RING 2: and the one after)\n"
assert s.count(a) == 1
s = s.replace(a, a + "    float2 win[8];   // SPLIT: the next block's window samples ipred - 4 .. ipred + 3, prefetched\n"
                     "    int ipred = -(1 << 30);\n")
b = """            float2 a, b;
            interp_pair(y, 0, t, a, b);
            asm volatile("" ::"v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y));   // computed here, not sunk into the branch
"""
assert s.count(b) == 1
nb = """            float2 a, b;
            {
                const float fi = floorf(t);
                const int i = (int)fi;
                const int d = i - ipred;
                const int dd = __builtin_amdgcn_readfirstlane(d);
                // float rounding of t can move one lane's floor differently: the window only when the
                // shift is the same on every lane (then a scalar branch), else direct reads
                const bool uni = __ballot(d != dd) == 0;
                float2 wv6[6];   // y[i - 3 .. i + 2]
                if (uni && (dd == 0 || dd == 1 || dd == -1)) {
#pragma unroll
                    for (int m = 0; m < 6; ++m) wv6[m] = dd == 0 ? win[m + 1] : (dd == 1 ? win[m + 2] : win[m]);
                } else {
#pragma unroll
                    for (int m = 0; m < 6; ++m) wv6[m] = y[i - 3 + m];
                }
                const float K6 = 1.0f / 6.0f;
                const float f = t - fi;
                const float fm1 = f - 1.0f, fm2 = f - 2.0f, fp1 = f + 1.0f;
                const float cm = -(f * fm1 * fm2) * K6;
                const float c0 = (fp1 * fm1 * fm2) * 0.5f;
                const float c1 = -(fp1 * f * fm2) * 0.5f;
                const float c2 = (fp1 * f * fm1) * K6;
                auto one = [&](int m0) -> float2 {   // samples m0 .. m0 + 3 of wv6 = y[j - 1 .. j + 2]
                    float r = cm * wv6[m0].x, q = cm * wv6[m0].y;
                    r = fmaf(c0, wv6[m0 + 1].x, r); q = fmaf(c0, wv6[m0 + 1].y, q);
                    r = fmaf(c1, wv6[m0 + 2].x, r); q = fmaf(c1, wv6[m0 + 2].y, q);
                    r = fmaf(c2, wv6[m0 + 3].x, r); q = fmaf(c2, wv6[m0 + 3].y, q);
                    return make_float2(r, q);
                };
                a = one(2);   // on: y[i - 1 .. i + 2]
                b = one(0);   // mid: y[i - 3 .. i]
                // the next block's window at the position the current delta predicts
                const float tn = (float)(4 * (kb + 64 + lane)) + off;
                ipred = (int)floorf(tn);
#pragma unroll
                for (int m = 0; m < 8; ++m) win[m] = y[ipred - 4 + m];
            }
            asm volatile("" ::"v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y));   // computed here, not sunk into the branch
"""
s = s.replace(b, nb)
sys.stdout.write(s)
