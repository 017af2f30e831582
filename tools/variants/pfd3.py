# k_chanfilt_w with three input tiles in flight per wave (pa / pb / pc) instead of two
import sys
s = sys.stdin.read()
k = s.index("void k_chanfilt_w(")
head, body = s[:k], s[k:]
a = "        load_tile(pf, t + PFD);\n"
assert body.count(a) == 1
body = body.replace(a, "        load_tile(pf, t + 3);\n")
old = """    static_assert(PFD == 2, "pa / pb below");
    float4 pa[5], pb[5];
    if (ntile > 0) {
        load_tile(pa, 0);
        load_tile(pb, 1);
    }
    int t = 0;
    for (; t + 1 < ntile; t += 2) {
        tile(t, pa);
        tile(t + 1, pb);
    }
    if (t < ntile) tile(t, pa);
"""
new = """    float4 pa[5], pb[5], pc[5];
    if (ntile > 0) {
        load_tile(pa, 0);
        load_tile(pb, 1);
        load_tile(pc, 2);
    }
    int t = 0;
    for (; t + 2 < ntile; t += 3) {
        tile(t, pa);
        tile(t + 1, pb);
        tile(t + 2, pc);
    }
    if (t < ntile) tile(t, pa);
    if (t + 1 < ntile) tile(t + 1, pb);
"""
assert body.count(old) == 1
sys.stdout.write(head + body.replace(old, new))
