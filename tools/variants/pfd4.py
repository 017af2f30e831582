# k_chanfilt_w with four input tiles in flight per wave (pa / pb / pc / pd) instead of three
import sys
s = sys.stdin.read()
s = s.replace("constexpr int PFDW = 3;", "constexpr int PFDW = 4;").replace('static_assert(PFDW == 3, "pa / pb / pc below");', "")
old = """    float4 pa[5], pb[5], pc[5];
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
new = """    float4 pa[5], pb[5], pc[5], pd[5];
    if (ntile > 0) {
        load_tile(pa, 0);
        load_tile(pb, 1);
        load_tile(pc, 2);
        load_tile(pd, 3);
    }
    int t = 0;
    for (; t + 3 < ntile; t += 4) {
        tile(t, pa);
        tile(t + 1, pb);
        tile(t + 2, pc);
        tile(t + 3, pd);
    }
    if (t < ntile) tile(t, pa);
    if (t + 1 < ntile) tile(t + 1, pb);
    if (t + 2 < ntile) tile(t + 2, pc);
"""
assert s.count(old) == 1
sys.stdout.write(s.replace(old, new))
