# bit-identical candidate: the banked decimator's section-0 lanes load every sample of their stream
# themselves (exec-masked to bank 0), so a tick is ONE DPP move -- row_shr:4 under bank_mask 0xE,
# bank 0 keeping its own sample as the move's old value -- instead of two (row_shr:4, then the
# bank-0 sample from bank j with row_shl:4j).  Costs 4x the load instructions on a quarter of the
# lanes (the same bytes).  Applies to compat_demod.hip.
import sys
s = sys.stdin.read()


def sub(a, b):
    global s
    assert s.count(a) == 1, a[:80]
    s = s.replace(a, b)


# ---- forward pass: bank 0 loads floats [2 n0 + comp, +4) for every 2-sample pair of the batch
sub("""    constexpr int NW = SKB / 8;   // 8-sample windows per batch
    const float *xw = xr + 4 * sec + comp;
    auto ld = [&](f4u (&v)[NW], long t0) __attribute__((always_inline)) {
        const float *src = xw + 2 * (t0 - pad);
#pragma unroll
        for (int k = 0; k < NW; ++k) v[k] = *reinterpret_cast<const f4u *>(src + 16 * k);
    };""",
    """    constexpr int NW = SKB / 2;   // 2-sample vectors per batch (bank 0 only)
    const float *xw = xr + comp;
    auto ld = [&](f4u (&v)[NW], long t0) __attribute__((always_inline)) {
        if (sec == 0) {
            const float *src = xw + 2 * (t0 - pad);
#pragma unroll
            for (int k = 0; k < NW; ++k) v[k] = *reinterpret_cast<const f4u *>(src + 4 * k);
        }
    };""")
sub("""            const f4u &pv = v[u >> 3];
            const float e = (u & 1) ? pv.z : pv.x;
            const float left = from_left_bank(y);
            float xin;
            switch ((u >> 1) & 3) {
                case 0: xin = bank0_from<0>(left, e); break;
                case 1: xin = bank0_from<1>(left, e); break;
                case 2: xin = bank0_from<2>(left, e); break;
                default: xin = bank0_from<3>(left, e); break;
            }
            y = bq.step(xin);   // every section active: pad >= 3""",
    """            const f4u &pv = v[u >> 1];
            const float e = (u & 1) ? pv.z : pv.x;
            y = bq.step(dppf<0x114, 0xE, false>(e, y));   // every section active: pad >= 3""")
sub("""        for (int k = 0; k < NW; ++k) asm volatile("" ::"v"(v[k]));""",
    """        for (int k = 0; k < NW; ++k) asm volatile("" ::"v"(v[k].y), "v"(v[k].w));""")

# ---- reverse pass: bank 0 loads the 4 chunks of every 16-tick window
sub("""        const float *sw = sp + L - 4 - 4 * sec;
        auto ld = [&](float4 (&v)[NL], long t0) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < NL; ++k) v[k] = *reinterpret_cast<const float4 *>(sw - t0 - 16 * k);
        };
        auto run = [&](float4 (&v)[NL], long t0) __attribute__((always_inline)) {""",
    """        const float *sw = sp + L - 4;
        auto ld = [&](float4 (&v)[4 * NL], long t0) __attribute__((always_inline)) {
            if (sec == 0) {
#pragma unroll
                for (int k = 0; k < 4 * NL; ++k) v[k] = *reinterpret_cast<const float4 *>(sw - t0 - 4 * k);
            }
        };
        auto run = [&](float4 (&v)[4 * NL], long t0) __attribute__((always_inline)) {""")
sub("""                const float4 &pv = v[u >> 4];
                const int el = 3 - (u & 3);
                const float e = el == 3 ? pv.w : el == 2 ? pv.z : el == 1 ? pv.y : pv.x;
                const float left = from_left_bank(y);
                float xin;
                switch ((u >> 2) & 3) {
                    case 0: xin = bank0_from<0>(left, e); break;
                    case 1: xin = bank0_from<1>(left, e); break;
                    case 2: xin = bank0_from<2>(left, e); break;
                    default: xin = bank0_from<3>(left, e); break;
                }
                y = bq.step(xin);""",
    """                const float4 &pv = v[u >> 2];
                const int el = 3 - (u & 3);
                const float e = el == 3 ? pv.w : el == 2 ? pv.z : el == 1 ? pv.y : pv.x;
                y = bq.step(dppf<0x114, 0xE, false>(e, y));""")
sub("""            float4 xs[SOS_PD][NL];""", """            float4 xs[SOS_PD][4 * NL];""")
import os
if os.environ.get("BANK0_SPLIT"):
    # split each loaded vector into four independent registers (a non-volatile asm that ties each
    # element to its own output), so the DPP move can take a dead sample register as its old value
    # instead of copying it out of a live 128-bit tuple
    sub("""            const f4u &pv = v[u >> 1];
            const float e = (u & 1) ? pv.z : pv.x;""",
        """            float e;
            if ((u & 1) == 0) {
                float a, b, c, d;
                asm("" : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "0"(v[u >> 1].x), "1"(v[u >> 1].y), "2"(v[u >> 1].z), "3"(v[u >> 1].w));
                e = a;
                ez = c;
            } else {
                e = ez;
            }""")
    sub("""        float o[16];
#pragma unroll
        for (int u = 0; u < SKB; ++u) {""", """        float o[16];
        float ez = 0;
#pragma unroll
        for (int u = 0; u < SKB; ++u) {""")
    sub("""        for (int k = 0; k < NW; ++k) asm volatile("" ::"v"(v[k].y), "v"(v[k].w));""", """        for (int k = 0; k < 0; ++k) {}""")
    sub("""                const float4 &pv = v[u >> 2];
                const int el = 3 - (u & 3);
                const float e = el == 3 ? pv.w : el == 2 ? pv.z : el == 1 ? pv.y : pv.x;""",
        """                if ((u & 3) == 0)
                    asm("" : "=v"(e4[0]), "=v"(e4[1]), "=v"(e4[2]), "=v"(e4[3]) : "0"(v[u >> 2].x), "1"(v[u >> 2].y), "2"(v[u >> 2].z), "3"(v[u >> 2].w));
                const float e = e4[3 - (u & 3)];""")
    sub("""            const long tq0 = tcur(t0 + PH) / QT;   // wave-uniform: output index of tick PH
#pragma unroll""", """            const long tq0 = tcur(t0 + PH) / QT;   // wave-uniform: output index of tick PH
            float e4[4];
#pragma unroll""")
sys.stdout.write(s)
