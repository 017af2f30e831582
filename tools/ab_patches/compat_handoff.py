# bit-identical variant (measured, not kept: profiles/r05_ab_compat_handoff_*.txt): the banked
# decimator's per-tick hand-off split so the recursion's chain carries one DPP move -- the bank-0
# sample moves (row_shl:4J, bank_mask 0x1) for a whole batch first, then per tick one row_shr:4
# under bank_mask 0xE keeps them in bank 0.  Removes every s_nop from the loops; serial passes
# -0.6 % / -3 %, but the pipelined compat step is slower (8.23-9.68 against 8.00-8.01 ms).
import sys
s = sys.stdin.read()
anchor = "__device__ __forceinline__ float from_left_bank(float y) { return dppf<0x114, 0xf, true>(0.f, y); }   // row_shr:4\n"
assert s.count(anchor) == 1
s = s.replace(anchor, anchor + """template <int J>
__device__ __forceinline__ float bank0_take(float e) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, e), J == 0 ? 0xE4 : 0x100 + 4 * J,
                                                              0xf, 0x1, false));
}
__device__ __forceinline__ float bank_input(float pre, float y) { return dppf<0x114, 0xE, false>(pre, y); }
""")
a = """        float o[16];
#pragma unroll
        for (int u = 0; u < SKB; ++u) {
            const f4u &pv = v[u >> 3];
            const float e = (u & 1) ? pv.z : pv.x;
            const float left = from_left_bank(y);
            float xin;
            switch ((u >> 1) & 3) {
                case 0: xin = bank0_from<0>(left, e); break;
                case 1: xin = bank0_from<1>(left, e); break;
                case 2: xin = bank0_from<2>(left, e); break;
                default: xin = bank0_from<3>(left, e); break;
            }
            y = bq.step(xin);"""
b = """        float o[16];
        float pre[SKB];
#pragma unroll
        for (int u = 0; u < SKB; ++u) {
            const f4u &pv = v[u >> 3];
            const float e = (u & 1) ? pv.z : pv.x;
            switch ((u >> 1) & 3) {
                case 0: pre[u] = bank0_take<0>(e); break;
                case 1: pre[u] = bank0_take<1>(e); break;
                case 2: pre[u] = bank0_take<2>(e); break;
                default: pre[u] = bank0_take<3>(e); break;
            }
        }
#pragma unroll
        for (int u = 0; u < SKB; ++u) asm volatile("" : "+v"(pre[u]));
#pragma unroll
        for (int u = 0; u < SKB; ++u) {
            y = bq.step(bank_input(pre[u], y));"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """            const long tq0 = tcur(t0 + PH) / QT;   // wave-uniform: output index of tick PH
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const float4 &pv = v[u >> 4];
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
                y = bq.step(xin);"""
b = """            const long tq0 = tcur(t0 + PH) / QT;   // wave-uniform: output index of tick PH
            float pre[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const float4 &pv = v[u >> 4];
                const int el = 3 - (u & 3);
                const float e = el == 3 ? pv.w : el == 2 ? pv.z : el == 1 ? pv.y : pv.x;
                switch ((u >> 2) & 3) {
                    case 0: pre[u] = bank0_take<0>(e); break;
                    case 1: pre[u] = bank0_take<1>(e); break;
                    case 2: pre[u] = bank0_take<2>(e); break;
                    default: pre[u] = bank0_take<3>(e); break;
                }
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) asm volatile("" : "+v"(pre[u]));
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                y = bq.step(bank_input(pre[u], y));"""
assert s.count(a) == 1
s = s.replace(a, b)
sys.stdout.write(s)
