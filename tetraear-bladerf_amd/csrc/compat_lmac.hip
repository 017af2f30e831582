// compat_lmac.hip -- TetraDecoder lower MAC on gfx950, bit-exact with the reference.
//
// Reference path:
//   symbols_to_bits          /root/reference/tetraear/core/decoder.py:140-169
//   find_sync (22-bit TS1/TS2 correlation, greedy +250 skip)     decoder.py:171-295
//   decode threshold cascade + burst slicing                      decoder.py:835-888
//   parse_burst / _detect_burst_type / _extract_* / _check_crc    protocol.py:192-329
//   _calculate_crc16 (CRC-16/CCITT-FALSE, no final XOR)           protocol.py:331-347
//
// One wave per symbol stream.  Window bits are assembled from symbols into a 24-bit register
// word per position (no bit array is materialised), so correlation is XOR + popcount.  The
// sequential greedy scan uses wave ballots: each iteration tests 64 positions and jumps to the
// first hit + 250.  Everything is integer; results are bit-exact by construction.
#include "common.h"

namespace {

constexpr uint32_t MASK22 = 0x3FFFFFu;
// TS1 / TS2 (decoder.py:197-198), LSB-first: bit j of the word = pattern[j]
__host__ __device__ constexpr uint32_t pack22(const int (&p)[22]) {
    uint32_t w = 0;
    for (int j = 0; j < 22; ++j) w |= (uint32_t)p[j] << j;
    return w;
}
constexpr int TS1[22] = {1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0};
constexpr int TS2[22] = {0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0};
// SYNC_CONTINUOUS_DOWNLINK / SYNC_DISCONTINUOUS_DOWNLINK (protocol.py:162-163)
constexpr int SCD[22] = {1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0};
constexpr int SDD[22] = {0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 0, 0, 1, 1};
constexpr uint32_t W_TS1 = pack22(TS1), W_TS2 = pack22(TS2), W_SCD = pack22(SCD), W_SDD = pack22(SDD);

// 8-PSK -> QPSK neighbour map (decoder.py:158-164)
__device__ __forceinline__ uint32_t map8(int64_t s) {
    switch (s) {
        case 0: case 1: case 2: return 0;
        case 3: case 4: return 1;
        case 5: return 3;
        case 6: case 7: return 2;
        default: return 0;
    }
}

struct Stream {
    const int64_t *s;
    long S;
    bool dq;
    __device__ uint32_t val(long k) const {   // mapped symbol (0..3)
        if (k >= S) return 0;
        const int64_t v = s[k];
        return dq ? (uint32_t)(v & 3) : map8(v);
    }
    __device__ uint32_t bit(long i) const {   // bits[i] of symbols_to_bits
        const uint32_t v = val(i >> 1);
        return (i & 1) ? (v & 1u) : (v >> 1);
    }
    // 22 bits starting at bit i, LSB-first
    __device__ uint32_t window(long i) const {
        const long k0 = i >> 1;
        uint32_t W = 0;
#pragma unroll
        for (int m = 0; m < 12; ++m) {
            const uint32_t v = val(k0 + m);
            W |= ((v >> 1) << (2 * m)) | ((v & 1u) << (2 * m + 1));
        }
        return (W >> (i & 1)) & MASK22;
    }
};

__device__ __forceinline__ int match(uint32_t w, uint32_t pat) { return 22 - __popc((w ^ pat) & MASK22); }

__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ bool stream_is_dqpsk(const int64_t *s, long S, int lane) {
    int64_t mx = INT64_MIN;
    for (long k = lane; k < S; k += 64) mx = s[k] > mx ? s[k] : mx;
    mx = wave_max_i64(mx);
    return S == 0 || mx <= 3;   // max(symbols) <= 3 (decoder.py:149-150)
}

// Greedy scan with count threshold k.  Returns number of hits (positions in pos[0..min(n,maxp))).
// *maxc (optional): max of the correlations find_sync evaluates (TS2 skipped at a TS1 hit).
template <typename SS>
__device__ int greedy(const SS &st, long nw, int k, int lane, int64_t *pos, int maxp, int *maxc) {
    int n = 0, mc = 0;
    long cur = 0;
    while (cur < nw) {
        const long i = cur + lane;
        int c1 = 0, c2 = 0;
        bool hit = false;
        if (i < nw) {
            const uint32_t w = st.window(i);
            c1 = match(w, W_TS1);
            c2 = match(w, W_TS2);
            hit = c1 >= k || c2 >= k;
        }
        const unsigned long long bal = __ballot(hit);
        long first = nw;   // first hit in this chunk, or past its end
        if (bal) first = cur + __ffsll((long long)bal) - 1;
        if (maxc && i < nw && i <= first) {
            const int ev = c1 >= k ? c1 : max(c1, c2);
            mc = max(mc, ev);
        }
        if (bal) {
            if (lane == 0 && n < maxp) pos[n] = first;
            ++n;
            cur = first + 250;   // decoder.py:256
        } else {
            cur += 64;
        }
    }
    if (maxc) *maxc = wave_max_i32(mc);
    return n;
}

__device__ __forceinline__ uint32_t crc_bit(uint32_t crc, uint32_t b) {
    crc ^= (b & 1u) << 15;
    crc = (crc & 0x8000u) ? ((crc << 1) ^ 0x1021u) : (crc << 1);
    return crc & 0xFFFFu;
}

// _check_crc over L data bits given by get(i) (protocol.py:292-329)
template <typename F>
__device__ bool check_crc(F get, long L) {
    if (L < 16) return false;
    long ones = 0;
    for (long i = 0; i < L; ++i) ones += get(i);
    if (ones == 0 || ones == L) return false;
    uint32_t rx = 0;
    for (int k = 0; k < 16; ++k) rx = (rx << 1) | get(L - 16 + k);
    uint32_t c = 0xFFFF, r = 0xFFFF;
    for (long i = 0; i < L - 16; ++i) {
        c = crc_bit(c, get(i));
        r = crc_bit(r, get(L - 17 - i));
    }
    return __popc(c ^ rx) <= 2 || __popc(r ^ rx) <= 2;
}

// parse_burst on 255 mapped symbols given by sym(t): type, and crc_ok
template <typename F>
__device__ void parse_burst(F symv, int *btype, bool *ok) {
    auto bit = [&](long i) -> uint32_t { const uint32_t v = symv(i >> 1); return (i & 1) ? (v & 1u) : (v >> 1); };
    uint32_t w = 0;
    for (int j = 0; j < 22; ++j) w |= bit(255 + j) << j;   // bits[len//2 : +22] (protocol.py:249-250)
    const int m = max(match(w, W_SCD), match(w, W_SDD));
    const bool sync = m * 5 > 88;                             // max(count)/22 > 0.8  <=>  count > 17.6
    *btype = sync ? 5 : 2;
    if (sync) {
        *ok = check_crc(bit, 510);
    } else {   // bits[0:108] ++ bits[122:230] (protocol.py:285-287)
        auto dbit = [&](long i) -> uint32_t { return bit(i < 108 ? i : i + 14); };
        *ok = check_crc(dbit, 216);
    }
}

// The CRC register as a linear function of the message bits (GF(2)): crc_bit(c, b) = S(c) ^ b S(0x8000)
// with S the shift-and-reduce step, so after n bits m_0..m_{n-1} from 0xFFFF the register is
// init[n] ^ XOR over the 1-bits m_i of t[n - 1 - i], t[d] = S^(d+1)(0x8000), init[n] = S^n(0xFFFF).
// That lets a wave check a burst's CRC in parallel (k_lmac: 64 lanes, eight bits each) instead of
// one lane stepping 494 bits twice -- the same registers, so the same decisions.
constexpr int LCRC_N = 494;   // the longest message _check_crc sees: 510 - 16 bits
struct LinCrc {
    uint32_t t[LCRC_N];
    uint32_t init[LCRC_N + 1];
};
constexpr uint32_t crc_shift(uint32_t c) { return ((c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1)) & 0xFFFFu; }
constexpr LinCrc make_lin_crc() {
    LinCrc l{};
    uint32_t r = crc_shift(0x8000u);
    for (int d = 0; d < LCRC_N; ++d) { l.t[d] = r; r = crc_shift(r); }
    uint32_t s = 0xFFFFu;
    for (int n = 0; n <= LCRC_N; ++n) { l.init[n] = s; s = crc_shift(s); }
    return l;
}
__constant__ LinCrc LCRC = make_lin_crc();

__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_add_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// check_crc (protocol.py:292-329) by a whole wave, L <= LCRC_N + 16 (every lane calls it): lane l
// takes bits l, l + 64, ...; the forward register sums t[n-1-i], the reversed one (bit L-17-i fed
// at step i) t[i], both from init[n], n = L - 16; rx gathers the last 16 bits MSB first.
template <typename F>
__device__ bool check_crc_wave(F get, int L, int lane) {
    if (L < 16) return false;
    const int n = L - 16;
    uint32_t ones = 0, c = 0, r = 0, rx = 0;
    for (int i = lane; i < L; i += 64) {
        const uint32_t b = get(i);
        ones += b;
        if (i < n) {
            const uint32_t m = 0u - b;
            c ^= LCRC.t[n - 1 - i] & m;
            r ^= LCRC.t[i] & m;
        } else {
            rx |= b << (L - 1 - i);
        }
    }
    ones = wave_add_u32(ones);
    c = wave_xor_u32(c) ^ LCRC.init[n];
    r = wave_xor_u32(r) ^ LCRC.init[n];
    rx = wave_or_u32(rx);
    if (ones == 0 || ones == (uint32_t)L) return false;
    return __popc(c ^ rx) <= 2 || __popc(r ^ rx) <= 2;
}

// parse_burst by a whole wave (the result is wave-uniform): the sync word's 22 bits by a ballot
template <typename F>
__device__ void parse_burst_wave(F symv, int lane, int *btype, bool *ok) {
    auto bit = [&](long i) -> uint32_t { const uint32_t v = symv(i >> 1); return (i & 1) ? (v & 1u) : (v >> 1); };
    const uint32_t w = (uint32_t)__ballot(lane < 22 && bit(255 + lane)) & MASK22;   // bits[255 : 277]
    const int m = max(match(w, W_SCD), match(w, W_SDD));
    const bool sync = m * 5 > 88;
    *btype = sync ? 5 : 2;
    if (sync) {
        *ok = check_crc_wave(bit, 510, lane);
    } else {
        *ok = check_crc_wave([&](long i) -> uint32_t { return bit(i < 108 ? i : i + 14); }, 216, lane);
    }
}

// The stream's bits (symbols_to_bits of the mapped symbols) packed LSB-first into LDS words, bit i
// at word i >> 5: a 22-bit window is one funnel shift of two words, where Stream::window assembled it
// from 12 global symbol loads.  Words past the stream are zero, as Stream::val is past S.
struct PackedStream {
    const uint32_t *w;
    long S;
    __device__ uint32_t bit(long i) const { return (w[i >> 5] >> (i & 31)) & 1u; }
    __device__ uint32_t val(long k) const { return (bit(2 * k) << 1) | bit(2 * k + 1); }
    __device__ uint32_t window(long i) const {
        const long q = i >> 5;
        return __builtin_amdgcn_alignbit(w[q + 1], w[q], (uint32_t)(i & 31)) & MASK22;
    }
};
// LDS words k_lmac packs a stream of up to `stride` symbols into (two past the last bit: window reads)
__host__ __device__ inline long lmac_words(long stride) { return (2 * stride + 31) / 32 + 2; }
constexpr long LMAC_LDS_MAX = 48 * 1024;   // larger rows take the global-memory Stream

// symbols_to_bits into LDS: 32 symbols per ballot (lane j: component j & 1 of symbol j >> 1, so the
// ballot is the 64 bits in stream order), eight ballots' loads issued ahead
__device__ void pack_stream(const Stream &st, uint32_t *w, long nwords, int lane) {
    for (long i = lane; i < nwords; i += 64) w[i] = 0;
    __syncthreads();
    constexpr int PK = 8;
    const int sl = lane >> 1, comp = lane & 1;
    for (long s00 = 0; s00 < st.S; s00 += 32 * PK) {
        uint32_t v[PK];
#pragma unroll
        for (int u = 0; u < PK; ++u) v[u] = st.val(s00 + 32 * u + sl);   // 0 past S
#pragma unroll
        for (int u = 0; u < PK; ++u) {
            const long s0 = s00 + 32 * u;
            if (s0 >= st.S) break;   // uniform
            const unsigned long long b = __ballot(comp ? (v[u] & 1u) : (v[u] >> 1));
            if (lane < 2) w[s0 / 16 + lane] = (uint32_t)(b >> (32 * lane));
        }
    }
    __syncthreads();
}

template <typename SS>
__device__ void lmac_body(const SS &st, int ch, int lane, long stride, const int8_t *__restrict__ kmax,
                          int32_t *__restrict__ nsync, int32_t *__restrict__ rec, uint8_t *__restrict__ fbits,
                          uint8_t *__restrict__ bbits, int64_t *pos) {
    const long nb = 2 * st.S, nw = nb - 21;
    int n = 0;
    if (nw > 0) {
        int mx = 0;
        for (long i = lane; i < nw; i += 64) {
            const uint32_t w = st.window(i);
            mx = max(mx, max(match(w, W_TS1), match(w, W_TS2)));
        }
        mx = wave_max_i32(mx);
        const int k = kmax[mx];
        if (k >= 0) n = greedy(st, nw, k, lane, pos, TETRA_MAX_SYNC, nullptr);
    }
    __syncthreads();
    if (n > TETRA_MAX_SYNC) n = TETRA_MAX_SYNC;
    if (lane == 0) nsync[ch] = n;
    int32_t *rp = rec + (size_t)ch * TETRA_MAX_SYNC * TETRA_F_FIELDS;
    uint8_t *fb = fbits + (size_t)ch * TETRA_MAX_SYNC * 510;
    uint8_t *bb = bbits + (size_t)ch * TETRA_MAX_SYNC * 510;
    for (int f = 0; f < n; ++f) {
        const long p = pos[f], start = p - 216;
        const bool valid = start >= 0 && (start >> 1) + 255 <= st.S;
        const long nbits = valid ? min((long)510, nb - start) : 0;
        const long s0 = valid ? (start >> 1) : 0;
        if (valid) {
            for (long t = lane; t < 510; t += 64) {
                fb[(size_t)f * 510 + t] = t < nbits ? (uint8_t)st.bit(start + t) : 0;
                const uint32_t v = st.val(s0 + (t >> 1));
                bb[(size_t)f * 510 + t] = (uint8_t)((t & 1) ? (v & 1u) : (v >> 1));
            }
        }
        int bt = 0;
        bool ok = false;
        int hdr = 0;
        if (valid && nbits >= 510) {   // wave-uniform
            parse_burst_wave([&](long t) { return st.val(s0 + t); }, lane, &bt, &ok);
            hdr = (int)((st.bit(start) << 3) | (st.bit(start + 1) << 2) | (st.bit(start + 2) << 1) | st.bit(start + 3));
        }
        if (lane == 0) {
            int32_t *r = rp + f * TETRA_F_FIELDS;
            r[TETRA_F_POS] = (int32_t)p;
            r[TETRA_F_START] = (int32_t)start;
            r[TETRA_F_VALID] = valid;
            r[TETRA_F_NBITS] = (int32_t)nbits;
            r[TETRA_F_NUMBER] = valid ? (int32_t)(start / 510) : -1;
            r[TETRA_F_BTYPE] = bt;
            r[TETRA_F_CRC] = ok;
            r[TETRA_F_HDR] = hdr;
        }
    }
}

__global__ __launch_bounds__(64) void k_lmac(const int64_t *__restrict__ sym, const int32_t *__restrict__ nsym,
                                             int C, long stride, const int8_t *__restrict__ kmax,
                                             int32_t *__restrict__ nsync, int32_t *__restrict__ rec,
                                             uint8_t *__restrict__ fbits, uint8_t *__restrict__ bbits) {
    const int ch = blockIdx.x, lane = threadIdx.x;
    if (ch >= C) return;   // whole workgroup (one wave)
    __shared__ int64_t pos[TETRA_MAX_SYNC];
    extern __shared__ uint32_t words[];   // lmac_words(stride) when the launch gives them
    Stream st{sym + (size_t)ch * stride, (long)nsym[ch], false};
    st.dq = stream_is_dqpsk(st.s, st.S, lane);
    const long nwords = lmac_words(stride);
    if (nwords * 4 <= LMAC_LDS_MAX && st.S <= stride) {   // (a count past the row: the global form, as before)
        pack_stream(st, words, nwords, lane);
        lmac_body(PackedStream{words, st.S}, ch, lane, stride, kmax, nsync, rec, fbits, bbits, pos);
    } else {
        lmac_body(st, ch, lane, stride, kmax, nsync, rec, fbits, bbits, pos);
    }
}

__global__ __launch_bounds__(64) void k_find_sync(const uint8_t *__restrict__ bits, long nbits, int k,
                                                  int64_t *__restrict__ pos, int maxp, int32_t *__restrict__ out2) {
    const int lane = threadIdx.x;
    // bits given directly: wrap them as a "stream" whose symbols are the bit pairs
    // bits given directly; a value other than 0/1 matches neither pattern (numpy ==)
    struct BitStream {
        const uint8_t *b;
        long n;
        __device__ void window(long i, uint32_t &w, uint32_t &inv) const {
            w = 0;
            inv = 0;
            for (int j = 0; j < 22; ++j) {
                const uint32_t v = b[i + j];
                w |= (v & 1u) << j;
                inv |= (uint32_t)(v > 1u) << j;
            }
        }
    } bs{bits, nbits};
    const long nw = nbits - 21;
    int n = 0, mc = 0;
    long cur = 0;
    while (cur < nw) {
        const long i = cur + lane;
        int c1 = 0, c2 = 0;
        bool hit = false;
        if (i < nw) {
            uint32_t w, inv;
            bs.window(i, w, inv);
            c1 = 22 - __popc(((w ^ W_TS1) | inv) & MASK22);
            c2 = 22 - __popc(((w ^ W_TS2) | inv) & MASK22);
            hit = c1 >= k || c2 >= k;
        }
        const unsigned long long bal = __ballot(hit);
        const long first = bal ? cur + __ffsll((long long)bal) - 1 : nw;
        if (i < nw && i <= first) mc = max(mc, c1 >= k ? c1 : max(c1, c2));
        if (bal) {
            if (lane == 0 && n < maxp) pos[n] = first;
            ++n;
            cur = first + 250;
        } else {
            cur += 64;
        }
    }
    mc = wave_max_i32(mc);
    if (lane == 0) { out2[0] = n; out2[1] = mc; }
}

__global__ void k_match(const uint8_t *__restrict__ bits, int F, long L, long off, const uint8_t *__restrict__ pat,
                        int32_t *__restrict__ cnt) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    const uint8_t *b = bits + (size_t)f * L + off;
    int c = 0;
    for (int j = 0; j < 22 && off + j < L; ++j) c += b[j] == pat[j];
    cnt[f] = c;
}

__global__ void k_sym2bits(const int64_t *__restrict__ sym, long S, int64_t *__restrict__ bits, int64_t *__restrict__ mapped) {
    // one block: first decide the branch, then map
    __shared__ int dq;
    const int lane = threadIdx.x;
    if (threadIdx.x < 64) {
        const bool d = stream_is_dqpsk(sym, S, lane);
        if (lane == 0) dq = d;
    }
    __syncthreads();
    Stream st{sym, S, dq != 0};
    for (long k = threadIdx.x; k < S; k += blockDim.x) {
        const uint32_t v = st.val(k);
        mapped[k] = v;
        bits[2 * k] = v >> 1;
        bits[2 * k + 1] = v & 1u;
    }
}

__global__ void k_parse_bursts(const int64_t *__restrict__ sym, int F, int32_t *__restrict__ btype,
                               uint8_t *__restrict__ ok, uint8_t *__restrict__ bits) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    const int64_t *s = sym + (size_t)f * 255;
    auto v = [&](long t) -> uint32_t { return (uint32_t)(s[t] & 3); };   // sym >> 1 & 1, sym & 1
    int bt;
    bool o;
    parse_burst(v, &bt, &o);
    btype[f] = bt;
    ok[f] = o;
    for (int t = 0; t < 510; ++t) {
        const uint32_t x = v(t >> 1);
        bits[(size_t)f * 510 + t] = (uint8_t)((t & 1) ? (x & 1u) : (x >> 1));
    }
}

__global__ void k_crc16(const uint8_t *__restrict__ bits, int F, long L, int rev, uint16_t *__restrict__ out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    const uint8_t *b = bits + (size_t)f * L;
    uint32_t c = 0xFFFF;
    for (long i = 0; i < L; ++i) c = crc_bit(c, b[rev ? L - 1 - i : i]);
    out[f] = (uint16_t)c;
}

__global__ void k_check_crc(const uint8_t *__restrict__ bits, int F, long L, uint8_t *__restrict__ out) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    const uint8_t *b = bits + (size_t)f * L;
    out[f] = check_crc([&](long i) -> uint32_t { return b[i] & 1u; }, L);
}

// parse_mac_pdu's per-frame part (protocol.py:349-596): one wave per frame; lane j packs data byte
// j (MSB first, zero-padded past the data bits), lane 0 reads the header fields.  The stateful part
// (fragment buffer, SYSINFO state, statistics) is the host's, in frame order.
__global__ __launch_bounds__(64) void k_mac_headers(const uint8_t *__restrict__ bits, const int32_t *__restrict__ nbits,
                                                    int F, long stride, int32_t *__restrict__ fields,
                                                    uint8_t *__restrict__ data, long dstride) {
    const int f = blockIdx.x, lane = threadIdx.x;
    if (f >= F) return;
    const uint8_t *b = bits + (size_t)f * stride;
    const long n = nbits[f];
    // a bit is a nonzero byte, in the header fields as in the data bytes below (BitArray semantics)
    auto bit = [&](long p) { return (int)(b[p] != 0); };
    auto uint_at = [&](long p, int w) {   // int(''.join(str(x) for x in bits[p:p+w]), 2)
        int v = 0;
        for (int i = 0; i < w; ++i) v = (v << 1) | bit(p + i);
        return v;
    };
    // header (every lane computes it: the data range below depends on it)
    int status = 1, ptype = 0, mode = 0, fill = 0, addr = -1, length = 0, sys = 0, mcc = 0, mnc = 0, cc = 0;
    long dpos = 0, dbits = 0;
    if (n >= 8) {
        const int pti = (bit(0) << 1) | bit(1);
        ptype = pti == 0 ? 0 : pti == 1 ? 1 : pti == 2 ? 3 : 2;
        mode = (bit(2) << 1) | bit(3);
        status = 0;
        if (ptype == 0 || ptype == 2) {            // RESOURCE (:399-449) / END (:506-544)
            fill = bit(4);
            long pos = 5;
            if (ptype == 0) {
                if (n < pos + 24) status = 1;
                else { addr = uint_at(pos, 24); pos += 24; }
            }
            if (status == 0 && n < pos + 6) status = 1;
            if (status == 0) {
                length = uint_at(pos, 6);
                pos += 6;
                const long dl = 8L * length;
                if (dl > n - pos + 16) status = 1;                          // :433-434, :525-526
                else { dpos = pos; dbits = (dl > 0 && n >= pos + dl) ? dl : n - pos; }
            }
        } else if (ptype == 1) {                   // FRAG (:451-469)
            fill = bit(4);
            dpos = 5;
            dbits = n - 5;
        } else {                                   // BROADCAST (:471-504)
            if (mode == 0) {
                if (n < 4 + 30) status = 1;
                else {
                    sys = 1;
                    mcc = uint_at(4, 10);
                    mnc = uint_at(14, 14);
                    cc = uint_at(28, 6);
                    if (mcc < 200 || mcc > 799 || mnc > 999) status = 2;
                }
            }
            dpos = 4;
            dbits = n - 4;
        }
    }
    if (status != 0) dbits = 0;
    uint8_t *o = data + (size_t)f * dstride;
    for (long j = lane; 8 * j < dbits; j += 64) {
        unsigned v = 0;
        for (int k = 0; k < 8; ++k) v = (v << 1) | (8 * j + k < dbits ? (b[dpos + 8 * j + k] != 0) : 0u);
        o[j] = (uint8_t)v;
    }
    if (lane == 0) {
        int32_t *r = fields + (size_t)f * TETRA_MAC_FIELDS;
        r[TETRA_MAC_STATUS] = status;
        r[TETRA_MAC_PTYPE] = ptype;
        r[TETRA_MAC_MODE] = mode;
        r[TETRA_MAC_FILL] = fill;
        r[TETRA_MAC_ADDR] = addr;
        r[TETRA_MAC_LENGTH] = length;
        r[TETRA_MAC_DATA_BITS] = (int32_t)dbits;
        r[TETRA_MAC_SYSINFO] = sys;
        r[TETRA_MAC_MCC] = mcc;
        r[TETRA_MAC_MNC] = mnc;
        r[TETRA_MAC_CC] = cc;
        r[TETRA_MAC_CC + 1] = 0;
    }
}

}  // namespace

extern "C" {

int tetra_mac_headers(tetra_ctx *ctx, const uint8_t *bits, const int32_t *nbits, size_t F, size_t stride,
                      int32_t *fields, uint8_t *data, size_t data_stride) {
    if (!ctx || (F && (!bits || !nbits || !fields || !data))) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    if (data_stride < (stride + 7) / 8) return tetra_fail(ctx, TETRA_E_INVALID, "data_stride < (stride + 7) / 8");
    std::vector<int32_t> nb(F);
    HIP_TRY(ctx, hipMemcpy(nb.data(), nbits, F * 4, hipMemcpyDefault));
    for (size_t f = 0; f < F; ++f)
        if (nb[f] < 0 || (size_t)nb[f] > stride) return tetra_fail(ctx, TETRA_E_INVALID, "nbits[%zu] outside [0, stride]", f);
    Staging st(ctx);
    const uint8_t *b = (const uint8_t *)st.in(bits, F * stride);
    const int32_t *n = (const int32_t *)st.in(nb.data(), F * 4);
    int32_t *fo = (int32_t *)st.out(fields, F * TETRA_MAC_FIELDS * 4);
    uint8_t *d = (uint8_t *)st.out(data, F * data_stride);
    if (!b || !n || !fo || !d) return st.finish();
    PROF(ctx, "mac_headers");
    hipLaunchKernelGGL(k_mac_headers, dim3((unsigned)F), dim3(64), 0, ctx->stream, b, n, (int)F, (long)stride, fo, d,
                       (long)data_stride);
    return st.finish();
}

int tetra_lmac_compat(tetra_ctx *ctx, const int64_t *sym, const int32_t *nsym, size_t C, size_t stride,
                      const int8_t *k_of_max, int32_t *nsync, int32_t *rec, uint8_t *frame_bits, uint8_t *burst_bits) {
    if (!ctx || !k_of_max) return TETRA_E_INVALID;
    if (C == 0) return TETRA_OK;
    Staging st(ctx);
    const int64_t *s = (const int64_t *)st.in(sym, C * stride * 8);
    const int32_t *n = (const int32_t *)st.in(nsym, C * 4);
    const int8_t *k = (const int8_t *)st.in(k_of_max, 23);
    int32_t *ns = (int32_t *)st.out(nsync, C * 4);
    int32_t *r = (int32_t *)st.out(rec, C * TETRA_MAX_SYNC * TETRA_F_FIELDS * 4);
    uint8_t *fb = (uint8_t *)st.out(frame_bits, C * TETRA_MAX_SYNC * 510);
    uint8_t *bb = (uint8_t *)st.out(burst_bits, C * TETRA_MAX_SYNC * 510);
    if (!s || !n || !k || !ns || !r || !fb || !bb) return st.finish();
    PROF(ctx, "compat_lmac");
    const long lw = lmac_words((long)stride) * 4;
    hipLaunchKernelGGL(k_lmac, dim3((unsigned)C), dim3(64), lw <= LMAC_LDS_MAX ? (unsigned)lw : 0u, ctx->stream, s, n,
                       (int)C, (long)stride, k, ns, r, fb, bb);
    return st.finish();
}

int tetra_symbols_to_bits(tetra_ctx *ctx, const int64_t *sym, size_t S, int64_t *bits, int64_t *mapped) {
    if (!ctx) return TETRA_E_INVALID;
    if (S == 0) return TETRA_OK;
    Staging st(ctx);
    const int64_t *s = (const int64_t *)st.in(sym, S * 8);
    int64_t *b = (int64_t *)st.out(bits, S * 16);
    int64_t *m = (int64_t *)st.out(mapped, S * 8);
    if (!s || !b || !m) return st.finish();
    hipLaunchKernelGGL(k_sym2bits, dim3(1), dim3(256), 0, ctx->stream, s, (long)S, b, m);
    return st.finish();
}

int tetra_find_sync(tetra_ctx *ctx, const uint8_t *bits, size_t nbits, int kthr, int64_t *pos, int maxpos,
                    int32_t *npos, int32_t *maxc) {
    if (!ctx || !npos || !maxc || maxpos < 0) return TETRA_E_INVALID;
    *npos = 0;
    *maxc = 0;
    if (nbits < 22) return TETRA_OK;
    Staging st(ctx);
    const uint8_t *b = (const uint8_t *)st.in(bits, nbits);
    int64_t *p = (int64_t *)st.out(pos, (size_t)(maxpos > 0 ? maxpos : 1) * 8);
    int32_t h2[2];
    int32_t *o2 = (int32_t *)st.out(h2, 8);
    if (!b || !p || !o2) return st.finish();
    hipLaunchKernelGGL(k_find_sync, dim3(1), dim3(64), 0, ctx->stream, b, (long)nbits, kthr, p, maxpos, o2);
    int rc = st.finish();
    if (rc) return rc;
    *npos = h2[0];
    *maxc = h2[1];
    return TETRA_OK;
}

int tetra_match_count(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, const uint8_t *pattern22, size_t offset,
                      int32_t *counts) {
    if (!ctx || !pattern22) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    Staging st(ctx);
    const uint8_t *b = (const uint8_t *)st.in(bits, F * L);
    const uint8_t *p = (const uint8_t *)st.in(pattern22, 22);
    int32_t *c = (int32_t *)st.out(counts, F * 4);
    if (!b || !p || !c) return st.finish();
    hipLaunchKernelGGL(k_match, dim3(grid_for(F, 64)), dim3(64), 0, ctx->stream, b, (int)F, (long)L, (long)offset, p, c);
    return st.finish();
}

int tetra_parse_bursts(tetra_ctx *ctx, const int64_t *sym, size_t F, int32_t *btype, uint8_t *crc_ok, uint8_t *bits) {
    if (!ctx) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    Staging st(ctx);
    const int64_t *s = (const int64_t *)st.in(sym, F * 255 * 8);
    int32_t *t = (int32_t *)st.out(btype, F * 4);
    uint8_t *o = (uint8_t *)st.out(crc_ok, F);
    uint8_t *b = (uint8_t *)st.out(bits, F * 510);
    if (!s || !t || !o || !b) return st.finish();
    hipLaunchKernelGGL(k_parse_bursts, dim3(grid_for(F, 64)), dim3(64), 0, ctx->stream, s, (int)F, t, o, b);
    return st.finish();
}

int tetra_crc16(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, int reversed, uint16_t *crc) {
    if (!ctx) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    Staging st(ctx);
    const uint8_t *b = (const uint8_t *)st.in(bits, F * L);
    uint16_t *c = (uint16_t *)st.out(crc, F * 2);
    if (!b || !c) return st.finish();
    hipLaunchKernelGGL(k_crc16, dim3(grid_for(F, 64)), dim3(64), 0, ctx->stream, b, (int)F, (long)L, reversed, c);
    return st.finish();
}

int tetra_check_crc(tetra_ctx *ctx, const uint8_t *bits, size_t F, size_t L, uint8_t *ok) {
    if (!ctx) return TETRA_E_INVALID;
    if (F == 0) return TETRA_OK;
    Staging st(ctx);
    const uint8_t *b = (const uint8_t *)st.in(bits, F * L);
    uint8_t *o = (uint8_t *)st.out(ok, F);
    if (!b || !o) return st.finish();
    hipLaunchKernelGGL(k_check_crc, dim3(grid_for(F, 64)), dim3(64), 0, ctx->stream, b, (int)F, (long)L, o);
    return st.finish();
}

}  // extern "C"
