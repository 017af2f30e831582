# sym_direct.py with the tracking loop's symbol stores written through (sc1 buffer stores, as
# copy_out writes), so their lines do not sit dirty in L2 and get evicted into the read stream.
import sys
s = sys.stdin.read()
def sub(a, b):
    global s
    assert s.count(a) == 1, (a, s.count(a))
    s = s.replace(a, b)
sub("const TrackOut o = timing_track<true>(ly, M2, to.gain, to.soft_scale, stage ? stage->sym : to.sym + so, scr,",
    "const TrackOut o = timing_track<true>(ly, M2, to.gain, to.soft_scale, to.sym + so, scr,")
sub("    copy_out(reinterpret_cast<uint8_t *>(to.sym + so), reinterpret_cast<const uint8_t *>(stage->sym), 8 * o.S, tid);\n", "")
sub("            sp[S + lane] = on;\n", """            if constexpr (SPLIT) {
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(sp, 0, 0x7fffffff, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(on.x), __float_as_uint(on.y)}, r, 8 * (S + lane), 0, 16);
            } else {
                sp[S + lane] = on;
            }
""")
sys.stdout.write(s)
