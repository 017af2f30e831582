# the per-wave demod with stage 1's 48-tap chain cut to its first group (image stores and the rest kept): timing only
import sys
s = sys.stdin.read()
a = """            rd(ta, xa, 0);
            rd(tb, xb, 1);
            __builtin_amdgcn_sched_barrier(0);
            fm(ta, xa);
            __builtin_amdgcn_sched_barrier(0);
            rd(ta, xa, 2);
            __builtin_amdgcn_sched_barrier(0);
            fm(tb, xb);
            __builtin_amdgcn_sched_barrier(0);
            fm(ta, xa);
            lin[k - kbase] = make_float2(a.x, a.y);
            if (wv > 0"""
assert a in s
sys.stdout.write(s.replace(a, """            rd(ta, xa, 0);
            fm(ta, xa);
            lin[k - kbase] = make_float2(a.x, a.y);
            if (wv > 0"""))
