# the fused tail's Gardner tracking stops after its first block, the CFO wave released as at the
# channel's end (timing only)
import sys
s = sys.stdin.read()
a = "__hip_atomic_store(prog, S | (nv < 64 ? PROG_DONE : 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);"
assert s.count(a) == 1
s = s.replace(a, "__hip_atomic_store(prog, S | PROG_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);")
b = "        if (nv < 64) break;\n    }\n    o.S = S;"
assert s.count(b) == 1
sys.stdout.write(s.replace(b, "        if (nv < 64 || SPLIT) break;   // timing variant\n    }\n    o.S = S;"))
