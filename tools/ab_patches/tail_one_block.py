# timing only: the fused tail's Gardner tracking stops after its first block (the tail without its
# tracking chain); the CFO wave is released as at the channel's end
import sys
s = sys.stdin.read()
b = "        if (nv < 64) break;\n    }\n    if constexpr (SPLIT) {   // the last block's d_j, and the end"
assert s.count(b) == 1
sys.stdout.write(s.replace(b, "        if (nv < 64 || SPLIT) break;   // timing variant\n    }\n    if constexpr (SPLIT) {   // the last block's d_j, and the end"))
