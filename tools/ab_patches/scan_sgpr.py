# bit-identical candidate: k_sosb_scan reads the Phi^(2^r) table straight from global memory with a
# wave-uniform address (scalar loads, SGPR operands) instead of staging it in LDS.  Applies to
# compat_demod.hip.
import sys
s = sys.stdin.read()


def sub(a, b):
    global s
    assert s.count(a) == 1, a[:80]
    s = s.replace(a, b)


sub("""    __shared__ double ph[SB_NPOW * 64];   // the Phi^(2^r) table, read by every thread at every level
    const int k = threadIdx.x, s = blockIdx.x, ch = s >> 1, comp = s & 1;
    const bool on = k < G.Tn;
    for (int i = k; i < SB_NPOW * 64; i += blockDim.x) ph[i] = phi[i];   // visible after the first level's barrier
""", """    const int k = threadIdx.x, s = blockIdx.x, ch = s >> 1, comp = s & 1;
    const bool on = k < G.Tn;
""")
sub("""            const double *P = ph + r * 64;""", """            const double *P = phi + __builtin_amdgcn_readfirstlane(r) * 64;""")
sys.stdout.write(s)
