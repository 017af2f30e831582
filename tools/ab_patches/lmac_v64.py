# Lower-MAC trellis and traceback held to 64 VGPRs (8 waves per SIMD), so a wave of either fits
# beside two channel-filter waves (2 x 224 of a SIMD's 512 VGPRs) when the bench's pipeline runs
# them side by side.  The trellis row moves to dynamic LDS (a static 7 KB array caps the occupancy
# the compiler plans for, and with it the VGPR budget it honours); the traceback keeps four survivor
# groups in flight instead of eight.
import sys
s = sys.stdin.read()
def sub(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
sub("__global__ __launch_bounds__(64) void k_etsi_viterbi(",
    "__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_etsi_viterbi(")
sub("__global__ __launch_bounds__(64) void k_etsi_traceback(",
    "__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_etsi_traceback(")
sub("    __shared__ __attribute__((aligned(16))) int8_t rows[16 * VROW];",
    "    extern __shared__ __attribute__((aligned(16))) int8_t rows[];   // 16 * VROW")
sub("hipLaunchKernelGGL(k_etsi_viterbi, vgrid(4), dim3(64), 0,", "hipLaunchKernelGGL(k_etsi_viterbi, vgrid(4), dim3(64), 16 * VROW,")
sub("hipLaunchKernelGGL(k_etsi_viterbi, vgrid(mask), dim3(64), 0,", "hipLaunchKernelGGL(k_etsi_viterbi, vgrid(mask), dim3(64), 16 * VROW,")
sub("    for (int g0 = NG - 1; g0 >= 0; g0 -= 8) {\n        uint4 w[8];\n#pragma unroll\n        for (int u = 0; u < 8; ++u) w[u]",
    "    for (int g0 = NG - 1; g0 >= 0; g0 -= 4) {\n        uint4 w[4];\n#pragma unroll\n        for (int u = 0; u < 4; ++u) w[u]")
sub("#pragma unroll\n        for (int u = 0; u < 8; ++u) {\n            const int gi = g0 - u;",
    "#pragma unroll\n        for (int u = 0; u < 4; ++u) {\n            const int gi = g0 - u;")
sys.stdout.write(s)
