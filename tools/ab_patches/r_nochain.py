# k_chanfilt_r with stage 1's chain cut to its first 10 taps (the DPP groups dropped): timing only
import sys
s = sys.stdin.read()
for p in ("1, 5>(ar, ai, xre, xim, hv + 10)", "1, 5>(ar, ai, xre + 5, xim + 5, hv + 15)", "2, 5>(ar, ai, xre, xim, hv + 20)",
          "2, 5>(ar, ai, xre + 5, xim + 5, hv + 25)", "3, 5>(ar, ai, xre, xim, hv + 30)", "3, 5>(ar, ai, xre + 5, xim + 5, hv + 35)",
          "4, 5>(ar, ai, xre, xim, hv + 40)", "4, 3>(ar, ai, xre + 5, xim + 5, hv + 45)"):
    a = "        fmac_rows<" + p + ";\n"
    assert s.count(a) == 1, p
    s = s.replace(a, "")
sys.stdout.write(s)
