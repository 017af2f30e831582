# skip_tail and skip_mfma together: timing only
import os, subprocess, sys
here = os.path.dirname(os.path.abspath(__file__))
s = sys.stdin.read()
for f in ("skip_tail.py", "skip_mfma.py"):
    s = subprocess.run([sys.executable, os.path.join(here, f)], input=s, capture_output=True, text=True, check=True).stdout
sys.stdout.write(s)
