# timing only: compat_fwd_nostore + compat_noload together (the banked passes' recursion alone)
import subprocess, sys, os
d = os.path.dirname(os.path.abspath(__file__))
s = sys.stdin.read()
for p in ("compat_fwd_nostore.py", "compat_noload.py"):
    s = subprocess.run([sys.executable, os.path.join(d, p)], input=s, capture_output=True, text=True, check=True).stdout
sys.stdout.write(s)
