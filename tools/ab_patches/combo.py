# several variant patches applied in order: COMBO="l2_input,skip_stage1" (timing only)
import os
import subprocess
import sys
d = os.path.dirname(os.path.abspath(__file__))
s = sys.stdin.read()
for v in os.environ["COMBO"].split(","):
    s = subprocess.run([sys.executable, os.path.join(d, v + ".py")], input=s, capture_output=True, text=True,
                       check=True).stdout
sys.stdout.write(s)
